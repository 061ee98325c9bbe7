// stream.hip — vocab-wide log-softmax + target gather (cs_logsoftmax_gather).
#include "cs_kernels.cuh"

namespace {

// Work items (row, split) are walked grid-stride so a capped grid also works.
template <int DT, bool CAP, bool FIXED, int BLOCK, int UNROLL>
__global__ __launch_bounds__(BLOCK, BLOCK >= 1024 ? 8 : 1) void lsg_stream_kernel(
    const char* __restrict__ logits, int64_t n_items, int64_t vocab, int64_t ld_bytes,
    int32_t nsplit, int64_t split_len, const int32_t* __restrict__ tgt, int32_t k, float cap,
    float inv_cap, float* __restrict__ out_tok, float* __restrict__ out_lse,
    float2* __restrict__ part) {
  __shared__ float sm_m[BLOCK / 64];
  __shared__ float sm_s[BLOCK / 64];
  __shared__ float sm_lse;
  constexpr bool TAB = CapTable<DT, CAP, FIXED>::kOn;
  __shared__ float ctab[TAB ? kCapTab : 1];
  const int tid = threadIdx.x;
  if constexpr (TAB) {
    build_cap_table<BLOCK>(ctab, cap, inv_cap);
    __syncthreads();
  }

  for (int64_t bid = blockIdx.x; bid < n_items; bid += gridDim.x) {
    const int64_t row = bid / nsplit;
    const int32_t split = static_cast<int32_t>(bid - row * nsplit);
    const char* rp = logits + row * ld_bytes;
    const int64_t v0 = static_cast<int64_t>(split) * split_len;
    const int64_t v1 = min(vocab, v0 + split_len);
    const float2 ms =
        block_lse_partial<DT, CAP, FIXED, BLOCK, UNROLL>(rp, v0, v1 - v0, cap, inv_cap, sm_m, sm_s,
                                                         ctab);
    if (tid == 0) {
      if (nsplit > 1) {
        part[bid] = ms;
      } else {
        const float lse = ms.x + logf(ms.y);
        sm_lse = lse;
        if (out_lse) out_lse[row] = lse;
      }
    }
    __syncthreads();
    if (nsplit == 1 && k > 0)
      gather_targets(rp, vocab, sm_lse, tgt + row * k, k, out_tok + row * k, CAP, cap, inv_cap,
                     DT, tid, BLOCK);
    __syncthreads();  // sm_* are reused by the next work item
  }
}

// Split rows in the canonical split arithmetic (split_partial, cs_kernels.cuh): BLOCK / 256
// splits per workgroup, each split's (m, s) to part[row * nsplit + split] for lsg_merge_kernel.
template <int DT, bool CAP, bool FIXED, int BLOCK>
__global__ __launch_bounds__(BLOCK, BLOCK >= 1024 ? 8 : 1) void lsg_split_kernel(
    const char* __restrict__ logits, int64_t n_items, int64_t vocab, int64_t ld_bytes,
    int32_t nsplit, int64_t split_len, float cap, float inv_cap, float2* __restrict__ part) {
  __shared__ float sm_m[BLOCK / 64];
  __shared__ float sm_s[BLOCK / 64];
  constexpr bool TAB = CapTable<DT, CAP, FIXED>::kOn;
  __shared__ float ctab[TAB ? kCapTab : 1];
  if constexpr (TAB) {
    build_cap_table<BLOCK>(ctab, cap, inv_cap);
    __syncthreads();
  }
  const int32_t per_row = split_items(nsplit, BLOCK);
  for (int64_t bid = blockIdx.x; bid < n_items; bid += gridDim.x) {
    const int64_t row = bid / per_row;
    const int32_t item = static_cast<int32_t>(bid - row * per_row);
    int32_t split;
    bool valid;
    const float2 ms = split_partial<DT, CAP, FIXED, BLOCK>(logits + row * ld_bytes, item, nsplit,
                                                          split_len, vocab, cap, inv_cap, sm_m,
                                                          sm_s, ctab, split, valid);
    if (valid && threadIdx.x % kSplitSub == 0) part[row * nsplit + split] = ms;
    __syncthreads();  // sm_* are reused by the next work item
  }
}

// split-V finish: merge the (m, s) partials of one row in split order, then gather.
template <int DT, bool CAP>
__global__ __launch_bounds__(kMergeBlock) void lsg_merge_kernel(
    const char* __restrict__ logits, int64_t vocab, int64_t ld_bytes, int32_t nsplit,
    const float2* __restrict__ part, const int32_t* __restrict__ tgt, int32_t k, float cap,
    float inv_cap, float* __restrict__ out_tok, float* __restrict__ out_lse) {
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x;
  float m = -INFINITY, s = 0.0f;
  for (int j = lane; j < nsplit; j += kMergeBlock) {
    const float2 p = part[row * nsplit + j];
    lse_merge(m, s, p.x, p.y);
  }
  wave_lse_reduce(m, s);
  const float lse = m + logf(s);
  if (lane == 0 && out_lse) out_lse[row] = lse;
  if (k > 0)
    gather_targets(logits + row * ld_bytes, vocab, lse, tgt + row * k, k, out_tok + row * k, CAP,
                   cap, inv_cap, DT, lane, kMergeBlock);
}

// Streaming-kernel configurations compiled into the library.  Variant 0 (default) is
// shape-aware, from the in-process A/B on the bench's data (profiles/r01_lsg_variants.jsonl):
//   single pass (rows >= 2048): 1024 threads x 2 vectors in flight  (C2: 7.25 TB/s, 90.6 %)
//   split-V (fewer rows):        the canonical split arithmetic (split_partial, cs_kernels.cuh):
//                                256-thread sub-blocks x 2 vectors, 4 splits per 1024 threads
// CS_LSG_VARIANT=<n> (host environment, read per launch) forces one configuration for
// A/B timing (tools/lsg_variants.py).  All variants compute the same values up to the
// order of the fp32 partial merges inside a row (|diff| ~ 1e-6).
template <int DT, bool CAP, int BLOCK, int UNROLL>
void launch_stream(const void* logits, int64_t items, int64_t vocab, int64_t ld_bytes,
                   const SplitPlan& plan, const int32_t* tgt, int32_t k, float cap, float inv_cap,
                   float* out_tok, float* out_lse, float2* part, hipStream_t st) {
  const char* lg = static_cast<const char*>(logits);
  if constexpr (CAP) {
    if (fixed_lse_ok(cap)) {
      hipLaunchKernelGGL((lsg_stream_kernel<DT, CAP, true, BLOCK, UNROLL>),
                         dim3(static_cast<uint32_t>(items)), dim3(BLOCK), 0, st, lg, items, vocab,
                         ld_bytes, plan.nsplit, plan.split_len, tgt, k, cap, inv_cap, out_tok,
                         out_lse, part);
      return;
    }
  }
  hipLaunchKernelGGL((lsg_stream_kernel<DT, CAP, false, BLOCK, UNROLL>),
                       dim3(static_cast<uint32_t>(items)), dim3(BLOCK), 0, st, lg, items, vocab,
                       ld_bytes, plan.nsplit, plan.split_len, tgt, k, cap, inv_cap, out_tok,
                       out_lse, part);
}

int lsg_variant() {
  static const int v = [] {            // A/B knob (tools/lsg_variants.py), read once
    const char* e = getenv("CS_LSG_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

template <int DT, bool CAP>
void launch_lsg(const void* logits, int64_t rows, int64_t vocab, int64_t ld_bytes,
                const SplitPlan& plan, const int32_t* tgt, int32_t k, float cap, float* out_tok,
                float* out_lse, float2* part, hipStream_t st, bool finish = true) {
  const float inv_cap = CAP ? 1.0f / cap : 0.0f;
  const int64_t items = rows * plan.nsplit;
  switch (lsg_variant()) {
    case 1:  // 512 x 4
      launch_stream<DT, CAP, 512, 4>(logits, items, vocab, ld_bytes, plan, tgt, k, cap, inv_cap,
                                     out_tok, out_lse, part, st);
      break;
    case 2:
      launch_stream<DT, CAP, 1024, 1>(logits, items, vocab, ld_bytes, plan, tgt, k, cap, inv_cap,
                                      out_tok, out_lse, part, st);
      break;
    case 3:
      launch_stream<DT, CAP, 1024, 2>(logits, items, vocab, ld_bytes, plan, tgt, k, cap, inv_cap,
                                      out_tok, out_lse, part, st);
      break;
    case 4:
      launch_stream<DT, CAP, 256, 8>(logits, items, vocab, ld_bytes, plan, tgt, k, cap, inv_cap,
                                     out_tok, out_lse, part, st);
      break;
    case 5:
      launch_stream<DT, CAP, kBlock, kUnroll>(logits, items, vocab, ld_bytes, plan, tgt, k, cap,
                                              inv_cap, out_tok, out_lse, part, st);
      break;
    case 6:
      launch_stream<DT, CAP, 1024, 4>(logits, items, vocab, ld_bytes, plan, tgt, k, cap, inv_cap,
                                      out_tok, out_lse, part, st);
      break;
    case 7:
      launch_stream<DT, CAP, 512, 8>(logits, items, vocab, ld_bytes, plan, tgt, k, cap, inv_cap,
                                     out_tok, out_lse, part, st);
      break;
    default:
      if (plan.nsplit == 1) {
        launch_stream<DT, CAP, 1024, 2>(logits, items, vocab, ld_bytes, plan, tgt, k, cap,
                                        inv_cap, out_tok, out_lse, part, st);
      } else {
        // the canonical split arithmetic, four splits per 1024-thread workgroup
        const int64_t n_items = rows * split_items(plan.nsplit, 1024);
        const char* lg = static_cast<const char*>(logits);
        bool done = false;
        if constexpr (CAP) {
          if (fixed_lse_ok(cap)) {
            hipLaunchKernelGGL((lsg_split_kernel<DT, CAP, true, 1024>),
                               dim3(static_cast<uint32_t>(n_items)), dim3(1024), 0, st, lg, n_items,
                               vocab, ld_bytes, plan.nsplit, plan.split_len, cap, inv_cap, part);
            done = true;
          }
        }
        if (!done)
          hipLaunchKernelGGL((lsg_split_kernel<DT, CAP, false, 1024>),
                             dim3(static_cast<uint32_t>(n_items)), dim3(1024), 0, st, lg, n_items,
                             vocab, ld_bytes, plan.nsplit, plan.split_len, cap, inv_cap, part);
      }
      break;
  }
  if (plan.nsplit > 1 && finish) {
    hipLaunchKernelGGL((lsg_merge_kernel<DT, CAP>), dim3(static_cast<uint32_t>(rows)),
                       dim3(kMergeBlock), 0, st, static_cast<const char*>(logits), vocab, ld_bytes,
                       plan.nsplit, part, tgt, k, cap, inv_cap, out_tok, out_lse);
  }
}

}  // namespace

extern "C" {

const char* cs_version(void) { return "consensus_scoring 0.1.0 (gfx950)"; }

const char* cs_last_error(void) { return cs_g_last_error.c_str(); }

size_t cs_workspace_size(int64_t rows, int64_t vocab, int32_t k) {
  (void)k;
  const SplitPlan p = plan_split(rows, vocab, CS_BF16);
  const SplitPlan q = plan_split(rows, vocab, CS_F32);
  const int32_t ns = p.nsplit > q.nsplit ? p.nsplit : q.nsplit;
  if (ns <= 1) return 0;
  return static_cast<size_t>(rows) * static_cast<size_t>(ns) * sizeof(float2);
}

int cs_logsoftmax_gather(const void* logits, int dtype, int64_t rows, int64_t vocab, int64_t ld,
                         const int32_t* target_ids, int32_t k, float softcap, float* out_tok_lp,
                         float* out_row_lse, void* workspace, size_t workspace_bytes,
                         cs_stream_t stream) {
  if (dtype != CS_F32 && dtype != CS_BF16 && dtype != CS_F16)
    return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: unknown dtype");
  if (rows < 0 || vocab <= 0 || ld < vocab || k < 0)
    return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: need rows >= 0, vocab > 0, ld >= vocab, k >= 0");
  if (rows > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: rows exceeds 2^31-1");
  if (rows == 0) return CS_OK;
  if (!logits) return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: logits is NULL");
  if (k > 0 && (!target_ids || !out_tok_lp))
    return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: k > 0 needs target_ids and out_tok_lp");
  if (!(softcap >= 0.0f) || std::isinf(softcap))
    return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: softcap must be finite and >= 0");
  if (reinterpret_cast<uintptr_t>(logits) % elt_size(dtype) != 0)
    return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: logits not element-aligned");
  const SplitPlan plan = plan_split(rows, vocab, dtype);
  const int64_t grid = rows * plan.nsplit;
  if (grid > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_logsoftmax_gather: grid too large");
  float2* part = nullptr;
  if (plan.nsplit > 1) {
    const size_t need = static_cast<size_t>(rows) * plan.nsplit * sizeof(float2);
    if (!workspace || workspace_bytes < need)
      return fail(CS_ERR_WORKSPACE, "cs_logsoftmax_gather: workspace smaller than cs_workspace_size()");
    if (reinterpret_cast<uintptr_t>(workspace) % 8 != 0)
      return fail(CS_ERR_WORKSPACE, "cs_logsoftmax_gather: workspace not 8-byte aligned");
    part = static_cast<float2*>(workspace);
  }
  const int64_t ld_bytes = ld * elt_size(dtype);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool cap = softcap > 0.0f;
  switch (dtype) {
    case CS_F32:
      if (cap)
        launch_lsg<CS_F32, true>(logits, rows, vocab, ld_bytes, plan, target_ids, k, softcap,
                                 out_tok_lp, out_row_lse, part, st);
      else
        launch_lsg<CS_F32, false>(logits, rows, vocab, ld_bytes, plan, target_ids, k, softcap,
                                  out_tok_lp, out_row_lse, part, st);
      break;
    case CS_BF16:
      if (cap)
        launch_lsg<CS_BF16, true>(logits, rows, vocab, ld_bytes, plan, target_ids, k, softcap,
                                  out_tok_lp, out_row_lse, part, st);
      else
        launch_lsg<CS_BF16, false>(logits, rows, vocab, ld_bytes, plan, target_ids, k, softcap,
                                   out_tok_lp, out_row_lse, part, st);
      break;
    default:
      if (cap)
        launch_lsg<CS_F16, true>(logits, rows, vocab, ld_bytes, plan, target_ids, k, softcap,
                                 out_tok_lp, out_row_lse, part, st);
      else
        launch_lsg<CS_F16, false>(logits, rows, vocab, ld_bytes, plan, target_ids, k, softcap,
                                  out_tok_lp, out_row_lse, part, st);
      break;
  }
  return check_launch("cs_logsoftmax_gather");
}

}  // extern "C"
