// fold.hip — segment folds, welfare over agents, stable top-k.
#include "cs_kernels.cuh"

namespace {

// ---------------------------------------------------------------------------
// per-candidate folding
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void seg_reduce_kernel(const float* __restrict__ lp,
                                                         const int32_t* __restrict__ off,
                                                         int64_t n_seg, float* __restrict__ sum_lp,
                                                         float* __restrict__ sum_p,
                                                         int32_t* __restrict__ cnt,
                                                         float* __restrict__ last) {
  const int64_t seg = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (seg >= n_seg) return;  // wave-uniform
  const int64_t b = off[seg], e = off[seg + 1];
  double a = 0.0, p = 0.0;
  int c = 0;
  for (int64_t i = b + lane; i < e; i += 64) {
    const float v = lp[i];
    if (!__builtin_isnan(v)) {
      a += static_cast<double>(v);
      p += exp(static_cast<double>(v));
      c += 1;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    p += __shfl_xor(p, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  if (lane == 0) {
    if (sum_lp) sum_lp[seg] = static_cast<float>(a);
    if (sum_p) sum_p[seg] = static_cast<float>(p);
    if (cnt) cnt[seg] = c;
    if (last) last[seg] = (e > b) ? lp[e - 1] : __builtin_nanf("");
  }
}

__global__ __launch_bounds__(256) void welfare_kernel(const float* __restrict__ U, int32_t A,
                                                      int32_t C, int64_t ldu, int kind, double eps,
                                                      int nonfinite, float nan_val,
                                                      float posinf_val, float neginf_val,
                                                      float* __restrict__ W) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (c >= C) return;
  double acc = 0.0;
  bool any = false;
  for (int32_t a = 0; a < A; ++a) {
    float u = U[a * ldu + c];
    if (!__builtin_isfinite(u)) {
      if (nonfinite == CS_NONFINITE_SKIP) continue;
      u = __builtin_isnan(u) ? nan_val : (u > 0.0f ? posinf_val : neginf_val);
    }
    const double d = static_cast<double>(u);
    switch (kind) {
      case CS_WELFARE_MIN:
        acc = any ? fmin(acc, d) : d;
        break;
      case CS_WELFARE_MAX:
        acc = any ? fmax(acc, d) : d;
        break;
      case CS_WELFARE_SUM:
        acc += d;
        break;
      default:  // CS_WELFARE_SUMLOG
        acc += log(fmax(d, eps));
        break;
    }
    any = true;
  }
  W[c] = any ? static_cast<float>(acc) : __builtin_nanf("");
}

// ---------------------------------------------------------------------------
// stable top-k by selection (k <= kTopkSelectMax): one 256-thread workgroup per segment,
// radix select over the (order key, ~index) composite keys read straight from W (one
// coalesced pass per digit, no key array), the <= k + 64 survivors ranked by counting.
// The keys are distinct, so the result is exactly the full sort's first k (value desc,
// index asc, NaN last) — what topk_kernel's LDS bitonic gives, without its log^2(n)
// barrier stages (55 for 1,024 slots).
// ---------------------------------------------------------------------------
constexpr int kTopkSelectMax = 256;

__global__ __launch_bounds__(256) void topk_select_kernel(const float* __restrict__ W,
                                                          int32_t seg_len, int64_t ld, int32_t k,
                                                          int32_t* __restrict__ out_idx,
                                                          float* __restrict__ out_val) {
  __shared__ uint32_t hist[kTopkBins];
  __shared__ unsigned long long cand[kTopkCand];
  __shared__ uint32_t sm_w[256 / 64];
  __shared__ int sm_res[2];
  __shared__ uint32_t sm_n;
  const int64_t seg = blockIdx.x;
  const float* base = W + seg * ld;
  const int tid = threadIdx.x;
  auto key = [&](int i) -> unsigned long long {
    return (static_cast<unsigned long long>(order_key(base[i])) << 32) |
           static_cast<unsigned long long>(0xffffffffu - static_cast<uint32_t>(i));
  };
  auto each = [&](auto f) {
    for (int i = tid; i < seg_len; i += 256) f(key(i));
  };
  if (tid == 0) sm_n = 0u;
  // the last digit (shift 4) leaves at most k + 15 candidates: the 64-bit keys are distinct
  const RadixCut cut = radix_select<256>(each, static_cast<uint32_t>(k),
                                         static_cast<uint32_t>(k + 64), hist, sm_w, sm_res);
  each([&](unsigned long long c) {
    if ((c >> cut.shift) >= cut.prefix) {
      const uint32_t at = atomicAdd(&sm_n, 1u);
      if (at < kTopkCand) cand[at] = c;
    }
  });
  __syncthreads();
  const int nc = static_cast<int>(min(sm_n, static_cast<uint32_t>(kTopkCand)));
  rank_candidates<256>(cand, nc, k, [&](int r, unsigned long long c) {
    const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(c & 0xffffffffull);
    out_idx[seg * k + r] = static_cast<int32_t>(idx);
    if (out_val) out_val[seg * k + r] = base[idx];
  });
}

}  // namespace

extern "C" {

int cs_segment_reduce(const float* tok_lp, int64_t n, const int32_t* seg_offsets, int64_t n_seg,
                      float* out_sum_lp, float* out_sum_p, int32_t* out_count, float* out_last,
                      cs_stream_t stream) {
  if (n < 0 || n_seg < 0) return fail(CS_ERR_INVALID, "cs_segment_reduce: negative size");
  if (n_seg == 0) return CS_OK;
  if (!seg_offsets || (n > 0 && !tok_lp))
    return fail(CS_ERR_INVALID, "cs_segment_reduce: NULL input");
  const int64_t blocks = (n_seg + 3) / 4;
  if (blocks > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_segment_reduce: too many segments");
  hipLaunchKernelGGL(seg_reduce_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), tok_lp, seg_offsets, n_seg, out_sum_lp,
                     out_sum_p, out_count, out_last);
  return check_launch("cs_segment_reduce");
}

int cs_welfare_reduce(const float* U, int32_t A, int32_t C, int64_t ldu, int kind, float eps,
                      int nonfinite, float nan_val, float posinf_val, float neginf_val, float* W,
                      cs_stream_t stream) {
  if (A < 0 || C < 0 || ldu < C) return fail(CS_ERR_INVALID, "cs_welfare_reduce: bad shape");
  if (kind < CS_WELFARE_MIN || kind > CS_WELFARE_MAX)
    return fail(CS_ERR_INVALID, "cs_welfare_reduce: unknown welfare kind");
  if (nonfinite != CS_NONFINITE_SKIP && nonfinite != CS_NONFINITE_REPLACE)
    return fail(CS_ERR_INVALID, "cs_welfare_reduce: unknown nonfinite mode");
  if (C == 0) return CS_OK;
  if (!W || (A > 0 && !U)) return fail(CS_ERR_INVALID, "cs_welfare_reduce: NULL pointer");
  const int64_t blocks = (static_cast<int64_t>(C) + 255) / 256;
  hipLaunchKernelGGL(welfare_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), U, A, C, ldu, kind,
                     static_cast<double>(eps), nonfinite, nan_val, posinf_val, neginf_val, W);
  return check_launch("cs_welfare_reduce");
}

int cs_segmented_topk(const float* W, int32_t n_seg, int32_t seg_len, int64_t ld, int32_t k,
                      int32_t* out_idx, float* out_val, cs_stream_t stream) {
  if (n_seg < 0 || seg_len < 0 || k < 0 || ld < seg_len)
    return fail(CS_ERR_INVALID, "cs_segmented_topk: bad shape");
  if (seg_len > 16384) return fail(CS_ERR_INVALID, "cs_segmented_topk: seg_len > 16384");
  if (k > seg_len) return fail(CS_ERR_INVALID, "cs_segmented_topk: k > seg_len");
  if (n_seg == 0 || k == 0) return CS_OK;
  if (!W || !out_idx) return fail(CS_ERR_INVALID, "cs_segmented_topk: NULL pointer");
  if (k <= kTopkSelectMax && seg_len > 64) {
    hipLaunchKernelGGL(topk_select_kernel, dim3(static_cast<uint32_t>(n_seg)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), W, seg_len, ld, k, out_idx, out_val);
    return check_launch("cs_segmented_topk");
  }
  int32_t n2 = 2;
  while (n2 < seg_len) n2 <<= 1;
  hipLaunchKernelGGL(topk_kernel, dim3(static_cast<uint32_t>(n_seg)), dim3(256),
                     static_cast<size_t>(n2) * sizeof(unsigned long long),
                     static_cast<hipStream_t>(stream), W, seg_len, ld, n2, k, out_idx, out_val);
  return check_launch("cs_segmented_topk");
}


// workspace: [done counter | pad to 64 B][row counters: kBeamMaxRows u32][row partials
// rows*nsplit x 8 B].  The counters sit at fixed offsets whatever the shape, so calls of
// different shapes can share one workspace: every call leaves them at zero.

}  // extern "C"
