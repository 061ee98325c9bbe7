// proposer.hip — candidate proposers: vocab top-k and seeded sampling.
#include "cs_kernels.cuh"

namespace {

// One (row, 4096-element chunk) per workgroup: the chunk's k largest composite keys
// (order key, ~token id), descending, zero-padded when the chunk holds fewer than k.
template <int DT, bool CAP>
__global__ __launch_bounds__(256) void vocab_topk_chunk_kernel(
    const char* __restrict__ logits, int64_t vocab, int64_t ld_bytes, int32_t nchunk, int32_t k,
    float cap, float inv_cap, unsigned long long* __restrict__ part) {
  // 32 KB: histogram (16 KB) + candidates (8 KB), or the whole chunk for the fallback sort
  __shared__ __attribute__((aligned(16))) unsigned long long lds[kTopkChunk];
  __shared__ uint32_t sm_w[4];
  __shared__ int sm_res[2];
  __shared__ uint32_t sm_n;
  uint32_t* hist = reinterpret_cast<uint32_t*>(lds);
  unsigned long long* cand = lds + kTopkBins / 2;
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x / nchunk;
  const int32_t chunk = static_cast<int32_t>(blockIdx.x - row * nchunk);
  const char* rp = logits + row * ld_bytes;
  const int64_t v0 = static_cast<int64_t>(chunk) * kTopkChunk;
  const int n = static_cast<int>(min(static_cast<int64_t>(kTopkChunk), vocab - v0));
#ifdef CS_TRACE_TOPK
  const unsigned long long q0 = wall_clock64();
#endif
  unsigned long long key[kTopkPer];
#pragma unroll
  for (int j = 0; j < kTopkPer; ++j) {
    const int i = tid + 256 * j;
    float x = 0.0f;
    if (i < n) x = load_any<DT>(rp, v0 + i);
    key[j] = 0ull;
    if (i < n) {
      if (CAP) x = softcap_fn(x, cap, inv_cap);
      key[j] = (static_cast<unsigned long long>(order_key(x)) << 32) |
               static_cast<unsigned long long>(0xffffffffu - static_cast<uint32_t>(v0 + i));
    }
  }
  if (tid == 0) sm_n = 0u;
#ifdef CS_TRACE_TOPK
  __syncthreads();
  const unsigned long long q1 = wall_clock64();
#endif
  const RadixCut cut = radix_select<256>(
      [&](auto f) {
#pragma unroll
        for (int j = 0; j < kTopkPer; ++j)
          if (key[j]) f(key[j]);
      },
      static_cast<uint32_t>(k), static_cast<uint32_t>(2 * k + 64), hist, sm_w, sm_res);
#ifdef CS_TRACE_TOPK
  const unsigned long long q2 = wall_clock64();
#endif
  unsigned long long* out = part + (row * nchunk + chunk) * static_cast<int64_t>(k);
  if (cut.count <= kTopkCand) {  // block-uniform (always, unless > 1024 keys tie exactly)
#pragma unroll
    for (int j = 0; j < kTopkPer; ++j)
      if (key[j] && (key[j] >> cut.shift) >= cut.prefix) cand[atomicAdd(&sm_n, 1u)] = key[j];
    __syncthreads();
    const int nc = static_cast<int>(sm_n);
    rank_candidates(cand, nc, k, [&](int r, unsigned long long kc) { out[r] = kc; });
    for (int r = nc + tid; r < k; r += 256) out[r] = 0ull;
#ifdef CS_TRACE_TOPK
    __syncthreads();
    if (tid == 0 && blockIdx.x % 97 == 0)
      printf("TOPK chunk %d load %llu select %llu rank %llu nc %d levels %d (x10ns)\n", (int)blockIdx.x,
             q1 - q0, q2 - q1, wall_clock64() - q2, nc, (52 - cut.shift) / 12 + 1);
#endif
    return;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kTopkPer; ++j) lds[tid + 256 * j] = key[j];
  __syncthreads();
  bitonic_desc(lds, kTopkChunk, tid, 256);
  for (int r = tid; r < k; r += 256) out[r] = lds[r];
}

__device__ __forceinline__ void emit_token(int32_t* ids, float* vals, int64_t at,
                                           unsigned long long c) {
  ids[at] = static_cast<int32_t>(0xffffffffu - static_cast<uint32_t>(c & 0xffffffffull));
  if (vals) vals[at] = key_to_float(static_cast<uint32_t>(c >> 32));
}

// One row per workgroup: the k largest of the row's nkeys chunk winners (zero = padding).
// Dynamic LDS: max(n2, 4096) keys (histogram + candidates, or the fallback sort).
__global__ __launch_bounds__(256) void vocab_topk_merge_kernel(
    const unsigned long long* __restrict__ part, int32_t nkeys, int32_t n2, int32_t k,
    int32_t* __restrict__ out_ids, float* __restrict__ out_vals) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long mk[];
  __shared__ uint32_t sm_w[4];
  __shared__ int sm_res[2];
  __shared__ uint32_t sm_n;
  uint32_t* hist = reinterpret_cast<uint32_t*>(mk);
  unsigned long long* cand = mk + kTopkBins / 2;
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  const unsigned long long* pr = part + row * nkeys;
  if (tid == 0) sm_n = 0u;
  const RadixCut cut = radix_select<256>(
      [&](auto f) {
        for (int i = tid; i < nkeys; i += 256) {
          const unsigned long long c = pr[i];
          if (c) f(c);
        }
      },
      static_cast<uint32_t>(k), static_cast<uint32_t>(2 * k + 64), hist, sm_w, sm_res);
  if (cut.count <= kTopkCand) {  // block-uniform
    for (int i = tid; i < nkeys; i += 256) {
      const unsigned long long c = pr[i];
      if (c && (c >> cut.shift) >= cut.prefix) cand[atomicAdd(&sm_n, 1u)] = c;
    }
    __syncthreads();
    const int nc = static_cast<int>(sm_n);
    rank_candidates(cand, nc, k,
                    [&](int r, unsigned long long c) { emit_token(out_ids, out_vals, row * k + r, c); });
    for (int r = nc + tid; r < k; r += 256) emit_token(out_ids, out_vals, row * k + r, 0ull);
    return;
  }
  __syncthreads();
  for (int i = tid; i < n2; i += 256) mk[i] = (i < nkeys) ? pr[i] : 0ull;
  __syncthreads();
  bitonic_desc(mk, n2, tid, 256);
  for (int r = tid; r < k; r += 256) emit_token(out_ids, out_vals, row * k + r, mk[r]);
}

// Counter-based uniform strictly inside (0, 1): splitmix64 finaliser of (seed, token), top
// 23 bits + 0.5 (exactly representable in fp32).  oracle/oracle.py:cs_uniform restates it
// bit for bit.
__device__ __forceinline__ float cs_uniform(unsigned long long seed, unsigned long long v) {
  unsigned long long x = seed * 0x9E3779B97F4A7C15ull + (v + 1ull) * 0xD1B54A32D192ED03ull;
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (static_cast<float>(static_cast<uint32_t>(x >> 41)) + 0.5f) * (1.0f / 8388608.0f);
}

struct DrawBest {
  float s;
  int32_t idx;
};

__device__ __forceinline__ void draw_merge(float& s, int32_t& i, float s2, int32_t i2) {
  if (s2 > s || (s2 == s && i2 < i)) {
    s = s2;
    i = i2;
  }
}

template <int DT, bool CAP>
__global__ __launch_bounds__(256) void vocab_sample_kernel(
    const char* __restrict__ logits, int64_t vocab, int64_t ld_bytes, int32_t nsplit,
    int64_t split_len, float inv_temp, float cap, float inv_cap,
    const unsigned long long* __restrict__ seeds, int32_t n_draw, float2* __restrict__ lse_part,
    DrawBest* __restrict__ draw_part) {
  __shared__ float sm_m[4], sm_s[4];
  __shared__ float sm_bs[4][kMaxDraws];
  __shared__ int32_t sm_bi[4][kMaxDraws];
  const int tid = threadIdx.x;
  const int64_t bid = blockIdx.x;
  const int64_t row = bid / nsplit;
  const int32_t split = static_cast<int32_t>(bid - row * nsplit);
  const char* rp = logits + row * ld_bytes;
  const int64_t v0 = static_cast<int64_t>(split) * split_len;
  const int64_t v1 = min(vocab, v0 + split_len);
  unsigned long long sd[kMaxDraws];
  float bs[kMaxDraws];
  int32_t bi[kMaxDraws];
#pragma unroll
  for (int d = 0; d < kMaxDraws; ++d) {
    sd[d] = (d < n_draw) ? seeds[row * n_draw + d] : 0ull;
    bs[d] = -INFINITY;
    bi[d] = 0x7fffffff;
  }
  float m = -INFINITY, s = 0.0f;
  for (int64_t v = v0 + tid; v < v1; v += 256) {
    float x = load_any<DT>(rp, v);
    if (CAP) x = softcap_fn(x, cap, inv_cap);
    const float y = x * inv_temp;
    lse_accum<1>(m, s, &y);
#pragma unroll
    for (int d = 0; d < kMaxDraws; ++d) {
      if (d < n_draw) {
        const float u = cs_uniform(sd[d], static_cast<unsigned long long>(v));
        const float sc = y - logf(-logf(u));
        if (sc > bs[d]) {
          bs[d] = sc;
          bi[d] = static_cast<int32_t>(v);
        }
      }
    }
  }
  wave_lse_reduce(m, s);
#pragma unroll
  for (int d = 0; d < kMaxDraws; ++d) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float s2 = __shfl_xor(bs[d], o, 64);
      const int32_t i2 = __shfl_xor(bi[d], o, 64);
      draw_merge(bs[d], bi[d], s2, i2);
    }
  }
  const int wave = tid >> 6;
  if ((tid & 63) == 0) {
    sm_m[wave] = m;
    sm_s[wave] = s;
#pragma unroll
    for (int d = 0; d < kMaxDraws; ++d) {
      sm_bs[wave][d] = bs[d];
      sm_bi[wave][d] = bi[d];
    }
  }
  __syncthreads();
  if (tid == 0) {
    float mm = sm_m[0], ss = sm_s[0];
    for (int w = 1; w < 4; ++w) lse_merge(mm, ss, sm_m[w], sm_s[w]);
    lse_part[bid] = make_float2(mm, ss);
  }
  if (tid < n_draw) {
    float b = sm_bs[0][tid];
    int32_t i = sm_bi[0][tid];
    for (int w = 1; w < 4; ++w) draw_merge(b, i, sm_bs[w][tid], sm_bi[w][tid]);
    draw_part[bid * n_draw + tid] = DrawBest{b, i};
  }
}

template <int DT, bool CAP>
__global__ __launch_bounds__(64) void vocab_sample_merge_kernel(
    const char* __restrict__ logits, int64_t ld_bytes, int32_t nsplit, float inv_temp, float cap,
    float inv_cap, const float2* __restrict__ lse_part, const DrawBest* __restrict__ draw_part,
    int32_t n_draw, int32_t* __restrict__ out_ids, float* __restrict__ out_lp) {
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x;
  float m = -INFINITY, s = 0.0f;
  for (int j = lane; j < nsplit; j += 64) {
    const float2 p = lse_part[row * nsplit + j];
    lse_merge(m, s, p.x, p.y);
  }
  wave_lse_reduce(m, s);
  const float lse = m + logf(s);
  for (int d = lane; d < n_draw; d += 64) {
    float b = -INFINITY;
    int32_t i = 0x7fffffff;
    for (int j = 0; j < nsplit; ++j) {  // split order: ties keep the lower token id
      const DrawBest p = draw_part[(row * nsplit + j) * n_draw + d];
      draw_merge(b, i, p.s, p.idx);
    }
    out_ids[row * n_draw + d] = i;
    if (out_lp) {
      float x = load_any<DT>(logits + row * ld_bytes, i);
      if (CAP) x = softcap_fn(x, cap, inv_cap);
      out_lp[row * n_draw + d] = x * inv_temp - lse;
    }
  }
}

int32_t topk_nchunk(int64_t vocab) {
  return static_cast<int32_t>((vocab + kTopkChunk - 1) / kTopkChunk);
}

}  // namespace

extern "C" {

size_t cs_vocab_topk_workspace_size(int64_t rows, int64_t vocab, int32_t k) {
  if (rows <= 0 || vocab <= 0 || k <= 0) return 0;
  return static_cast<size_t>(rows) * topk_nchunk(vocab) * static_cast<size_t>(k) *
         sizeof(unsigned long long);
}

int cs_vocab_topk(const void* logits, int dtype, int64_t rows, int64_t vocab, int64_t ld, int32_t k,
                  float softcap, int32_t* out_ids, float* out_vals, void* workspace,
                  size_t workspace_bytes, cs_stream_t stream) {
  if (dtype != CS_F32 && dtype != CS_BF16 && dtype != CS_F16)
    return fail(CS_ERR_INVALID, "cs_vocab_topk: unknown dtype");
  if (rows < 0 || vocab <= 0 || ld < vocab || k <= 0 || k > 256 || k > vocab)
    return fail(CS_ERR_INVALID, "cs_vocab_topk: need rows >= 0, vocab > 0, ld >= vocab, 0 < k <= min(256, vocab)");
  if (!(softcap >= 0.0f) || std::isinf(softcap))
    return fail(CS_ERR_INVALID, "cs_vocab_topk: softcap must be finite and >= 0");
  if (rows == 0) return CS_OK;
  if (!logits || !out_ids) return fail(CS_ERR_INVALID, "cs_vocab_topk: NULL pointer");
  const int32_t nchunk = topk_nchunk(vocab);
  const int64_t nkeys = static_cast<int64_t>(nchunk) * (k < kTopkChunk ? k : kTopkChunk);
  if (nkeys > 16384) return fail(CS_ERR_INVALID, "cs_vocab_topk: vocab chunks x k exceeds 16384");
  if (rows * nchunk > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_vocab_topk: grid too large");
  const size_t need = cs_vocab_topk_workspace_size(rows, vocab, k);
  if (!workspace || workspace_bytes < need)
    return fail(CS_ERR_WORKSPACE, "cs_vocab_topk: workspace smaller than cs_vocab_topk_workspace_size()");
  auto* part = static_cast<unsigned long long*>(workspace);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t ld_bytes = ld * elt_size(dtype);
  const float inv_cap = softcap > 0.0f ? 1.0f / softcap : 0.0f;
  const dim3 g1(static_cast<uint32_t>(rows * nchunk));
  const char* lg = static_cast<const char*>(logits);
#define CS_TOPK_LAUNCH(DTV, CAPV)                                                               \
  hipLaunchKernelGGL((vocab_topk_chunk_kernel<DTV, CAPV>), g1, dim3(256), 0, st, lg, vocab,    \
                     ld_bytes, nchunk, k, softcap, inv_cap, part)
  const bool cap = softcap > 0.0f;
  if (dtype == CS_F32) { if (cap) CS_TOPK_LAUNCH(CS_F32, true); else CS_TOPK_LAUNCH(CS_F32, false); }
  else if (dtype == CS_BF16) { if (cap) CS_TOPK_LAUNCH(CS_BF16, true); else CS_TOPK_LAUNCH(CS_BF16, false); }
  else { if (cap) CS_TOPK_LAUNCH(CS_F16, true); else CS_TOPK_LAUNCH(CS_F16, false); }
#undef CS_TOPK_LAUNCH
  int32_t n2 = 2;
  while (n2 < nkeys) n2 <<= 1;
  const int32_t lds_keys = n2 > kTopkChunk ? n2 : kTopkChunk;
  hipLaunchKernelGGL(vocab_topk_merge_kernel, dim3(static_cast<uint32_t>(rows)), dim3(256),
                     static_cast<size_t>(lds_keys) * sizeof(unsigned long long), st, part,
                     static_cast<int32_t>(nkeys), n2, k, out_ids, out_vals);
  return check_launch("cs_vocab_topk");
}

size_t cs_vocab_sample_workspace_size(int64_t rows, int64_t vocab, int32_t n_draw) {
  if (rows <= 0 || vocab <= 0 || n_draw <= 0) return 0;
  const SplitPlan p = plan_split(rows, vocab, CS_F32);  // elementwise loop: same split for every dtype
  return static_cast<size_t>(rows) * p.nsplit * (sizeof(float2) + n_draw * sizeof(DrawBest));
}

int cs_vocab_sample(const void* logits, int dtype, int64_t rows, int64_t vocab, int64_t ld,
                    float temperature, float softcap, const uint64_t* seeds, int32_t n_draw,
                    int32_t* out_ids, float* out_lp, void* workspace, size_t workspace_bytes,
                    cs_stream_t stream) {
  if (dtype != CS_F32 && dtype != CS_BF16 && dtype != CS_F16)
    return fail(CS_ERR_INVALID, "cs_vocab_sample: unknown dtype");
  if (rows < 0 || vocab <= 0 || ld < vocab || n_draw <= 0 || n_draw > kMaxDraws)
    return fail(CS_ERR_INVALID, "cs_vocab_sample: need rows >= 0, vocab > 0, ld >= vocab, 0 < n_draw <= 16");
  if (!(temperature > 0.0f) || std::isinf(temperature))
    return fail(CS_ERR_INVALID, "cs_vocab_sample: temperature must be finite and > 0");
  if (!(softcap >= 0.0f) || std::isinf(softcap))
    return fail(CS_ERR_INVALID, "cs_vocab_sample: softcap must be finite and >= 0");
  if (rows == 0) return CS_OK;
  if (!logits || !seeds || !out_ids) return fail(CS_ERR_INVALID, "cs_vocab_sample: NULL pointer");
  const SplitPlan plan = plan_split(rows, vocab, CS_F32);
  if (rows * plan.nsplit > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_vocab_sample: grid too large");
  const size_t need = cs_vocab_sample_workspace_size(rows, vocab, n_draw);
  if (!workspace || workspace_bytes < need)
    return fail(CS_ERR_WORKSPACE, "cs_vocab_sample: workspace smaller than cs_vocab_sample_workspace_size()");
  if (reinterpret_cast<uintptr_t>(workspace) % 8 != 0)
    return fail(CS_ERR_WORKSPACE, "cs_vocab_sample: workspace not 8-byte aligned");
  auto* lse_part = static_cast<float2*>(workspace);
  auto* draw_part = reinterpret_cast<DrawBest*>(lse_part + rows * plan.nsplit);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t ld_bytes = ld * elt_size(dtype);
  const float inv_cap = softcap > 0.0f ? 1.0f / softcap : 0.0f;
  const float inv_t = 1.0f / temperature;
  const char* lg = static_cast<const char*>(logits);
  const auto* sd = reinterpret_cast<const unsigned long long*>(seeds);
  const dim3 g1(static_cast<uint32_t>(rows * plan.nsplit)), g2(static_cast<uint32_t>(rows));
#define CS_SAMPLE_LAUNCH(DTV, CAPV)                                                              \
  do {                                                                                          \
    hipLaunchKernelGGL((vocab_sample_kernel<DTV, CAPV>), g1, dim3(256), 0, st, lg, vocab,       \
                       ld_bytes, plan.nsplit, plan.split_len, inv_t, softcap, inv_cap, sd,      \
                       n_draw, lse_part, draw_part);                                            \
    hipLaunchKernelGGL((vocab_sample_merge_kernel<DTV, CAPV>), g2, dim3(64), 0, st, lg,         \
                       ld_bytes, plan.nsplit, inv_t, softcap, inv_cap, lse_part, draw_part,     \
                       n_draw, out_ids, out_lp);                                                \
  } while (0)
  const bool cap = softcap > 0.0f;
  if (dtype == CS_F32) { if (cap) CS_SAMPLE_LAUNCH(CS_F32, true); else CS_SAMPLE_LAUNCH(CS_F32, false); }
  else if (dtype == CS_BF16) { if (cap) CS_SAMPLE_LAUNCH(CS_BF16, true); else CS_SAMPLE_LAUNCH(CS_BF16, false); }
  else { if (cap) CS_SAMPLE_LAUNCH(CS_F16, true); else CS_SAMPLE_LAUNCH(CS_F16, false); }
#undef CS_SAMPLE_LAUNCH
  return check_launch("cs_vocab_sample");
}

}  // extern "C"
