// consensus_scoring.hip — gfx950 (MI355X / CDNA4) kernels behind include/consensus_scoring.h.
//
// What the reference does (serially, remotely): for every (agent, candidate) it
// asks a hosted LLM for prompt log-probs (src/utils.py:201-281), folds them into a
// per-agent utility (src/methods/*.py) and reduces across agents with min / sum /
// sum-of-log (src/methods/beam_search.py:558, src/methods/best_of_n.py:401-408,
// src/evaluation.py:337-381, core.py:108-113).  Here the same arithmetic runs on
// the logits rows the local forward produced:
//
//   lsg_stream_kernel   HBM-bound: one pass over [rows, vocab] logits, online
//                       max / sum-exp per lane (exp2 on pre-scaled values), 4 x 16 B
//                       loads in flight per lane, wave64 butterfly + LDS merge.
//                       Few rows -> split-V: (row, split) workgroups write (m, s)
//                       partials and lsg_merge_kernel finishes lse + gather.
//   seg_reduce_kernel   one wave per candidate segment, fp64 sums in fixed order.
//   welfare_kernel      one lane per candidate column, agents folded in order.
//   topk_kernel         per-segment bitonic sort of (order-key, ~index) in LDS.
//
// No float atomics anywhere: every output is bitwise reproducible run to run.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "consensus_scoring.h"

namespace {

constexpr int kBlock = 256;   // streaming workgroup: 4 waves of 64
constexpr int kUnroll = 4;    // 16-byte vectors in flight per lane per iteration
constexpr int kMergeBlock = 64;
// split-V below this many workgroups: one 1024-thread workgroup per row already streams at
// the launch's floor once rows >= 256 (tools/split_sweep.py; profiles/r01_split_sweep.jsonl)
constexpr int64_t kTargetWgs = 256;
constexpr float kLog2e = 1.4426950408889634f;

thread_local std::string g_last_error = "";

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return fail(CS_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  }
  return CS_OK;
}

// ---------------------------------------------------------------------------
// element decoding
// ---------------------------------------------------------------------------
template <int DT>
struct Elt;
template <>
struct Elt<CS_F32> {
  static constexpr int kSize = 4;
  static constexpr int kPerVec = 4;
};
template <>
struct Elt<CS_BF16> {
  static constexpr int kSize = 2;
  static constexpr int kPerVec = 8;
};
template <>
struct Elt<CS_F16> {
  static constexpr int kSize = 2;
  static constexpr int kPerVec = 8;
};

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // one 16-byte global_load_dwordx4


template <int DT>
__device__ __forceinline__ void unpack_vec(const u32x4& q, float* v) {
  const uint32_t w[4] = {q[0], q[1], q[2], q[3]};
  if constexpr (DT == CS_F32) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(w[i]);
  } else if constexpr (DT == CS_BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);             // element 2i: low half
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);  // element 2i+1: high half
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const half2_t h = __builtin_bit_cast(half2_t, w[i]);
      v[2 * i] = (float)h[0];
      v[2 * i + 1] = (float)h[1];
    }
  }
}

template <int DT>
__device__ __forceinline__ float load_one(const char* row, int64_t i) {
  if constexpr (DT == CS_F32) {
    return reinterpret_cast<const float*>(row)[i];
  } else if constexpr (DT == CS_BF16) {
    return __uint_as_float(static_cast<uint32_t>(reinterpret_cast<const uint16_t*>(row)[i]) << 16);
  } else {
    return (float)reinterpret_cast<const _Float16*>(row)[i];
  }
}

// Gemma-2 final-logit soft-capping, cap * tanh(x / cap), written through one exp2 and
// the hardware reciprocal (1 ulp) so the vocab stream and the target gather use the
// identical function:  r = 1 / (exp(2x/cap) + 1),  cap * tanh(x/cap) = cap - 2 cap r.
// |error| ~ 1e-6 * cap, far inside the 1e-3 budget.  The constant 2 log2(e) / cap is
// formed once per kernel (loop-invariant), so an element costs mul, exp2, add, rcp, fma.
__device__ __forceinline__ float softcap_rcp(float x, float inv_cap) {
  return __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x * ((2.0f * kLog2e) * inv_cap)) + 1.0f);
}
__device__ __forceinline__ float softcap_fn(float x, float cap, float inv_cap) {
  return fmaf(-2.0f * cap, softcap_rcp(x, inv_cap), cap);
}
// exp(cap * tanh(x / cap)) for the fixed-offset sum, straight from the reciprocal:
// exp2(cap log2e - 2 cap log2e r), one fma instead of rebuilding x' and scaling it.
__device__ __forceinline__ float softcap_exp(float x, float cap, float inv_cap) {
  return __builtin_amdgcn_exp2f(fmaf((-2.0f * kLog2e) * cap, softcap_rcp(x, inv_cap), kLog2e * cap));
}

// ---------------------------------------------------------------------------
// online log-sum-exp state
// ---------------------------------------------------------------------------
// (m, s) represents sum_i exp(x_i) = s * exp(m).  m == -inf  <=>  empty.
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  // Symmetric in its two operands (two rounded products, one add; the library is built
  // with -ffp-contract=off), so both lanes of a butterfly pair compute the same merge
  // and every lane of a reduced wave holds bit-identical (m, s).
  s = s * __builtin_amdgcn_exp2f((m - mn) * kLog2e) + s2 * __builtin_amdgcn_exp2f((m2 - mn) * kLog2e);
  m = mn;
}

template <int N, bool FIXED = false>
__device__ __forceinline__ void lse_accum(float& m, float& s, const float* v) {
  if constexpr (FIXED) {  // m stays 0 (bounded soft-capped logits): s += sum exp(v)
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < N; ++i) acc += __builtin_amdgcn_exp2f(v[i] * kLog2e);
    s += acc;
    return;
  }
  float cm = v[0];
#pragma unroll
  for (int i = 1; i < N; ++i) cm = fmaxf(cm, v[i]);
  const float mn = fmaxf(m, cm);
  if (mn == -INFINITY) return;
  const float off = mn * kLog2e;
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) acc += __builtin_amdgcn_exp2f(fmaf(v[i], kLog2e, -off));
  s = fmaf(s, __builtin_amdgcn_exp2f(fmaf(m, kLog2e, -off)), acc);
  m = mn;
}

// N raw elements into (m, s): soft-capped first when CAP; with FIXED (bounded capped
// logits) the sum needs no running max and takes softcap_exp directly.
template <int N, bool CAP, bool FIXED>
__device__ __forceinline__ void accum_elems(float& m, float& s, float* v, float cap, float inv_cap) {
  if constexpr (CAP && FIXED) {
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < N; ++i) acc += softcap_exp(v[i], cap, inv_cap);
    s += acc;
  } else {
    if constexpr (CAP) {
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = softcap_fn(v[i], cap, inv_cap);
    }
    lse_accum<N, FIXED>(m, s, v);
  }
}

__device__ __forceinline__ void wave_lse_reduce(float& m, float& s) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float m2 = __shfl_xor(m, off, 64);
    const float s2 = __shfl_xor(s, off, 64);
    lse_merge(m, s, m2, s2);
  }
}

__device__ __forceinline__ void gather_targets(const char* row, int64_t vocab, float lse,
                                               const int32_t* __restrict__ tgt, int32_t k,
                                               float* __restrict__ out, bool cap_on, float cap,
                                               float inv_cap, int dt, int lane, int nlanes) {
  for (int j = lane; j < k; j += nlanes) {
    const int32_t t = tgt[j];
    float r = __builtin_nanf("");
    if (t >= 0 && t < vocab) {
      float x;
      if (dt == CS_F32)
        x = load_one<CS_F32>(row, t);
      else if (dt == CS_BF16)
        x = load_one<CS_BF16>(row, t);
      else
        x = load_one<CS_F16>(row, t);
      if (cap_on) x = softcap_fn(x, cap, inv_cap);
      r = x - lse;
    }
    out[j] = r;
  }
}

// ---------------------------------------------------------------------------
// streaming kernel: one workgroup per (row, split) work item
// ---------------------------------------------------------------------------
// One workgroup's (m, s) over logits[v0, v0 + n) of one row: scalar head up to the
// first 16-byte boundary and scalar tail after the last full vector, UNROLL
// non-temporal 16-byte loads in flight per lane (each logits byte is read once),
// wave64 butterfly, then the waves merged in order through LDS.  The result is valid
// in thread 0.  FIXED (soft-capped logits, |x'| <= cap <= 60): the sum needs no running
// max, s = sum exp(x') with m = 0, so the inner loop has no max / rescale.
template <int DT, bool CAP, bool FIXED, int BLOCK, int UNROLL>
__device__ __forceinline__ float2 block_lse_partial(const char* __restrict__ rp, int64_t v0,
                                                    int64_t n, float cap, float inv_cap,
                                                    float* sm_m, float* sm_s) {
  constexpr int ESZ = Elt<DT>::kSize;
  constexpr int EPV = Elt<DT>::kPerVec;
  constexpr int NW = BLOCK / 64;
  const int tid = threadIdx.x;
  float m = FIXED ? 0.0f : -INFINITY, s = 0.0f;

  const uintptr_t a0 = reinterpret_cast<uintptr_t>(rp + v0 * ESZ);
  int64_t head = static_cast<int64_t>(((16u - (a0 & 15u)) & 15u) / ESZ);
  if (head > n) head = n;
  const int64_t nvec = (n - head) / EPV;
  const int64_t tail0 = head + nvec * EPV;
  {
    float x = -INFINITY;
    bool have = false;
    if (tid < head) {
      x = load_one<DT>(rp, v0 + tid);
      have = true;
    } else if (tid >= 64 && tid - 64 < n - tail0) {
      x = load_one<DT>(rp, v0 + tail0 + (tid - 64));
      have = true;
    }
    if (have) {
      if constexpr (CAP && FIXED) {
        s += softcap_exp(x, cap, inv_cap);
      } else {
        if (CAP) x = softcap_fn(x, cap, inv_cap);
        if (x != -INFINITY) lse_accum<1, FIXED>(m, s, &x);
      }
    }
  }

  const u32x4* vp = reinterpret_cast<const u32x4*>(rp + (v0 + head) * ESZ);
  int64_t i = tid;
  constexpr int STEP = UNROLL * BLOCK;
  for (; i + (UNROLL - 1) * BLOCK < nvec; i += STEP) {
    u32x4 q[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) q[u] = __builtin_nontemporal_load(vp + i + u * BLOCK);
    float v[UNROLL * EPV];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) unpack_vec<DT>(q[u], v + u * EPV);
    accum_elems<UNROLL * EPV, CAP, FIXED>(m, s, v, cap, inv_cap);
  }
  for (; i < nvec; i += BLOCK) {
    const u32x4 q = __builtin_nontemporal_load(vp + i);
    float v[EPV];
    unpack_vec<DT>(q, v);
    accum_elems<EPV, CAP, FIXED>(m, s, v, cap, inv_cap);
  }

  wave_lse_reduce(m, s);
  const int wave = tid >> 6;
  if ((tid & 63) == 0) {
    sm_m[wave] = m;
    sm_s[wave] = s;
  }
  __syncthreads();
  float mm = sm_m[0], ss = sm_s[0];
  if (tid == 0) {
#pragma unroll
    for (int w = 1; w < NW; ++w) lse_merge(mm, ss, sm_m[w], sm_s[w]);
  }
  return make_float2(mm, ss);
}

// The fixed-offset sum is exact enough and cannot overflow for |x'| <= 60:
// e^60 * 2^31 < FLT_MAX and e^-60 is a normal float.
inline bool fixed_lse_ok(float cap) { return cap > 0.0f && cap <= 60.0f; }

// Work items (row, split) are walked grid-stride so a capped grid also works.
template <int DT, bool CAP, bool FIXED, int BLOCK, int UNROLL>
__global__ __launch_bounds__(BLOCK) void lsg_stream_kernel(
    const char* __restrict__ logits, int64_t n_items, int64_t vocab, int64_t ld_bytes,
    int32_t nsplit, int64_t split_len, const int32_t* __restrict__ tgt, int32_t k, float cap,
    float inv_cap, float* __restrict__ out_tok, float* __restrict__ out_lse,
    float2* __restrict__ part) {
  __shared__ float sm_m[BLOCK / 64];
  __shared__ float sm_s[BLOCK / 64];
  __shared__ float sm_lse;
  const int tid = threadIdx.x;

  for (int64_t bid = blockIdx.x; bid < n_items; bid += gridDim.x) {
    const int64_t row = bid / nsplit;
    const int32_t split = static_cast<int32_t>(bid - row * nsplit);
    const char* rp = logits + row * ld_bytes;
    const int64_t v0 = static_cast<int64_t>(split) * split_len;
    const int64_t v1 = min(vocab, v0 + split_len);
    const float2 ms =
        block_lse_partial<DT, CAP, FIXED, BLOCK, UNROLL>(rp, v0, v1 - v0, cap, inv_cap, sm_m, sm_s);
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

// Order key: larger float -> larger key; NaN below everything; -0 == +0.
__device__ __forceinline__ uint32_t order_key(float f) {
  if (__builtin_isnan(f)) return 0u;
  if (f == 0.0f) f = 0.0f;
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ W, int32_t seg_len,
                                                   int64_t ld, int32_t n2, int32_t k,
                                                   int32_t* __restrict__ out_idx,
                                                   float* __restrict__ out_val) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long ck[];
  const int64_t seg = blockIdx.x;
  const float* base = W + seg * ld;
  const int tid = threadIdx.x;
  // composite key: (order key, ~index) -> descending sort = value desc, index asc.
  for (int i = tid; i < n2; i += 256) {
    ck[i] = (i < seg_len) ? ((static_cast<unsigned long long>(order_key(base[i])) << 32) |
                             static_cast<unsigned long long>(0xffffffffu - static_cast<uint32_t>(i)))
                          : 0ull;
  }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (n2 >> 1); t += 256) {
        const int lo = ((t & ~(stride - 1)) << 1) | (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const unsigned long long a = ck[lo], b = ck[hi];
        if ((a < b) == desc) {
          ck[lo] = b;
          ck[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int r = tid; r < k; r += 256) {
    const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(ck[r] & 0xffffffffull);
    out_idx[seg * k + r] = static_cast<int32_t>(idx);
    if (out_val) out_val[seg * k + r] = base[idx];
  }
}

// ---------------------------------------------------------------------------
// host-side planning
// ---------------------------------------------------------------------------
int elt_size(int dtype) { return dtype == CS_F32 ? 4 : 2; }
int elt_per_vec(int dtype) { return dtype == CS_F32 ? 4 : 8; }

struct SplitPlan {
  int32_t nsplit;
  int64_t split_len;
};

int64_t target_wgs() {
  const char* e = getenv("CS_TARGET_WGS");  // tuning knob (tools/beam_ab.py); default 2048
  const int64_t v = e ? atoll(e) : 0;
  return v > 0 ? v : kTargetWgs;
}

SplitPlan plan_split(int64_t rows, int64_t vocab, int dtype) {
  SplitPlan p{1, vocab};
  const int64_t target = target_wgs();
  if (rows <= 0 || vocab <= 0 || rows >= target) return p;
  const int64_t grain = static_cast<int64_t>(kBlock) * elt_per_vec(dtype);  // one vector per lane
  const int64_t min_len = grain * kUnroll;  // >= one full unrolled sweep per split
  int64_t want = (target + rows - 1) / rows;
  int64_t max_split = vocab / min_len;
  if (max_split < 1) max_split = 1;
  if (want > max_split) want = max_split;
  if (want <= 1) return p;
  int64_t len = (vocab + want - 1) / want;
  len = ((len + grain - 1) / grain) * grain;
  p.split_len = len;
  p.nsplit = static_cast<int32_t>((vocab + len - 1) / len);
  if (p.nsplit <= 1) {
    p.nsplit = 1;
    p.split_len = vocab;
  }
  return p;
}

// Streaming-kernel configurations compiled into the library.  Variant 0 (default) is
// shape-aware, from the in-process A/B on the bench's data (profiles/r01_lsg_variants.jsonl):
//   single pass (rows >= 2048): 1024 threads x 2 vectors in flight  (C2: 7.25 TB/s, 90.6 %)
//   split-V (fewer rows):        256 threads x 8 vectors in flight
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
  const char* e = getenv("CS_LSG_VARIANT");
  return e ? atoi(e) : 0;
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
      if (plan.nsplit == 1)
        launch_stream<DT, CAP, 1024, 2>(logits, items, vocab, ld_bytes, plan, tgt, k, cap,
                                        inv_cap, out_tok, out_lse, part, st);
      else
        launch_stream<DT, CAP, 256, 8>(logits, items, vocab, ld_bytes, plan, tgt, k, cap,
                                       inv_cap, out_tok, out_lse, part, st);
      break;
  }
  if (plan.nsplit > 1 && finish) {
    hipLaunchKernelGGL((lsg_merge_kernel<DT, CAP>), dim3(static_cast<uint32_t>(rows)),
                       dim3(kMergeBlock), 0, st, static_cast<const char*>(logits), vocab, ld_bytes,
                       plan.nsplit, part, tgt, k, cap, inv_cap, out_tok, out_lse);
  }
}


// ---------------------------------------------------------------------------
// candidate proposer: vocab top-k and seeded Gumbel-max sampling
// ---------------------------------------------------------------------------
constexpr int kTopkChunk = 4096;   // vocab elements sorted per (row, chunk) workgroup
constexpr int kMaxDraws = 16;

__device__ __forceinline__ float key_to_float(uint32_t key) {
  if (key == 0u) return __builtin_nanf("");
  const uint32_t u = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
  return __uint_as_float(u);
}

template <int DT>
__device__ __forceinline__ float load_any(const char* row, int64_t i) {
  return load_one<DT>(row, i);
}

// Bitonic sort (descending) of n2 (power of two) 64-bit keys in LDS by `nthr` threads.
__device__ __forceinline__ void bitonic_desc(unsigned long long* ck, int n2, int tid, int nthr) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (n2 >> 1); t += nthr) {
        const int lo = ((t & ~(stride - 1)) << 1) | (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const unsigned long long a = ck[lo], b = ck[hi];
        if ((a < b) == desc) {
          ck[lo] = b;
          ck[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

// Top-k by histogram threshold (the fast path of both top-k kernels).  A block's keys are
// binned on their top 12 bits (sign, exponent and 3 mantissa bits of the value); the
// threshold bin t is the highest bin with count(bins > t) < k <= count(bins >= t), so
// every key of the top k lies in bins >= t.  Those candidates (typically k plus a few
// dozen) are ranked by counting in LDS: keys are distinct (the index is in the low word),
// so rank = #{larger keys} and the order is exactly the full sort's.  A block whose
// candidates overflow kTopkCand (massive ties: constant or masked rows) falls back to the
// full bitonic sort, which gives the identical result.
constexpr int kTopkBins = 4096;
constexpr int kTopkCand = 1024;
constexpr int kTopkPer = kTopkChunk / 256;   // keys per lane in the chunk kernel

__device__ __forceinline__ uint32_t key_bin(unsigned long long key) {
  return static_cast<uint32_t>(key >> 52);
}

// Threshold of an NT-thread block's histogram.  Thread i owns the kTopkBins / NT bins
// just below bin 4095 - i * (kTopkBins / NT), scanned from the top; returns
// (t, count(bins >= t)) in every thread, (0, total) when the block holds fewer than k
// keys.  sm_w holds NT / 64 wave totals.
template <int NT = 256>
__device__ __forceinline__ int2 hist_threshold(const uint32_t* hist, uint32_t k, uint32_t* sm_w,
                                               int* sm_res) {
  constexpr int PER = kTopkBins / NT;
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int top = kTopkBins - 1 - PER * tid;
  uint32_t c[PER];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    c[j] = hist[top - j];
    s += c[j];
  }
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) sm_w[wave] = inc;
  __syncthreads();
  uint32_t before = inc - s, total = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wave) before += sm_w[w];
    total += sm_w[w];
  }
  if (total < k) return make_int2(0, static_cast<int>(total));
  if (before < k && before + s >= k) {
    uint32_t acc = before;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (acc + c[j] >= k) {
        sm_res[0] = top - j;
        sm_res[1] = static_cast<int>(acc + c[j]);
        break;
      }
      acc += c[j];
    }
  }
  __syncthreads();
  return make_int2(sm_res[0], sm_res[1]);
}

// Rank the nc distinct candidate keys in LDS; key of rank r < k goes to emit(r, key).
template <int NT = 256, typename Emit>
__device__ __forceinline__ void rank_candidates(const unsigned long long* cand, int nc, int k,
                                                Emit emit) {
  for (int i = threadIdx.x; i < nc; i += NT) {
    const unsigned long long kc = cand[i];
    int r = 0;
#pragma unroll 8
    for (int j = 0; j < nc; ++j) r += cand[j] > kc ? 1 : 0;
    if (r < k) emit(r, kc);
  }
}

// Radix select over 12-bit digits from the top of the 64-bit keys: the first digit is
// hist_threshold's bin; while the keys that can still be among the k largest (every key
// of a higher bin, plus the threshold bin) number more than `limit`, the threshold bin is
// split on the next 12 bits.  Returns (shift, prefix, count): the keys with
// (key >> shift) >= prefix are the k largest plus the other keys of the last threshold
// bin, `count` of them.  The last digit sits at shift 4, where a bin holds at most 16
// distinct keys, so count <= k + 15 there.  Clustered values (e.g. beam rewards that
// share one exponent) refine instead of ranking hundreds of candidates.
// for_each(f) calls f(key) for each present key of the calling thread's share.
struct RadixCut {
  int shift;
  unsigned long long prefix;
  uint32_t count;
};

template <int NT, typename ForEach>
__device__ __forceinline__ RadixCut radix_select(ForEach for_each, uint32_t k, uint32_t limit,
                                                 uint32_t* hist, uint32_t* sm_w, int* sm_res) {
  int shift = 52;
  unsigned long long prefix = 0ull;
  uint32_t above = 0;
  for (;;) {
    for (int i = threadIdx.x; i < kTopkBins; i += NT) hist[i] = 0u;
    __syncthreads();
    const int sh = shift;
    const unsigned long long pf = prefix;
    for_each([&](unsigned long long key) {
      if (sh == 52 || (key >> (sh + 12)) == pf)
        atomicAdd(&hist[static_cast<uint32_t>(key >> sh) & (kTopkBins - 1)], 1u);
    });
    __syncthreads();
    const int2 th = hist_threshold<NT>(hist, k - above, sm_w, sm_res);
    const uint32_t in_bin = hist[th.x];
    prefix = (prefix << 12) | static_cast<unsigned long long>(th.x);
    const uint32_t count = above + static_cast<uint32_t>(th.y);
    if (count <= limit || shift < 12) return RadixCut{shift, prefix, count};
    above = count - in_bin;
    shift -= 12;
    __syncthreads();  // every thread has read hist before the next level clears it
  }
}

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

// ---------------------------------------------------------------------------
// beam step: one launch from logits to the ordered candidates
// ---------------------------------------------------------------------------
// A whole beam-search scoring step after the LM head (beam_search.py:495-560) in ONE
// launch, one workgroup per (agent row, vocab split):
//   1. stream the split -> (m, s) partial (block_lse_partial, as lsg_stream_kernel);
//   2. the LAST workgroup to finish a row (arrival counter per row) merges the row's
//      partials in split order (one wave, lanes over splits: lsg_merge_kernel's
//      arithmetic), gathers the row's K candidate tokens and writes
//      U[a, b*K+j] = R[a, b] + lp (fp32, the method's cumulative reward);
//   3. MIN / MAX welfare is order-free, so each row finisher also folds its K
//      utilities into a per-candidate key with one device-scope atomicMax (ordered
//      float keys; MIN stores inverted keys), and the LAST row to finish (one more
//      counter) only reads the C keys back.  SUM / SUMLOG (order matters in fp64) are
//      folded by the last row over the agents in agent order (welfare_kernel's fold,
//      non-finite skipped).  When B*K <= kFusedSort the last row then sorts the
//      (value desc, index asc) keys in LDS (topk_kernel's keys).
//   The candidate ids and their logits are loaded before the stream starts, so the
//   gather costs no memory round trip after the row's lse is known.
// Bit-identical to cs_logsoftmax_gather + cs_welfare_reduce + cs_segmented_topk.
// Hand-offs use sc1 stores / loads and arrival counters (no fences, see st_sc1).
// Nobody waits on anybody, so the launch cannot stall; the last arrivers reset the
// counters to zero, which keeps the workspace reusable (and graph-replayable) without
// a memset.
// Cross-workgroup hand-off without fences (MI355X_MICROARCH.md, hand-off table row 1):
// every handed-off byte is stored and loaded with sc1 (agent-scope relaxed atomics lower
// to global_store/global_load ... sc1: write-through past the L2, L1 bypassed), every
// storing wave waits vmcnt(0), the workgroup barriers, and ONE lane then adds to the
// arrival counter; the workgroup whose add returns the last count consumes.
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wait_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t arrive(uint32_t* cnt) {
  return __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Hand-off regions are padded so that every 128-byte line is read by ONE consumer
// workgroup, after all of it is published: a line is never in an L2 (per XCD) before its
// consumer's first read of it in the launch.
__host__ __device__ constexpr int64_t pad_line(int64_t n, int64_t elt_bytes) {
  return (n * elt_bytes + 127) / 128 * 128 / elt_bytes;
}

constexpr int kFusedSort = 1024;      // candidates sorted inside the launch
constexpr int kSelectMax = 256;       // n_order up to this: threshold selection, no full sort
constexpr int kBeamMaxRows = 65536;   // A * B (one arrival counter per row)
constexpr int kBeamMaxCand = 16384;   // B * K (one welfare key per candidate)
// workspace: [done counter | pad to 64 B][row counters][welfare keys][row partials]
constexpr size_t kBeamRowCntOff = 64;
constexpr size_t kBeamKeyOff = kBeamRowCntOff + sizeof(uint32_t) * kBeamMaxRows;
constexpr size_t kBeamCounterBytes = kBeamKeyOff + sizeof(uint32_t) * kBeamMaxCand;

// Welfare key of one utility for the atomic MIN / MAX fold: 0 = no finite value yet (the
// zeroed workspace state); order_key of a finite float is >= 0x00800000, so MAX keeps
// order_key(u) and MIN keeps ~order_key(u) (the largest inverted key is the minimum).
__device__ __forceinline__ uint32_t welfare_key(float u, bool is_min) {
  const uint32_t k = order_key(u);
  return is_min ? ~k : k;
}
__device__ __forceinline__ float welfare_from_key(uint32_t k, bool is_min) {
  if (k == 0u) return __builtin_nanf("");
  return key_to_float(is_min ? ~k : k);
}

__device__ __forceinline__ void welfare_fold(double& acc, bool& any, float u, int kind,
                                             double eps) {
  if (!__builtin_isfinite(u)) return;  // SKIP (and the masked tail of a batch)
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
    default:
      acc += log(fmax(d, eps));
      break;
  }
  any = true;
}

// Welfare of NQ candidates (c0, c0 + stride, ...) over all agents, in agent order; NQ x NA
// sc1 loads in flight per batch so the fold costs about one memory round trip per batch.
template <int NQ, int NA>
__device__ __forceinline__ void fold_candidates(uint32_t* U, int32_t A, int32_t C, int32_t c0,
                                                int32_t stride, int kind, double eps,
                                                double* acc, bool* any) {
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    acc[q] = 0.0;
    any[q] = false;
  }
  for (int32_t a0 = 0; a0 < A; a0 += NA) {
    float ub[NQ][NA];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int32_t c = c0 + q * stride;
#pragma unroll
      for (int j = 0; j < NA; ++j)
        ub[q][j] = (c < C && a0 + j < A)
                       ? __uint_as_float(ld_sc1(U + static_cast<int64_t>(a0 + j) * C + c))
                       : __builtin_nanf("");
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
#pragma unroll
      for (int j = 0; j < NA; ++j) welfare_fold(acc[q], any[q], ub[q][j], kind, eps);
    }
  }
}

// The kept beams' cumulative rewards: out_kept[a][r] = U[a][ord[r]] (ord in LDS), all
// A * n_order loads spread over the block so they are in flight together (U was written
// by other workgroups: sc1 loads).
template <int BLOCK>
__device__ __forceinline__ void keep_columns(uint32_t* U, float* out_kept, const int32_t* ord,
                                             int32_t A, int32_t C, int32_t n_order) {
  const int32_t n = A * n_order;
  for (int32_t i = threadIdx.x; i < n; i += BLOCK) {
    const int32_t a = i / n_order;
    const int32_t r = i - a * n_order;
    out_kept[i] = __uint_as_float(ld_sc1(U + static_cast<int64_t>(a) * C + ord[r]));
  }
}

// Descending bitonic sort of n2 (a power of two <= KPT * BLOCK) distinct keys held in
// registers: element i = r * BLOCK + tid lives in kv[r] of thread tid.  Exchanges at
// stride < 64 go through wave shuffles (no barrier), at stride >= BLOCK between the
// thread's own registers, and only the strides in between through LDS, double-buffered
// so that each such pass costs one barrier.  For n2 = 1024 on 1024 threads: 10 LDS
// passes of the 55 instead of 55 barrier-separated LDS passes.
__device__ __forceinline__ unsigned long long bitonic_pick(unsigned long long a,
                                                           unsigned long long b, int i, int stride,
                                                           int size) {
  const bool keep_max = ((i & stride) == 0) == ((i & size) == 0);
  return keep_max ? (a > b ? a : b) : (a < b ? a : b);
}

template <int BLOCK, int KPT>
__device__ __forceinline__ void bitonic_desc_regs(unsigned long long (&kv)[KPT], int n2,
                                                  unsigned long long* buf0,
                                                  unsigned long long* buf1) {
  const int tid = threadIdx.x;
  bool flip = false;
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= BLOCK) {
        const int rs = stride / BLOCK;
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
          if ((r & rs) == 0 && (r | rs) < KPT) {
            const int i = r * BLOCK + tid;
            if (i < n2) {
              const unsigned long long a = kv[r], b = kv[r | rs];
              const bool desc = (i & size) == 0;
              if ((a < b) == desc) {
                kv[r] = b;
                kv[r | rs] = a;
              }
            }
          }
        }
      } else if (stride >= 64) {
        unsigned long long* buf = flip ? buf1 : buf0;
        flip = !flip;
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
          const int i = r * BLOCK + tid;
          if (i < n2) buf[i] = kv[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
          const int i = r * BLOCK + tid;
          if (i < n2) kv[r] = bitonic_pick(kv[r], buf[i ^ stride], i, stride, size);
        }
      } else {
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
          const int i = r * BLOCK + tid;
          const unsigned long long b = __shfl_xor(kv[r], stride, 64);
          if (i < n2) kv[r] = bitonic_pick(kv[r], b, i, stride, size);
        }
      }
    }
  }
}

// LDS of the beam kernels' last-workgroup tail (welfare readback / fold, order, kept).
struct BeamLds {
  unsigned long long* keys;   // 2 * kFusedSort: bitonic buffers, or one 16 KB histogram
  unsigned long long* keys2;
  unsigned long long* sel_cand;  // kTopkCand
  float* sm_w;                   // kFusedSort
  int32_t* sm_ord;               // kFusedSort
  uint32_t* sm_tw;               // BLOCK / 64
  int* sm_res;                   // 2
  uint32_t* sm_n;
};

// Run by the last workgroup of a beam step once every U value (and, for MIN / MAX, every
// welfare key) is published: W for every candidate, then the order (radix-select top-n
// or the full bitonic sort) and the kept beams' rewards.
template <int BLOCK>
__device__ __forceinline__ void beam_tail(const BeamLds& L, uint32_t* Uw, uint32_t* wkey,
                                          float* __restrict__ W, int32_t A, int32_t C, int kind,
                                          double eps, int32_t n_order, int32_t n2,
                                          int32_t* __restrict__ out_order,
                                          float* __restrict__ out_val,
                                          float* __restrict__ out_kept) {
  const int tid = threadIdx.x;
  const bool order_free = kind == CS_WELFARE_MIN || kind == CS_WELFARE_MAX;
  const bool is_min = kind == CS_WELFARE_MIN;
  unsigned long long* keys = L.keys;
  unsigned long long* keys2 = L.keys2;
  unsigned long long* sel_cand = L.sel_cand;
  float* sm_w = L.sm_w;
  int32_t* sm_ord = L.sm_ord;
  uint32_t* sm_tw = L.sm_tw;
  int* sm_res = L.sm_res;
  uint32_t& sm_n = *L.sm_n;
  const bool sort_here = n_order > 0 && n2 <= kFusedSort;
  if (order_free) {
    for (int32_t c = tid; c < C; c += BLOCK) {
      const float w = welfare_from_key(ld_sc1(wkey + c), is_min);
      st_sc1(wkey + c, 0u);  // leave the workspace zeroed for the next call
      W[c] = w;
      if (sort_here) sm_w[c] = w;
    }
  } else {
    for (int32_t c = tid; c < C; c += BLOCK) {
      double acc[1];
      bool any[1];
      fold_candidates<1, 16>(Uw, A, C, c, BLOCK, kind, eps, acc, any);
      const float w = any[0] ? static_cast<float>(acc[0]) : __builtin_nanf("");
      W[c] = w;
      if (sort_here) sm_w[c] = w;
    }
  }
  if (!sort_here) return;  // block-uniform
  __syncthreads();
  if (n_order <= kSelectMax) {
    // the n_order best by histogram threshold + rank counting (as vocab_topk): the
    // candidates' (value, ~index) keys are distinct, so the order is the full sort's
    uint32_t* hist = reinterpret_cast<uint32_t*>(keys);      // keys + keys2: 16 KB
    unsigned long long* cand = sel_cand;
    if (tid == 0) sm_n = 0u;
    unsigned long long kc[kFusedSort / BLOCK];
#pragma unroll
    for (int r = 0; r < kFusedSort / BLOCK; ++r) {
      const int32_t c = r * BLOCK + tid;
      kc[r] = c < C ? (static_cast<unsigned long long>(order_key(sm_w[c])) << 32) |
                          static_cast<unsigned long long>(0xffffffffu - static_cast<uint32_t>(c))
                    : 0ull;
    }
    const RadixCut cut = radix_select<BLOCK>(
        [&](auto f) {
#pragma unroll
          for (int r = 0; r < kFusedSort / BLOCK; ++r)
            if (kc[r]) f(kc[r]);
        },
        static_cast<uint32_t>(n_order), static_cast<uint32_t>(n_order + 64), hist, sm_tw, sm_res);
    if (cut.count <= kTopkCand) {  // block-uniform
#pragma unroll
      for (int r = 0; r < kFusedSort / BLOCK; ++r)
        if (kc[r] && (kc[r] >> cut.shift) >= cut.prefix) cand[atomicAdd(&sm_n, 1u)] = kc[r];
      __syncthreads();
      rank_candidates<BLOCK>(cand, static_cast<int>(sm_n), n_order,
                             [&](int r, unsigned long long key) {
                               const int32_t c = static_cast<int32_t>(
                                   0xffffffffu - static_cast<uint32_t>(key & 0xffffffffull));
                               out_order[r] = c;
                               if (out_val) out_val[r] = sm_w[c];
                               sm_ord[r] = c;
                             });
      if (out_kept) {
        __syncthreads();
        keep_columns<BLOCK>(Uw, out_kept, sm_ord, A, C, n_order);
      }
      return;
    }
    __syncthreads();  // the fallback sort below reuses keys / keys2
  }
  constexpr int KPT = kFusedSort / BLOCK;
  unsigned long long kv[KPT];
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    const int32_t c = r * BLOCK + tid;
    kv[r] = c < C ? (static_cast<unsigned long long>(order_key(sm_w[c])) << 32) |
                        static_cast<unsigned long long>(0xffffffffu - static_cast<uint32_t>(c))
                  : 0ull;
  }
  bitonic_desc_regs<BLOCK, KPT>(kv, n2, keys, keys2);
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    const int32_t i = r * BLOCK + tid;
    if (i < n_order) {
      const int32_t c = static_cast<int32_t>(0xffffffffu - static_cast<uint32_t>(kv[r] & 0xffffffffull));
      out_order[i] = c;
      if (out_val) out_val[i] = sm_w[c];
      sm_ord[i] = c;
    }
  }
  if (out_kept) {
    __syncthreads();
    keep_columns<BLOCK>(Uw, out_kept, sm_ord, A, C, n_order);
  }
}

template <int DT, bool CAP, bool FIXED, int BLOCK, int UNROLL>
__global__ __launch_bounds__(BLOCK, BLOCK >= 1024 ? 8 : 4) void beam_step_kernel(
    const char* __restrict__ logits, int64_t vocab, int64_t ld_bytes, int32_t nsplit,
    int64_t split_len, int32_t A, int32_t B, int32_t K, const int32_t* __restrict__ tgt,
    const float* __restrict__ R, float cap, float inv_cap, int kind, double eps,
    unsigned long long* __restrict__ part, uint32_t* __restrict__ row_cnt,
    uint32_t* __restrict__ done_cnt, uint32_t* __restrict__ wkey, float* __restrict__ U,
    float* __restrict__ W, int32_t n_order, int32_t n2, int32_t* __restrict__ out_order,
    float* __restrict__ out_val, float* __restrict__ out_kept) {
  __shared__ float sm_m[BLOCK / 64];
  __shared__ float sm_s[BLOCK / 64];
  __shared__ float sm_lse;
  __shared__ int sm_last;
  // keys2 directly after keys: the selection path uses the pair as one 16 KB histogram
  __shared__ __attribute__((aligned(16))) unsigned long long keys[2 * kFusedSort];
  unsigned long long* keys2 = keys + kFusedSort;
  __shared__ __attribute__((aligned(16))) unsigned long long sel_cand[kTopkCand];
  __shared__ float sm_w[kFusedSort];
  __shared__ int32_t sm_ord[kFusedSort];
  __shared__ uint32_t sm_tw[BLOCK / 64];
  __shared__ int sm_res[2];
  __shared__ uint32_t sm_n;
  const BeamLds L{keys, keys2, sel_cand, sm_w, sm_ord, sm_tw, sm_res, &sm_n};
  const int tid = threadIdx.x;
  const int32_t rows = A * B;
  const int32_t C = B * K;
  const int64_t item = blockIdx.x;
  const int32_t row = static_cast<int32_t>(item / nsplit);
  const int32_t split = static_cast<int32_t>(item - static_cast<int64_t>(row) * nsplit);
  const int32_t ag = row / B;
  const int32_t bm = row - ag * B;
  const char* rp = logits + row * ld_bytes;
  const int64_t v0 = static_cast<int64_t>(split) * split_len;
  const int64_t v1 = min(vocab, v0 + split_len);
  uint32_t* Uw = reinterpret_cast<uint32_t*>(U);
  const bool order_free = kind == CS_WELFARE_MIN || kind == CS_WELFARE_MAX;
  const bool is_min = kind == CS_WELFARE_MIN;
  // the candidate ids and their logits are read now (used only at the row finish), so
  // the finisher's gather costs no memory round trip after the lse is known
  const int32_t t_pre = (tid < K) ? tgt[bm * K + tid] : -1;
  const bool ok = t_pre >= 0 && t_pre < vocab;
  const float xg = ok ? load_one<DT>(rp, t_pre) : 0.0f;

  // 1. stream
  const float2 ms =
      block_lse_partial<DT, CAP, FIXED, BLOCK, UNROLL>(rp, v0, v1 - v0, cap, inv_cap, sm_m, sm_s);

  // 2. row finish by the row's last arriver
  if (nsplit > 1) {
    if (tid == 0) {
      st_sc1(part + static_cast<int64_t>(row) * pad_line(nsplit, 8) + split,
             (static_cast<unsigned long long>(__float_as_uint(ms.y)) << 32) |
                              __float_as_uint(ms.x));
      wait_stores();
      sm_last = arrive(&row_cnt[row]) == static_cast<uint32_t>(nsplit - 1);
    }
    __syncthreads();
    if (!sm_last) return;  // block-uniform
    if (tid < 64) {
      float m = -INFINITY, s = 0.0f;
      for (int j = tid; j < nsplit; j += 64) {
        const unsigned long long p = ld_sc1(part + static_cast<int64_t>(row) * pad_line(nsplit, 8) + j);
        lse_merge(m, s, __uint_as_float(static_cast<uint32_t>(p)),
                  __uint_as_float(static_cast<uint32_t>(p >> 32)));
      }
      wave_lse_reduce(m, s);
      if (tid == 0) {
        sm_lse = m + logf(s);
        st_sc1(row_cnt + row, 0u);
      }
    }
  } else if (tid == 0) {
    sm_lse = ms.x + logf(ms.y);
  }
  {
    __syncthreads();
    const float r0 = R[row];
    const float lse = sm_lse;
    for (int32_t j = tid; j < K; j += BLOCK) {
      float x = xg;
      bool okj = ok;
      if (j >= BLOCK) {  // K > BLOCK: the remaining ids the early read did not cover
        const int32_t t = tgt[bm * K + j];
        okj = t >= 0 && t < vocab;
        if (okj) x = load_one<DT>(rp, t);
      }
      float lp = __builtin_nanf("");
      if (okj) {
        if (CAP) x = softcap_fn(x, cap, inv_cap);
        lp = x - lse;
      }
      const float u = r0 + lp;
      st_sc1(Uw + static_cast<int64_t>(ag) * C + bm * K + j, __float_as_uint(u));
      if (order_free && __builtin_isfinite(u))
        __hip_atomic_fetch_max(wkey + bm * K + j, welfare_key(u, is_min), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // 3. welfare + order by the last row
  wait_stores();
  __syncthreads();
  if (tid == 0) sm_last = arrive(done_cnt) == static_cast<uint32_t>(rows - 1);
  __syncthreads();
  if (!sm_last) return;  // block-uniform
  if (tid == 0) st_sc1(done_cnt, 0u);
  beam_tail<BLOCK>(L, Uw, wkey, W, A, C, kind, eps, n_order, n2, out_order, out_val, out_kept);
}

// ---------------------------------------------------------------------------
// beam decode step: proposer + scoring in ONE launch
// ---------------------------------------------------------------------------
// cs_vocab_topk on the B reference-policy rows and cs_beam_step on the A*B agent rows
// in one grid, so the proposer's latency hides under the agent-row stream:
//   * blocks [0, B * nchunk): proposer, one per (beam, 16 * BLOCK-element chunk) of the
//     reference row: the chunk's K best composite keys by radix select + rank counting
//     (as vocab_topk_chunk_kernel), handed off; the last chunk of a beam merges the
//     chunk winners the same way and publishes the beam's K candidate ids (out_ids);
//   * blocks [B * nchunk, ...): one per (agent row, vocab split), the beam step's stream;
//     the row's last split publishes the row's log-sum-exp;
//   * per beam an arrival counter takes A + 1 arrivals (its A agent rows and its
//     proposer); the LAST arriver gathers all A x K candidates of that beam (ids, row
//     lse, logits), writes U and folds MIN / MAX welfare keys;
//   * the last beam to finish runs the beam step's tail (beam_tail).
// Proposer blocks come first in the grid, so they are dispatched first.  No block waits
// on another (last-arriver hand-offs only), so the launch cannot stall.  Bit-identical to
// cs_vocab_topk + cs_beam_step (same selection, same lse arithmetic, same U formula).
// Proposer keys per lane: 16, unless that leaves fewer than 128 proposer workgroups
// (few beams, e.g. C5's B = 8): then 4, so the proposer finishes under the agent-row
// stream (tools/beam_ab.py, profiles/r01f_beam_ab.jsonl).  CS_DECODE_KP overrides.
int decode_kp(int32_t B, int64_t vocab, int32_t block, int32_t K) {
  const char* e = getenv("CS_DECODE_KP");
  if (e && (atoi(e) == 4 || atoi(e) == 16)) return atoi(e);
  const int64_t n16 = B * ((vocab + 16LL * block - 1) / (16LL * block));
  const int64_t n4c = (vocab + 4LL * block - 1) / (4LL * block);
  return (n16 < 128 && n4c * K <= 16384) ? 4 : 16;
}
int decode_rows_first() {  // tuning knob CS_DECODE_ROWS_FIRST
  const char* e = getenv("CS_DECODE_ROWS_FIRST");
  return (e && atoi(e) == 1) ? 1 : 0;
}
#ifdef CS_TRACE_DECODE
__device__ unsigned long long g_dec_t0 = ~0ull;
#define DEC_T(...) __VA_ARGS__
#else
#define DEC_T(...)
#endif
constexpr int kBeamMaxBeams = 4096;

template <int DT, bool CAP, bool FIXED, int BLOCK, int UNROLL, int KP>
__global__ __launch_bounds__(BLOCK, BLOCK >= 1024 ? 8 : 4) void beam_decode_kernel(
    const char* __restrict__ ref, int64_t ld_ref_bytes, int32_t nchunk_p, int32_t rows_first,
    const char* __restrict__ logits, int64_t vocab, int64_t ld_bytes, int32_t nsplit,
    int64_t split_len, int32_t A, int32_t B, int32_t K, const float* __restrict__ R, float cap,
    float inv_cap, int kind, double eps, unsigned long long* __restrict__ part,
    unsigned long long* __restrict__ ppart, uint32_t* __restrict__ row_cnt,
    uint32_t* __restrict__ prop_cnt, uint32_t* __restrict__ beam_cnt,
    uint32_t* __restrict__ done_cnt, uint32_t* __restrict__ wkey, uint32_t* __restrict__ lse_ws,
    uint32_t* __restrict__ ids_ws, int32_t* __restrict__ out_ids, float* __restrict__ U, float* __restrict__ W, int32_t n_order,
    int32_t n2, int32_t* __restrict__ out_order, float* __restrict__ out_val,
    float* __restrict__ out_kept) {
  __shared__ float sm_m[BLOCK / 64];
  __shared__ float sm_s[BLOCK / 64];
  __shared__ float sm_lse;
  __shared__ int sm_last;
  __shared__ __attribute__((aligned(16))) unsigned long long keys[2 * kFusedSort];
  unsigned long long* keys2 = keys + kFusedSort;
  __shared__ __attribute__((aligned(16))) unsigned long long sel_cand[kTopkCand];
  __shared__ float sm_w[kFusedSort];
  __shared__ int32_t sm_ord[kFusedSort];
  __shared__ uint32_t sm_tw[BLOCK / 64];
  __shared__ int sm_res[2];
  __shared__ uint32_t sm_n;
  const BeamLds L{keys, keys2, sel_cand, sm_w, sm_ord, sm_tw, sm_res, &sm_n};
  uint32_t* hist = reinterpret_cast<uint32_t*>(keys);  // 16 KB
  const int tid = threadIdx.x;
  const int32_t C = B * K;
  const int32_t n_prop = B * nchunk_p;
  const bool is_min = kind == CS_WELFARE_MIN;
  const bool order_free = kind == CS_WELFARE_MIN || kind == CS_WELFARE_MAX;
  uint32_t* Uw = reinterpret_cast<uint32_t*>(U);
  DEC_T(const unsigned long long q0 = wall_clock64(); if (tid == 0) atomicMin(&g_dec_t0, q0);)
  int32_t gb;  // the beam this block arrives at

  const int32_t n_rowblk = static_cast<int32_t>(gridDim.x) - n_prop;
  // block role: proposer blocks first in the grid, or after the row blocks
  const int32_t pblk = rows_first ? static_cast<int32_t>(blockIdx.x) - n_rowblk
                                  : static_cast<int32_t>(blockIdx.x);
  const int32_t rblk = rows_first ? static_cast<int32_t>(blockIdx.x)
                                  : static_cast<int32_t>(blockIdx.x) - n_prop;
  if (pblk >= 0 && pblk < n_prop) {
    // ---- proposer chunk ----
    constexpr int CH = KP * BLOCK;
    const int32_t b = pblk / nchunk_p;
    const int32_t chunk = pblk - b * nchunk_p;
    const char* rp = ref + b * ld_ref_bytes;
    const int64_t v0 = static_cast<int64_t>(chunk) * CH;
    const int n = static_cast<int>(min(static_cast<int64_t>(CH), vocab - v0));
    unsigned long long key[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      const int i = tid + BLOCK * j;
      float x = 0.0f;
      if (i < n) x = load_one<DT>(rp, v0 + i);
      key[j] = 0ull;
      if (i < n) {
        if (CAP) x = softcap_fn(x, cap, inv_cap);
        key[j] = (static_cast<unsigned long long>(order_key(x)) << 32) |
                 static_cast<unsigned long long>(0xffffffffu - static_cast<uint32_t>(v0 + i));
      }
    }
    if (tid == 0) sm_n = 0u;
    const RadixCut cut = radix_select<BLOCK>(
        [&](auto f) {
#pragma unroll
          for (int j = 0; j < KP; ++j)
            if (key[j]) f(key[j]);
        },
        static_cast<uint32_t>(K), static_cast<uint32_t>(2 * K + 64), hist, sm_tw, sm_res);
#pragma unroll
    for (int j = 0; j < KP; ++j)
      if (key[j] && (key[j] >> cut.shift) >= cut.prefix) sel_cand[atomicAdd(&sm_n, 1u)] = key[j];
    __syncthreads();
    const int32_t nkeys = nchunk_p * K;
    unsigned long long* pr = ppart + static_cast<int64_t>(b) * pad_line(nkeys, 8);
    unsigned long long* out = pr + static_cast<int64_t>(chunk) * K;
    const int nc = static_cast<int>(sm_n);
    rank_candidates<BLOCK>(sel_cand, nc, K, [&](int r, unsigned long long kc) { st_sc1(out + r, kc); });
    for (int r = nc + tid; r < K; r += BLOCK) st_sc1(out + r, 0ull);
    wait_stores();
    __syncthreads();
    if (tid == 0) {
      sm_last = arrive(&prop_cnt[b]) == static_cast<uint32_t>(nchunk_p - 1);
      sm_n = 0u;
    }
    __syncthreads();
    if (!sm_last) return;  // block-uniform
    if (tid == 0) st_sc1(prop_cnt + b, 0u);
    // the beam's K best among the chunk winners -> its candidate ids
    const RadixCut mcut = radix_select<BLOCK>(
        [&](auto f) {
          for (int i = tid; i < nkeys; i += BLOCK) {
            const unsigned long long c = ld_sc1(pr + i);
            if (c) f(c);
          }
        },
        static_cast<uint32_t>(K), static_cast<uint32_t>(2 * K + 64), hist, sm_tw, sm_res);
    for (int i = tid; i < nkeys; i += BLOCK) {
      const unsigned long long c = ld_sc1(pr + i);
      if (c && (c >> mcut.shift) >= mcut.prefix) sel_cand[atomicAdd(&sm_n, 1u)] = c;
    }
    __syncthreads();
    const int mc = static_cast<int>(sm_n);
    rank_candidates<BLOCK>(sel_cand, mc, K, [&](int r, unsigned long long c) {
      const uint32_t id = 0xffffffffu - static_cast<uint32_t>(c & 0xffffffffull);
      st_sc1(ids_ws + b * pad_line(K, 4) + r, id);
      out_ids[b * K + r] = static_cast<int32_t>(id);
    });
    for (int r = mc + tid; r < K; r += BLOCK) {
      st_sc1(ids_ws + b * pad_line(K, 4) + r, 0xffffffffu);
      out_ids[b * K + r] = -1;
    }
    DEC_T(if (tid == 0 && b == 0) printf("DEC proposer merge done b0 at %llu (start %llu)\n", wall_clock64() - g_dec_t0, q0 - g_dec_t0);)
    gb = b;
  } else {
    // ---- agent row stream ----
    const int64_t item = rblk;
    const int32_t row = static_cast<int32_t>(item / nsplit);
    const int32_t split = static_cast<int32_t>(item - static_cast<int64_t>(row) * nsplit);
    const char* rp = logits + row * ld_bytes;
    const int64_t v0 = static_cast<int64_t>(split) * split_len;
    const int64_t v1 = min(vocab, v0 + split_len);
    const float2 ms =
        block_lse_partial<DT, CAP, FIXED, BLOCK, UNROLL>(rp, v0, v1 - v0, cap, inv_cap, sm_m, sm_s);
    if (nsplit > 1) {
      if (tid == 0) {
        st_sc1(part + static_cast<int64_t>(row) * pad_line(nsplit, 8) + split,
               (static_cast<unsigned long long>(__float_as_uint(ms.y)) << 32) |
                                __float_as_uint(ms.x));
        wait_stores();
        sm_last = arrive(&row_cnt[row]) == static_cast<uint32_t>(nsplit - 1);
      }
      __syncthreads();
      if (!sm_last) return;  // block-uniform
      if (tid < 64) {
        float m = -INFINITY, sum = 0.0f;
        for (int j = tid; j < nsplit; j += 64) {
          const unsigned long long pv = ld_sc1(part + static_cast<int64_t>(row) * pad_line(nsplit, 8) + j);
          lse_merge(m, sum, __uint_as_float(static_cast<uint32_t>(pv)),
                    __uint_as_float(static_cast<uint32_t>(pv >> 32)));
        }
        wave_lse_reduce(m, sum);
        if (tid == 0) {
          st_sc1(lse_ws + (row % B) * pad_line(A, 4) + row / B, __float_as_uint(m + logf(sum)));
          st_sc1(row_cnt + row, 0u);
        }
      }
    } else if (tid == 0) {
      st_sc1(lse_ws + (row % B) * pad_line(A, 4) + row / B, __float_as_uint(ms.x + logf(ms.y)));
    }
    gb = row % B;
    DEC_T(if (tid == 0 && (row == 0 || row == A * B - 1)) printf("DEC row %d stream start %llu done %llu\n", row, q0 - g_dec_t0, wall_clock64() - g_dec_t0);)
  }

  // ---- arrival at beam gb (A agent rows + its proposer); the last one gathers ----
  wait_stores();
  __syncthreads();
  if (tid == 0) sm_last = arrive(&beam_cnt[gb]) == static_cast<uint32_t>(A);
  __syncthreads();
  if (!sm_last) return;  // block-uniform
  if (tid == 0) st_sc1(beam_cnt + gb, 0u);
  for (int32_t i = tid; i < A * K; i += BLOCK) {
    const int32_t a = i / K;
    const int32_t j = i - a * K;
    const int32_t row = a * B + gb;
    const int32_t t = static_cast<int32_t>(ld_sc1(ids_ws + gb * pad_line(K, 4) + j));
    const float lse = __uint_as_float(ld_sc1(lse_ws + gb * pad_line(A, 4) + a));
    float lp = __builtin_nanf("");
    if (t >= 0 && t < vocab) {
      float x = load_one<DT>(logits + row * ld_bytes, t);
      if (CAP) x = softcap_fn(x, cap, inv_cap);
      lp = x - lse;
    }
    const float u = R[row] + lp;
    st_sc1(Uw + static_cast<int64_t>(a) * C + gb * K + j, __float_as_uint(u));
    if (order_free && __builtin_isfinite(u))
      __hip_atomic_fetch_max(wkey + gb * K + j, welfare_key(u, is_min), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
  wait_stores();
  __syncthreads();
  if (tid == 0) sm_last = arrive(done_cnt) == static_cast<uint32_t>(B - 1);
  __syncthreads();
  if (!sm_last) return;  // block-uniform
  if (tid == 0) st_sc1(done_cnt, 0u);
  DEC_T(const unsigned long long q8 = wall_clock64();)
  beam_tail<BLOCK>(L, Uw, wkey, W, A, C, kind, eps, n_order, n2, out_order, out_val, out_kept);
  DEC_T(if (tid == 0) { printf("DEC last gather+done at %llu, tail end %llu\n", q8 - g_dec_t0, wall_clock64() - g_dec_t0); g_dec_t0 = ~0ull; })
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* cs_version(void) { return "consensus_scoring 0.1.0 (gfx950)"; }

const char* cs_last_error(void) { return g_last_error.c_str(); }

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
size_t cs_beam_step_workspace_size(int64_t rows, int64_t vocab) {
  if (rows <= 0 || vocab <= 0) return 0;
  const SplitPlan p = plan_split(rows, vocab, CS_BF16);
  const SplitPlan q = plan_split(rows, vocab, CS_F32);
  const int64_t ns = p.nsplit > q.nsplit ? p.nsplit : q.nsplit;
  return kBeamCounterBytes + static_cast<size_t>(rows) * pad_line(ns, 8) * sizeof(unsigned long long);
}

int cs_beam_step(const void* logits, int dtype, int32_t A, int32_t B, int64_t vocab, int64_t ld,
                 const int32_t* targets, int32_t K, const float* rewards_in, float softcap,
                 int welfare_kind, float eps, float* out_U, float* out_W, int32_t n_order,
                 int32_t* out_order, float* out_order_val, float* out_kept, void* workspace,
                 size_t workspace_bytes, cs_stream_t stream) {
  if (dtype != CS_F32 && dtype != CS_BF16 && dtype != CS_F16)
    return fail(CS_ERR_INVALID, "cs_beam_step: unknown dtype");
  if (A < 0 || B < 0 || K < 0 || vocab <= 0 || ld < vocab)
    return fail(CS_ERR_INVALID, "cs_beam_step: need A, B, K >= 0, vocab > 0, ld >= vocab");
  const int64_t rows = static_cast<int64_t>(A) * B;
  const int64_t C = static_cast<int64_t>(B) * K;
  if (C > 16384) return fail(CS_ERR_INVALID, "cs_beam_step: B*K exceeds 16384");
  if (rows > kBeamMaxRows) return fail(CS_ERR_INVALID, "cs_beam_step: A*B exceeds 65536");
  if (n_order < 0 || n_order > C) return fail(CS_ERR_INVALID, "cs_beam_step: need 0 <= n_order <= B*K");
  if (out_kept && (n_order == 0 || C > kFusedSort))
    return fail(CS_ERR_INVALID, "cs_beam_step: out_kept needs n_order > 0 and B*K <= 1024");
  if (welfare_kind < CS_WELFARE_MIN || welfare_kind > CS_WELFARE_MAX)
    return fail(CS_ERR_INVALID, "cs_beam_step: unknown welfare kind");
  if (!(softcap >= 0.0f) || std::isinf(softcap))
    return fail(CS_ERR_INVALID, "cs_beam_step: softcap must be finite and >= 0");
  if (C == 0) return CS_OK;
  if (A == 0) return fail(CS_ERR_INVALID, "cs_beam_step: no agents");
  if (!logits || !targets || !rewards_in || !out_U || !out_W || (n_order > 0 && !out_order))
    return fail(CS_ERR_INVALID, "cs_beam_step: NULL pointer");
  if (reinterpret_cast<uintptr_t>(logits) % elt_size(dtype) != 0)
    return fail(CS_ERR_INVALID, "cs_beam_step: logits not element-aligned");
  const SplitPlan plan = plan_split(rows, vocab, dtype);
  const size_t need = kBeamCounterBytes + static_cast<size_t>(rows) * pad_line(plan.nsplit, 8) *
                                              sizeof(unsigned long long);
  if (!workspace || workspace_bytes < need)
    return fail(CS_ERR_WORKSPACE, "cs_beam_step: workspace smaller than cs_beam_step_workspace_size()");
  if (reinterpret_cast<uintptr_t>(workspace) % 8 != 0)
    return fail(CS_ERR_WORKSPACE, "cs_beam_step: workspace not 8-byte aligned");
  if (rows * plan.nsplit > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_beam_step: grid too large");
  char* wsb = static_cast<char*>(workspace);
  auto* done_cnt = reinterpret_cast<uint32_t*>(wsb);
  auto* row_cnt = reinterpret_cast<uint32_t*>(wsb + kBeamRowCntOff);
  auto* wkey = reinterpret_cast<uint32_t*>(wsb + kBeamKeyOff);
  auto* part = reinterpret_cast<unsigned long long*>(wsb + kBeamCounterBytes);
  const int64_t ld_bytes = ld * elt_size(dtype);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool cap = softcap > 0.0f;
  const bool fixed = fixed_lse_ok(softcap);
  const float inv_cap = cap ? 1.0f / softcap : 0.0f;
  int32_t n2 = 2;
  while (n2 < C) n2 <<= 1;
  const char* lg = static_cast<const char*>(logits);
  const dim3 grid(static_cast<uint32_t>(rows * plan.nsplit));
  // the same streaming shapes as cs_logsoftmax_gather (bit-identical lse)
#define CS_BEAM_LAUNCH(DTV, CAPV, FIXV)                                                           \
  do {                                                                                            \
    if (plan.nsplit > 1)                                                                          \
      hipLaunchKernelGGL((beam_step_kernel<DTV, CAPV, FIXV, 256, 8>), grid, dim3(256), 0, st, lg, \
                         vocab, ld_bytes, plan.nsplit, plan.split_len, A, B, K, targets,          \
                         rewards_in, softcap, inv_cap, welfare_kind, static_cast<double>(eps),    \
                         part, row_cnt, done_cnt, wkey, out_U, out_W, n_order, n2, out_order,     \
                         out_order_val, out_kept);                                                \
    else                                                                                          \
      hipLaunchKernelGGL((beam_step_kernel<DTV, CAPV, FIXV, 1024, 2>), grid, dim3(1024), 0, st,   \
                         lg, vocab, ld_bytes, plan.nsplit, plan.split_len, A, B, K, targets,      \
                         rewards_in, softcap, inv_cap, welfare_kind, static_cast<double>(eps),    \
                         part, row_cnt, done_cnt, wkey, out_U, out_W, n_order, n2, out_order,     \
                         out_order_val, out_kept);                                                \
  } while (0)
  if (dtype == CS_F32) {
    if (fixed) CS_BEAM_LAUNCH(CS_F32, true, true);
    else if (cap) CS_BEAM_LAUNCH(CS_F32, true, false);
    else CS_BEAM_LAUNCH(CS_F32, false, false);
  } else if (dtype == CS_BF16) {
    if (fixed) CS_BEAM_LAUNCH(CS_BF16, true, true);
    else if (cap) CS_BEAM_LAUNCH(CS_BF16, true, false);
    else CS_BEAM_LAUNCH(CS_BF16, false, false);
  } else {
    if (fixed) CS_BEAM_LAUNCH(CS_F16, true, true);
    else if (cap) CS_BEAM_LAUNCH(CS_F16, true, false);
    else CS_BEAM_LAUNCH(CS_F16, false, false);
  }
#undef CS_BEAM_LAUNCH
  if (n_order > 0 && n2 > kFusedSort)
    hipLaunchKernelGGL(topk_kernel, dim3(1), dim3(256), static_cast<size_t>(n2) * sizeof(unsigned long long),
                       st, out_W, static_cast<int32_t>(C), static_cast<int64_t>(C), n2, n_order,
                       out_order, out_order_val);
  return check_launch("cs_beam_step");
}

namespace {
// cs_beam_decode_step workspace: [cs_beam_step counters | proposer counters | beam
// counters][row lse][proposer chunk winners][split partials]
struct DecodeLayout {
  SplitPlan plan;
  int32_t block;
  int32_t kp;
  int32_t nchunk_p;
  size_t lse_off, ids_off, ppart_off, part_off, total;
};
DecodeLayout decode_layout(int32_t A, int32_t B, int64_t vocab, int32_t K, int dtype) {
  DecodeLayout d;
  const int64_t rows = static_cast<int64_t>(A) * B;
  d.plan = plan_split(rows, vocab, dtype);
  d.block = d.plan.nsplit > 1 ? 256 : 1024;
  d.kp = decode_kp(B, vocab, d.block, K);
  const int64_t ch = static_cast<int64_t>(d.kp) * d.block;
  d.nchunk_p = static_cast<int32_t>((vocab + ch - 1) / ch);
  d.lse_off = kBeamCounterBytes + 2 * sizeof(uint32_t) * kBeamMaxBeams;
  d.ids_off = d.lse_off + sizeof(uint32_t) * static_cast<size_t>(B) * pad_line(A, 4);
  d.ppart_off = d.ids_off + sizeof(uint32_t) * static_cast<size_t>(B) * pad_line(K, 4);
  d.part_off = d.ppart_off + sizeof(unsigned long long) * static_cast<size_t>(B) *
                                 pad_line(static_cast<int64_t>(d.nchunk_p) * K, 8);
  d.total = d.part_off + sizeof(unsigned long long) * static_cast<size_t>(rows) *
                             pad_line(d.plan.nsplit, 8);
  return d;
}
}  // namespace

size_t cs_beam_decode_workspace_size(int32_t A, int32_t B, int64_t vocab, int32_t K) {
  if (A <= 0 || B <= 0 || vocab <= 0 || K <= 0) return 0;
  const DecodeLayout p = decode_layout(A, B, vocab, K, CS_BF16);
  const DecodeLayout q = decode_layout(A, B, vocab, K, CS_F32);
  return p.total > q.total ? p.total : q.total;
}

int cs_beam_decode_step(const void* ref_logits, int64_t ld_ref, const void* logits, int64_t ld,
                        int dtype, int32_t A, int32_t B, int64_t vocab, int32_t K, float softcap,
                        const float* rewards_in, int welfare_kind, float eps, int32_t* out_ids,
                        float* out_U, float* out_W, int32_t n_order, int32_t* out_order,
                        float* out_order_val, float* out_kept, void* workspace,
                        size_t workspace_bytes, cs_stream_t stream) {
  const char* w = "cs_beam_decode_step: ";
  if (dtype != CS_F32 && dtype != CS_BF16 && dtype != CS_F16)
    return fail(CS_ERR_INVALID, std::string(w) + "unknown dtype");
  if (A <= 0 || B <= 0 || K <= 0 || vocab <= 0 || ld < vocab || ld_ref < vocab)
    return fail(CS_ERR_INVALID, std::string(w) + "need A, B, K > 0, vocab > 0, ld and ld_ref >= vocab");
  if (K > 256 || K > vocab) return fail(CS_ERR_INVALID, std::string(w) + "need K <= min(256, vocab)");
  const int64_t rows = static_cast<int64_t>(A) * B;
  const int64_t C = static_cast<int64_t>(B) * K;
  if (C > 16384) return fail(CS_ERR_INVALID, std::string(w) + "B*K exceeds 16384");
  if (rows > kBeamMaxRows || B > kBeamMaxBeams)
    return fail(CS_ERR_INVALID, std::string(w) + "A*B exceeds 65536 or B exceeds 4096");
  if (n_order < 0 || n_order > C) return fail(CS_ERR_INVALID, std::string(w) + "need 0 <= n_order <= B*K");
  if (out_kept && (n_order == 0 || C > kFusedSort))
    return fail(CS_ERR_INVALID, std::string(w) + "out_kept needs n_order > 0 and B*K <= 1024");
  if (welfare_kind < CS_WELFARE_MIN || welfare_kind > CS_WELFARE_MAX)
    return fail(CS_ERR_INVALID, std::string(w) + "unknown welfare kind");
  if (!(softcap >= 0.0f) || std::isinf(softcap))
    return fail(CS_ERR_INVALID, std::string(w) + "softcap must be finite and >= 0");
  if (!ref_logits || !logits || !rewards_in || !out_ids || !out_U || !out_W ||
      (n_order > 0 && !out_order))
    return fail(CS_ERR_INVALID, std::string(w) + "NULL pointer");
  if (reinterpret_cast<uintptr_t>(logits) % elt_size(dtype) != 0 ||
      reinterpret_cast<uintptr_t>(ref_logits) % elt_size(dtype) != 0)
    return fail(CS_ERR_INVALID, std::string(w) + "logits not element-aligned");
  const DecodeLayout d = decode_layout(A, B, vocab, K, dtype);
  if (static_cast<int64_t>(d.nchunk_p) * K > 16384)
    return fail(CS_ERR_INVALID, std::string(w) + "proposer chunks x K exceeds 16384");
  if (!workspace || workspace_bytes < d.total)
    return fail(CS_ERR_WORKSPACE, std::string(w) + "workspace smaller than cs_beam_decode_workspace_size()");
  if (reinterpret_cast<uintptr_t>(workspace) % 8 != 0)
    return fail(CS_ERR_WORKSPACE, std::string(w) + "workspace not 8-byte aligned");
  const int64_t grid = static_cast<int64_t>(B) * d.nchunk_p + rows * d.plan.nsplit;
  if (grid > 0x7fffffffLL) return fail(CS_ERR_INVALID, std::string(w) + "grid too large");
  char* wsb = static_cast<char*>(workspace);
  auto* done_cnt = reinterpret_cast<uint32_t*>(wsb);
  auto* row_cnt = reinterpret_cast<uint32_t*>(wsb + kBeamRowCntOff);
  auto* wkey = reinterpret_cast<uint32_t*>(wsb + kBeamKeyOff);
  auto* prop_cnt = reinterpret_cast<uint32_t*>(wsb + kBeamCounterBytes);
  auto* beam_cnt = prop_cnt + kBeamMaxBeams;
  auto* lse_ws = reinterpret_cast<uint32_t*>(wsb + d.lse_off);
  auto* ids_ws = reinterpret_cast<uint32_t*>(wsb + d.ids_off);
  auto* ppart = reinterpret_cast<unsigned long long*>(wsb + d.ppart_off);
  auto* part = reinterpret_cast<unsigned long long*>(wsb + d.part_off);
  const int64_t esz = elt_size(dtype);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool cap = softcap > 0.0f;
  const bool fixed = fixed_lse_ok(softcap);
  const float inv_cap = cap ? 1.0f / softcap : 0.0f;
  int32_t n2 = 2;
  while (n2 < C) n2 <<= 1;
  const char* rg = static_cast<const char*>(ref_logits);
  const char* lg = static_cast<const char*>(logits);
  const int32_t rows_first = decode_rows_first();
#define CS_DECODE_GO(DTV, CAPV, FIXV, BL, UN, KPV)                                                 \
  hipLaunchKernelGGL((beam_decode_kernel<DTV, CAPV, FIXV, BL, UN, KPV>), dim3(grid), dim3(BL), 0,  \
                     st, rg, ld_ref * esz, d.nchunk_p, rows_first, lg, vocab, ld * esz,            \
                     d.plan.nsplit, d.plan.split_len, A, B, K, rewards_in, softcap, inv_cap,       \
                     welfare_kind, static_cast<double>(eps), part, ppart, row_cnt, prop_cnt,       \
                     beam_cnt, done_cnt, wkey, lse_ws, ids_ws, out_ids, out_U, out_W, n_order, n2, \
                     out_order, out_order_val, out_kept)
#define CS_DECODE_LAUNCH(DTV, CAPV, FIXV)                                                          \
  do {                                                                                             \
    if (d.block == 256) {                                                                          \
      if (d.kp == 4) CS_DECODE_GO(DTV, CAPV, FIXV, 256, 8, 4);                                    \
      else CS_DECODE_GO(DTV, CAPV, FIXV, 256, 8, 16);                                             \
    } else {                                                                                       \
      if (d.kp == 4) CS_DECODE_GO(DTV, CAPV, FIXV, 1024, 2, 4);                                   \
      else CS_DECODE_GO(DTV, CAPV, FIXV, 1024, 2, 16);                                            \
    }                                                                                              \
  } while (0)
  if (dtype == CS_F32) {
    if (fixed) CS_DECODE_LAUNCH(CS_F32, true, true);
    else if (cap) CS_DECODE_LAUNCH(CS_F32, true, false);
    else CS_DECODE_LAUNCH(CS_F32, false, false);
  } else if (dtype == CS_BF16) {
    if (fixed) CS_DECODE_LAUNCH(CS_BF16, true, true);
    else if (cap) CS_DECODE_LAUNCH(CS_BF16, true, false);
    else CS_DECODE_LAUNCH(CS_BF16, false, false);
  } else {
    if (fixed) CS_DECODE_LAUNCH(CS_F16, true, true);
    else if (cap) CS_DECODE_LAUNCH(CS_F16, true, false);
    else CS_DECODE_LAUNCH(CS_F16, false, false);
  }
#undef CS_DECODE_LAUNCH
#undef CS_DECODE_GO
  if (n_order > 0 && n2 > kFusedSort)
    hipLaunchKernelGGL(topk_kernel, dim3(1), dim3(256), static_cast<size_t>(n2) * sizeof(unsigned long long),
                       st, out_W, static_cast<int32_t>(C), static_cast<int64_t>(C), n2, n_order,
                       out_order, out_order_val);
  return check_launch("cs_beam_decode_step");
}

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
