// cs_kernels.cuh — shared device / host helpers of the gfx950 library behind
// include/consensus_scoring.h (included by every csrc/*.hip translation unit).
//
// What the reference does (serially, remotely): for every (agent, candidate) it asks a
// hosted LLM for prompt log-probs (src/utils.py:201-281), folds them into a per-agent
// utility (src/methods/*.py) and reduces across agents with min / sum / sum-of-log
// (src/methods/beam_search.py:558, src/methods/best_of_n.py:401-408,
// src/evaluation.py:337-381, core.py:108-113).  Here the same arithmetic runs on the
// logits rows the local forward produced.  Translation units:
//
//   stream.hip    lsg_stream_kernel (HBM-bound vocab stream: online max / sum-exp,
//                 16-byte non-temporal loads, wave64 butterfly + LDS merge) and the
//                 split-V lsg_merge_kernel -> cs_logsoftmax_gather
//   fold.hip      seg_reduce_kernel, welfare_kernel -> cs_segment_reduce,
//                 cs_welfare_reduce, cs_segmented_topk (topk_kernel lives here)
//   proposer.hip  vocab top-k (radix select) and seeded Gumbel-max sampling
//   beam.hip      cs_beam_step / cs_beam_decode_step: whole beam decode steps in one
//                 launch (last-arriver hand-offs, atomic welfare keys, radix select)
//
// No float atomics anywhere: every output is bitwise reproducible run to run.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "consensus_scoring.h"

// the thread's last error message, shared by every translation unit (cs_last_error)
inline thread_local std::string cs_g_last_error;

namespace {

constexpr int kBlock = 256;   // streaming workgroup: 4 waves of 64
constexpr int kUnroll = 4;    // 16-byte vectors in flight per lane per iteration
constexpr int kMergeBlock = 64;
// split-V below this many workgroups: one 1024-thread workgroup per row already streams at
// the launch's floor once rows >= 256 (tools/split_sweep.py; profiles/r01_split_sweep.jsonl)
constexpr int64_t kTargetWgs = 256;
constexpr float kLog2e = 1.4426950408889634f;

inline int fail(int code, const std::string& msg) {
  cs_g_last_error = msg;
  return code;
}

inline int check_launch(const char* what) {
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

// bf16 soft-cap table.  A bf16 logit takes 2^16 values, so exp(cap * tanh(x / cap)) --
// three transcendentals per element in the fixed-offset sum (softcap_exp) -- becomes one
// LDS lookup.  Only magnitude bits in [kCapLo, kCapHi] need entries of their own: below
// 2^-24 the value is that of x = 0 (exp2 of |arg| < 6e-9 rounds to 1), from 512 up it is
// saturated (x' = +-cap exactly in fp32).  Every entry is softcap_exp of its exact bf16
// value, so the sums are the transcendental path's sums.  NaN (magnitude > 0x7f80) is
// tracked beside the sum, since the clamp would map it to the saturated entry.
constexpr uint32_t kCapLo = 102u << 7;
constexpr uint32_t kCapHi = (136u << 7) | 127u;
constexpr int kCapSpan = static_cast<int>(kCapHi - kCapLo + 1);  // 4480 entries per sign
constexpr int kCapTab = 2 * kCapSpan;                             // 35,840 B of LDS

template <int DT, bool CAP, bool FIXED>
struct CapTable {
  static constexpr bool kOn = DT == CS_BF16 && CAP && FIXED;
};

template <int BLOCK>
__device__ __forceinline__ void build_cap_table(float* tab, float cap, float inv_cap) {
  for (int i = threadIdx.x; i < kCapTab; i += BLOCK) {
    const uint32_t neg = i >= kCapSpan ? 1u : 0u;
    const uint32_t c = static_cast<uint32_t>(i) - neg * kCapSpan;
    const uint32_t u = c < 128u ? 0u : kCapLo + c;  // the lowest bin stands for +-0
    tab[i] = softcap_exp(__uint_as_float(((neg << 15) | u) << 16), cap, inv_cap);
  }
}

// exp(softcap(x)) of one bf16 bit pattern b (low 16 bits of the argument)
__device__ __forceinline__ float cap_lookup(const float* tab, uint32_t u, uint32_t neg,
                                            uint32_t& nanmax) {
  nanmax = max(nanmax, u);
  const uint32_t c = min(max(u, kCapLo), kCapHi) - kCapLo;
  return tab[c + neg * kCapSpan];
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

// NQ 16-byte vectors of bf16 through the soft-cap table.  All 8 * NQ lookups are issued
// before the first add, and the sum is a fixed tree (four chains, element e in chain
// e % 4), so the LDS latency is paid once per batch, not once per element.  Every kernel
// sums through this one function, so their results stay bit-identical to each other.
template <int NQ>
__device__ __forceinline__ void cap_accum(float& s, uint32_t& nanmax, const u32x4* q,
                                          const float* __restrict__ tab) {
  float t[8 * NQ];
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t w = q[u][i];
      t[u * 8 + 2 * i] = cap_lookup(tab, w & 0x7fffu, (w >> 15) & 1u, nanmax);
      t[u * 8 + 2 * i + 1] = cap_lookup(tab, (w >> 16) & 0x7fffu, w >> 31, nanmax);
    }
  }
  float a[4] = {t[0], t[1], t[2], t[3]};
#pragma unroll
  for (int e = 4; e < 8 * NQ; ++e) a[e & 3] += t[e];
  s += (a[0] + a[1]) + (a[2] + a[3]);
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
// tid_in >= 0: the caller runs several BLOCK-thread sub-blocks side by side in one larger
// workgroup (tid_in = thread index within the sub-block, sm_m / sm_s the sub-block's NW
// slots; every sub-block reaches the workgroup barrier inside, so they run in lockstep).
template <int DT, bool CAP, bool FIXED, int BLOCK, int UNROLL, bool PIPE = false>
__device__ __forceinline__ float2 block_lse_partial(const char* __restrict__ rp, int64_t v0,
                                                    int64_t n, float cap, float inv_cap,
                                                    float* sm_m, float* sm_s,
                                                    const float* __restrict__ ctab = nullptr,
                                                    int tid_in = -1) {
  constexpr int ESZ = Elt<DT>::kSize;
  constexpr int EPV = Elt<DT>::kPerVec;
  constexpr int NW = BLOCK / 64;
  constexpr bool TAB = CapTable<DT, CAP, FIXED>::kOn;
  const int tid = tid_in >= 0 ? tid_in : static_cast<int>(threadIdx.x);
  float m = FIXED ? 0.0f : -INFINITY, s = 0.0f;
  uint32_t nanmax = 0u;

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
      if constexpr (TAB) {
        const uint32_t b = __float_as_uint(x) >> 16;
        s += cap_lookup(ctab, b & 0x7fffu, b >> 15, nanmax);
      } else if constexpr (CAP && FIXED) {
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
  auto consume = [&](u32x4* q) {
    if constexpr (TAB) {
      cap_accum<UNROLL>(s, nanmax, q, ctab);
    } else {
      float v[UNROLL * EPV];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) unpack_vec<DT>(q[u], v + u * EPV);
      accum_elems<UNROLL * EPV, CAP, FIXED>(m, s, v, cap, inv_cap);
    }
  };
  // PIPE (the beam kernels' soft-capped bf16 rows: the LDS exp-table path, <= 2 vectors
  // per lane): software-pipelined, the next UNROLL vectors issued before this batch is
  // consumed, so a wave keeps its loads in flight through its table lookups and the
  // proposer / tail work beside it (same elements, same order: bit-identical to the plain
  // loop).  The C3 decode launch 42.7 -> 40.0 us, the C3 cs_beam_step 33.9 -> 31.7 us;
  // measured slower in cs_logsoftmax_gather's own launches (C3 split rows 28.0 -> 33.5 us,
  // C2's plain rows 2.725 -> 2.75 ms) and past 2 vectors (VGPRs cost occupancy), so those
  // keep the plain loop (profiles/r06_ab_lsg.jsonl, r06_ab_beam.jsonl, r06b_beam_ab.jsonl)
  if (PIPE && TAB && UNROLL <= 2 && i + (UNROLL - 1) * BLOCK < nvec) {
    u32x4 q[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) q[u] = __builtin_nontemporal_load(vp + i + u * BLOCK);
    for (i += STEP; i + (UNROLL - 1) * BLOCK < nvec; i += STEP) {
      u32x4 nx[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) nx[u] = __builtin_nontemporal_load(vp + i + u * BLOCK);
      consume(q);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) q[u] = nx[u];
    }
    consume(q);
  } else {
    for (; i + (UNROLL - 1) * BLOCK < nvec; i += STEP) {
      u32x4 q[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) q[u] = __builtin_nontemporal_load(vp + i + u * BLOCK);
      consume(q);
    }
  }
  for (; i < nvec; i += BLOCK) {
    const u32x4 q = __builtin_nontemporal_load(vp + i);
    if constexpr (TAB) {
      cap_accum<1>(s, nanmax, &q, ctab);
    } else {
      float v[EPV];
      unpack_vec<DT>(q, v);
      accum_elems<EPV, CAP, FIXED>(m, s, v, cap, inv_cap);
    }
  }
  if (TAB && nanmax > 0x7f80u) s = __builtin_nanf("");

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

// Split rows (plan_split: nsplit > 1), ONE arithmetic for every kernel that splits a row's
// vocabulary (cs_logsoftmax_gather, cs_beam_step, cs_beam_decode_step), so their row lse are
// bit-identical whatever workgroup shape streams the row: split j covers
// [j * split_len, min(vocab, (j + 1) * split_len)) and its (m, s) is block_lse_partial over a
// kSplitSub-thread sub-block with kSplitUnroll vectors in flight per lane; the partials are
// merged in split order by one wave (split_merge).  A 256-thread workgroup streams one split,
// a 1024-thread workgroup kSplitQuad consecutive splits side by side (quarter q of quad item
// i: split kSplitQuad * i + q) -- the decode kernel's 1024-thread proposer chunks then share
// a launch with split rows (tools/beam_ab.py; DESIGN.md "The beam decode launch (round 5)").
constexpr int kSplitSub = 256;
constexpr int kSplitUnroll = 2;
constexpr int kSplitQuad = 4;
__host__ __device__ constexpr int32_t split_items(int32_t nsplit, int block) {
  return block >= kSplitSub * kSplitQuad ? (nsplit + kSplitQuad - 1) / kSplitQuad : nsplit;
}

// this thread's split of the row's work item `item` (0 <= item < split_items) and the
// split's (m, s), valid in the sub-block's thread 0 when `valid`
template <int DT, bool CAP, bool FIXED, int BLOCK, bool PIPE = false>
__device__ __forceinline__ float2 split_partial(const char* __restrict__ rp, int32_t item,
                                               int32_t nsplit, int64_t split_len, int64_t vocab,
                                               float cap, float inv_cap, float* sm_m, float* sm_s,
                                               const float* __restrict__ ctab, int32_t& split,
                                               bool& valid) {
  static_assert(BLOCK == kSplitSub || BLOCK == kSplitSub * kSplitQuad, "split sub-blocks");
  constexpr int SUBS = BLOCK / kSplitSub;
  const int q = SUBS > 1 ? static_cast<int>(threadIdx.x) / kSplitSub : 0;
  split = item * SUBS + q;
  valid = split < nsplit;
  const int64_t v0 = valid ? static_cast<int64_t>(split) * split_len : 0;
  const int64_t n = valid ? min(vocab, v0 + split_len) - v0 : 0;
  constexpr int NWS = kSplitSub / 64;
  return block_lse_partial<DT, CAP, FIXED, kSplitSub, kSplitUnroll, PIPE>(
      rp, v0, n, cap, inv_cap, sm_m + q * NWS, sm_s + q * NWS, ctab,
      static_cast<int>(threadIdx.x) % kSplitSub);
}

// the row's splits [0, nsplit) this work item holds (the arrival count it adds)
__device__ __forceinline__ int32_t split_count(int32_t item, int32_t nsplit, int block) {
  const int subs = block >= kSplitSub * kSplitQuad ? kSplitQuad : 1;
  const int32_t left = nsplit - item * subs;
  return left < subs ? left : subs;
}

// The fixed-offset sum is exact enough and cannot overflow for |x'| <= 60:
// e^60 * 2^31 < FLT_MAX and e^-60 is a normal float.
inline bool fixed_lse_ok(float cap) { return cap > 0.0f && cap <= 60.0f; }

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
inline int elt_size(int dtype) { return dtype == CS_F32 ? 4 : 2; }
inline int elt_per_vec(int dtype) { return dtype == CS_F32 ? 4 : 8; }

struct SplitPlan {
  int32_t nsplit;
  int64_t split_len;
};

inline int64_t target_wgs() {
  // tuning knob (tools/beam_ab.py, split_sweep.py), read once per translation unit
  static const int64_t v = [] {
    const char* e = getenv("CS_TARGET_WGS");
    const int64_t x = e ? atoll(e) : 0;
    return x > 0 ? x : kTargetWgs;
  }();
  return v;
}

// Fewer rows than target_wgs(): split the vocabulary so that about target_wgs() x
// kSplitQuad 256-thread split sub-blocks (target_wgs() 1024-thread workgroups of four) stream
// the rows -- each 1024-thread workgroup of the split kernels then has as many bytes in flight
// as a whole unsplit row's workgroup.
inline SplitPlan plan_split(int64_t rows, int64_t vocab, int dtype) {
  SplitPlan p{1, vocab};
  const int64_t target = target_wgs();
  if (rows <= 0 || vocab <= 0 || rows >= target) return p;
  const int64_t grain = static_cast<int64_t>(kBlock) * elt_per_vec(dtype);  // one vector per lane
  const int64_t min_len = grain * kUnroll;  // >= one full unrolled sweep per split
  int64_t want = (target * kSplitQuad + rows - 1) / rows;
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

// Lower bound on the k-th largest of a block's 32-bit order keys: each lane passes its
// largest key and every wave sorts those 64 (a wave64 bitonic sort in registers).  Two
// bounds come out of that sort, both valid, and the larger is returned:
//   * (k <= 64) the largest over the waves of each wave's k-th largest lane maximum: at
//     least k keys of that wave are >= it;
//   * the smallest over the NW = BLOCK / 64 waves of each wave's ceil(k / NW)-th largest
//     lane maximum: every wave holds ceil(k / NW) keys >= it, NW * ceil(k / NW) >= k.
// The first is tight for small k, the second for k of tens to hundreds spread over many
// waves (a C3 proposer chunk, k = 50 of 8,192 keys in 16 waves, passes ~100 keys).  Every
// key among the block's k largest is >= the bound, so collecting those and rank-counting
// replaces the histogram passes of radix_select (no LDS atomics on hot bins, two
// barriers).  sm_t holds 2 * BLOCK / 64 words.  Returns 0 (every key passes) when a wave
// has too few keys.
template <int BLOCK>
__device__ __forceinline__ uint32_t wave_bound(uint32_t lane_max, int k, uint32_t* sm_t) {
  constexpr int NW = BLOCK / 64;
  const int lane = threadIdx.x & 63;
  uint32_t v = lane_max;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint32_t o = __shfl_xor(v, stride, 64);
      const bool keep_max = ((lane & stride) == 0) == ((lane & size) == 0);
      v = keep_max ? max(v, o) : min(v, o);
    }
  }
  const uint32_t t1 = k <= 64 ? __shfl(v, k - 1, 64) : 0u;
  const uint32_t t2 = __shfl(v, (k + NW - 1) / NW - 1, 64);
  if (lane == 0) {
    sm_t[threadIdx.x >> 6] = t1;
    sm_t[NW + (threadIdx.x >> 6)] = t2;
  }
  __syncthreads();
  uint32_t b1 = 0u, b2 = 0xffffffffu;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    b1 = max(b1, sm_t[w]);
    b2 = min(b2, sm_t[NW + w]);
  }
  return max(b1, b2);
}
// the bound needs ceil(k / NW) <= 64
template <int BLOCK>
__host__ __device__ constexpr bool wave_bound_ok(int k) { return k <= 64 * (BLOCK / 64); }
constexpr int kWaveBoundMaxK = 16;   // larger k: radix_select (the bound passes too many)

// ---------------------------------------------------------------------------
// cross-workgroup hand-offs (beam.hip)
// ---------------------------------------------------------------------------
// Cross-workgroup hand-off without fences (MI355X_MICROARCH.md, hand-off table row 1):
// every handed-off byte is stored and loaded with sc1 (agent-scope relaxed atomics lower
// to global_store/global_load ... sc1: write-through past the L2, L1 bypassed), every
// storing wave waits vmcnt(0), the workgroup barriers, and ONE lane then adds to the
// arrival counter; the workgroup whose add returns the last count consumes.
// Memory-model note: these are RELAXED agent-scope atomics, not release / acquire.  What
// orders the hand-off is the gfx950 ISA behaviour of the sc1 forms (a store completes,
// s_waitcnt vmcnt(0), only once it is past the per-XCD L2; an sc1 load bypasses the L1 and
// reads past the L2), which the HIP memory model does not promise: an agent-scope release
// here would write back the whole L2 (buffer_wbl2) per arrival, tens of microseconds per
// step.  The assumption is pinned by tests/test_kernels_gpu.py (the fused launches against
// the unfused kernels word for word: the fuzz, and the shared-workspace stress of
// alternating shapes on a busy device and of hipGraph replays), and a failed launch
// re-zeroes the counters (ops.Workspace.reset).  tests/test_abi.py compiles these helpers
// with the library's flags and checks the disassembly: the store and the load must carry
// sc1 (a toolchain that lowered them otherwise would fail there, not silently on a GPU).
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
__device__ __forceinline__ uint32_t arrive(uint32_t* cnt, uint32_t n = 1u) {
  return __hip_atomic_fetch_add(cnt, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace
