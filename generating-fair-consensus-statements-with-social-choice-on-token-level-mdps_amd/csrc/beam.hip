// beam.hip — whole beam-search scoring / decode steps in one launch.
#include "cs_kernels.cuh"

namespace {

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
// The hand-off primitives (st_sc1 / ld_sc1 / wait_stores / arrive) live in
// cs_kernels.cuh; tests/test_abi.py pins their sc1 lowering on this toolchain.
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

template <int BLOCK>
__device__ __forceinline__ void beam_order(const BeamLds& L, uint32_t* Uw, int32_t A, int32_t C,
                                           int32_t n_order, int32_t n2,
                                           int32_t* __restrict__ out_order,
                                           float* __restrict__ out_val,
                                           float* __restrict__ out_kept);

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
  beam_order<BLOCK>(L, Uw, A, C, n_order, n2, out_order, out_val, out_kept);
}

// The order of the C welfare values in L.sm_w (written by the calling block): the n_order
// best (radix-select threshold / wave bound + rank counting, or the full bitonic sort) by
// (W desc, index asc), NaN last, and the kept beams' rewards out_kept[a][r] = U[a][order[r]].
template <int BLOCK>
__device__ __forceinline__ void beam_order(const BeamLds& L, uint32_t* Uw, int32_t A, int32_t C,
                                           int32_t n_order, int32_t n2,
                                           int32_t* __restrict__ out_order,
                                           float* __restrict__ out_val,
                                           float* __restrict__ out_kept) {
  const int tid = threadIdx.x;
  unsigned long long* keys = L.keys;
  unsigned long long* keys2 = L.keys2;
  unsigned long long* sel_cand = L.sel_cand;
  float* sm_w = L.sm_w;
  int32_t* sm_ord = L.sm_ord;
  uint32_t* sm_tw = L.sm_tw;
  int* sm_res = L.sm_res;
  uint32_t& sm_n = *L.sm_n;
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
    auto emit = [&](int r, unsigned long long key) {
      const int32_t c = static_cast<int32_t>(0xffffffffu - static_cast<uint32_t>(key & 0xffffffffull));
      out_order[r] = c;
      if (out_val) out_val[r] = sm_w[c];
      sm_ord[r] = c;
    };
    if (BLOCK <= 256 && n_order <= kWaveBoundMaxK) {
      // few kept beams (256-thread blocks): the wave bound instead of histogram passes
      __syncthreads();   // sm_n = 0 is visible before any append
      uint32_t lm = 0u;
#pragma unroll
      for (int r = 0; r < kFusedSort / BLOCK; ++r)
        if (kc[r]) lm = max(lm, static_cast<uint32_t>(kc[r] >> 32));
      const uint32_t t = wave_bound<BLOCK>(lm, n_order, sm_tw);
#pragma unroll
      for (int r = 0; r < kFusedSort / BLOCK; ++r) {
        if (kc[r] && static_cast<uint32_t>(kc[r] >> 32) >= t) {
          const uint32_t at = atomicAdd(&sm_n, 1u);
          if (at < kTopkCand) cand[at] = kc[r];
        }
      }
      __syncthreads();
      const uint32_t nc = sm_n;
      if (nc <= static_cast<uint32_t>(kTopkCand)) {  // block-uniform
        rank_candidates<BLOCK>(cand, static_cast<int>(nc), n_order, emit);
        if (out_kept) {
          __syncthreads();
          keep_columns<BLOCK>(Uw, out_kept, sm_ord, A, C, n_order);
        }
        return;
      }
      __syncthreads();
      if (tid == 0) sm_n = 0u;
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
      rank_candidates<BLOCK>(cand, static_cast<int>(sm_n), n_order, emit);
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
  // one LDS pool: the bf16 soft-cap table while a row streams, the proposer's and the
  // tail's buffers otherwise (keys2 directly after keys: the selection path uses the pair
  // as one 16 KB histogram)
  constexpr bool TAB = CapTable<DT, CAP, FIXED>::kOn;
  constexpr int kPoolTail = 2 * kFusedSort + kTopkCand + kFusedSort;  // u64 words
  constexpr int kPool = TAB && kCapTab / 2 > kPoolTail ? kCapTab / 2 : kPoolTail;
  __shared__ __attribute__((aligned(16))) unsigned long long pool[kPool];
  unsigned long long* keys = pool;
  unsigned long long* keys2 = keys + kFusedSort;
  unsigned long long* sel_cand = pool + 2 * kFusedSort;
  float* sm_w = reinterpret_cast<float*>(sel_cand + kTopkCand);
  int32_t* sm_ord = reinterpret_cast<int32_t*>(sm_w + kFusedSort);
  float* ctab = reinterpret_cast<float*>(pool);
  __shared__ uint32_t sm_tw[2 * BLOCK / 64];
  __shared__ int sm_res[2];
  __shared__ uint32_t sm_n;
  const BeamLds L{keys, keys2, sel_cand, sm_w, sm_ord, sm_tw, sm_res, &sm_n};
  const int tid = threadIdx.x;
  const int32_t rows = A * B;
  const int32_t C = B * K;
  const int64_t item = blockIdx.x;
  const int32_t per_row = nsplit > 1 ? split_items(nsplit, BLOCK) : 1;
  const int32_t row = static_cast<int32_t>(item / per_row);
  const int32_t sitem = static_cast<int32_t>(item - static_cast<int64_t>(row) * per_row);
  const int32_t ag = row / B;
  const int32_t bm = row - ag * B;
  const char* rp = logits + row * ld_bytes;
  uint32_t* Uw = reinterpret_cast<uint32_t*>(U);
  const bool order_free = kind == CS_WELFARE_MIN || kind == CS_WELFARE_MAX;
  const bool is_min = kind == CS_WELFARE_MIN;
  // the candidate ids and their logits are read now (used only at the row finish), so
  // the finisher's gather costs no memory round trip after the lse is known
  const int32_t t_pre = (tid < K) ? tgt[bm * K + tid] : -1;
  const bool ok = t_pre >= 0 && t_pre < vocab;
  const float xg = ok ? load_one<DT>(rp, t_pre) : 0.0f;

  // 1. stream
  if constexpr (TAB) {
    build_cap_table<BLOCK>(ctab, cap, inv_cap);
    __syncthreads();
  }
  int32_t split = 0;
  bool valid = true;
  // split rows: the canonical split arithmetic (split_partial), BLOCK / 256 splits per block
  const float2 ms =
      nsplit > 1 ? split_partial<DT, CAP, FIXED, BLOCK, true>(rp, sitem, nsplit, split_len, vocab, cap,
                                                        inv_cap, sm_m, sm_s, ctab, split, valid)
                 : block_lse_partial<DT, CAP, FIXED, BLOCK, UNROLL, true>(rp, 0, vocab, cap, inv_cap,
                                                                    sm_m, sm_s, ctab);

  // 2. row finish by the row's last arriver
  if (nsplit > 1) {
    if (valid && tid % kSplitSub == 0) {
      st_sc1(part + static_cast<int64_t>(row) * pad_line(nsplit, 8) + split,
             (static_cast<unsigned long long>(__float_as_uint(ms.y)) << 32) |
                              __float_as_uint(ms.x));
      wait_stores();
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t nv = static_cast<uint32_t>(split_count(sitem, nsplit, BLOCK));
      sm_last = arrive(&row_cnt[row], nv) + nv == static_cast<uint32_t>(nsplit);
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

// wave-bound selection in the decode proposer (chunk and merge): every block shape
// (CS_WB_ALL=1) or the 256-thread blocks with K <= 16 only (CS_WB_ALL=0)
#ifndef CS_WB_ALL
#define CS_WB_ALL 0
#endif
#define CS_WB_ON(BL, KK) \
  (CS_WB_ALL ? wave_bound_ok<BL>(KK) : ((BL) <= 256 && (KK) <= kWaveBoundMaxK))
#ifndef CS_PROP_PRIO
#define CS_PROP_PRIO 2   // instruction-issue priority of the proposer waves
#endif
#ifndef CS_DECODE_KP1024
#define CS_DECODE_KP1024 8   // proposer keys per lane in the 1024-thread fp32 blocks (4 or this)
#endif
#ifndef CS_DECODE_RAWKEYS
#define CS_DECODE_RAWKEYS 1  // 16-bit logits: the proposer keeps the raw values, not 32-bit keys
#endif
#ifndef CS_DECODE_KP1024_RAW
#define CS_DECODE_KP1024_RAW 16   // proposer elements per lane then (1024-thread blocks)
#endif
// elements per lane of a 1024-thread proposer chunk: 16-bit logits are held raw (two per
// register) and their order keys recomputed on each pass, so twice the elements fit the
// registers of the 32-bit keys -- half the proposer workgroups, and C3's whole grid
// (256 agent rows + 16 beams x 16 chunks) is resident in one round on 256 CUs
constexpr int kp1024(int dtype) {
  return (CS_DECODE_RAWKEYS && dtype != CS_F32) ? CS_DECODE_KP1024_RAW : CS_DECODE_KP1024;
}
#ifndef CS_DECODE_UN1024
#define CS_DECODE_UN1024 2   // 16-byte vectors in flight per lane in the 1024-thread rows
#endif
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
// Proposer keys per lane: the largest of 16 (256-thread blocks) or 8 (1024-thread blocks;
// 16 would spill) that still gives >= 128 proposer workgroups, else 4 (few beams, e.g.
// C5's B = 8), so the proposer finishes under the agent-row stream (tools/beam_ab.py
// --sweep; profiles/r01f_beam_ab*.jsonl).  CS_DECODE_KP overrides (4, 8 or 16).
int decode_kp(int32_t B, int64_t vocab, int32_t block, int32_t K, int dtype) {
  const int big = block >= 1024 ? kp1024(dtype) : 16;
  static const int env_kp = [] {       // read once
    const char* e = getenv("CS_DECODE_KP");
    return e ? atoi(e) : 0;
  }();
  if (env_kp == 4 || env_kp == big) return env_kp;
  const int64_t nbig = B * ((vocab + big * block - 1) / (big * static_cast<int64_t>(block)));
  const int64_t n4c = (vocab + 4LL * block - 1) / (4LL * block);
  return (nbig < 128 && n4c * K <= 16384) ? 4 : big;
}
// Grid order: the agent-row blocks first when they leave workgroup slots free for the
// proposer (C3: 256 rows on 256 CUs x 2 slots), the proposer first when the rows alone
// fill the chip (C5: 512 rows) — then the rows would starve the proposer to the end.
// CS_DECODE_ROWS_FIRST=0/1 overrides.
int decode_rows_first(int64_t row_blocks, int32_t block) {
  static const int env_rf = [] {       // read once: -1 = not set
    const char* e = getenv("CS_DECODE_ROWS_FIRST");
    return e ? (atoi(e) == 1 ? 1 : 0) : -1;
  }();
  if (env_rf >= 0) return env_rf;
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n_cu = v;
    else
      n_cu = 256;
  }
  const int64_t slots = static_cast<int64_t>(n_cu) * (block >= 1024 ? 2 : 4);
  return row_blocks < slots ? 1 : 0;
}
#ifdef CS_TRACE_DECODE
// slots: 0 first block start (min), 1 last proposer chunk start, 2 last proposer chunk
// published, 3 last proposer merge done, 4 last row block start, 5 first row lse,
// 6 last row lse, 7 last beam gather done, 8 tail start, 9 tail end (wall_clock64 ticks)
__device__ unsigned long long g_dec_ts[16];
#define DEC_T(...) __VA_ARGS__
#else
#define DEC_T(...)
#endif
constexpr int kBeamMaxBeams = 4096;

template <int DT, bool CAP, bool FIXED, int BLOCK, int UNROLL, int KP>
__global__ __launch_bounds__(BLOCK, BLOCK >= 1024 ? 8 : 4) void beam_decode_kernel(
    const char* __restrict__ ref, int64_t ld_ref_bytes, int32_t nchunk_p, int32_t rows_first,
    int32_t ref_vec,
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
  // one LDS pool: the bf16 soft-cap table while a row streams, the proposer's and the
  // tail's buffers otherwise (keys2 directly after keys: the selection path uses the pair
  // as one 16 KB histogram)
  constexpr bool TAB = CapTable<DT, CAP, FIXED>::kOn;
  constexpr int kPoolTail = 2 * kFusedSort + kTopkCand + kFusedSort;  // u64 words
  constexpr int kPool = TAB && kCapTab / 2 > kPoolTail ? kCapTab / 2 : kPoolTail;
  __shared__ __attribute__((aligned(16))) unsigned long long pool[kPool];
  unsigned long long* keys = pool;
  unsigned long long* keys2 = keys + kFusedSort;
  unsigned long long* sel_cand = pool + 2 * kFusedSort;
  float* sm_w = reinterpret_cast<float*>(sel_cand + kTopkCand);
  int32_t* sm_ord = reinterpret_cast<int32_t*>(sm_w + kFusedSort);
  float* ctab = reinterpret_cast<float*>(pool);
  __shared__ uint32_t sm_tw[2 * BLOCK / 64];
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
  DEC_T(const unsigned long long q0 = wall_clock64(); if (tid == 0) atomicMin(&g_dec_ts[0], q0);)
  int32_t gb;  // the beam this block arrives at
  bool ids_in_lds = false;  // this block merged beam gb's proposer: its ids are in LDS

  const int32_t n_rowblk = static_cast<int32_t>(gridDim.x) - n_prop;
  // block role: proposer blocks first in the grid, or after the row blocks
  const int32_t pblk = rows_first ? static_cast<int32_t>(blockIdx.x) - n_rowblk
                                  : static_cast<int32_t>(blockIdx.x);
  const int32_t rblk = rows_first ? static_cast<int32_t>(blockIdx.x)
                                  : static_cast<int32_t>(blockIdx.x) - n_prop;
  if (pblk >= 0 && pblk < n_prop) {
    // ---- proposer chunk ----
    // the proposer's short latency chain goes first when it shares a CU with a streaming
    // row block (instruction issue priority; the stream is bandwidth-bound, not issue-bound)
    __builtin_amdgcn_s_setprio(CS_PROP_PRIO);
    DEC_T(if (tid == 0) atomicMax(&g_dec_ts[1], q0);)
    constexpr int CH = KP * BLOCK;
    const int32_t b = pblk / nchunk_p;
    const int32_t chunk = pblk - b * nchunk_p;
    const char* rp = ref + b * ld_ref_bytes;
    const int64_t v0 = static_cast<int64_t>(chunk) * CH;
    const int n = static_cast<int>(min(static_cast<int64_t>(CH), vocab - v0));
    // 32-bit order keys in registers (the token id is implied by (j, lane)): half the
    // registers of 64-bit composite keys, so the 1024-thread variant does not spill.  RAW
    // (16-bit logits): the raw values instead, two per register, each pass recomputing the
    // identical key order_key(softcap(x)) from them (a few VALU ops per element per pass)
    constexpr bool RAW = CS_DECODE_RAWKEYS && DT != CS_F32;
    constexpr int NWORD = RAW ? (KP + 1) / 2 : KP;
    uint32_t okey[NWORD];
    constexpr int EPV = Elt<DT>::kPerVec;
    constexpr int RG = KP < EPV ? KP : EPV;   // RAW: consecutive elements per lane group
    const bool vec = KP % EPV == 0 && ref_vec && n == CH;
    if (vec) {
      // whole 16-byte-aligned chunk: KP / EPV non-temporal 16-byte loads per lane, all in
      // flight at once (element (j / EPV * BLOCK + tid) * EPV + j % EPV in okey[j]; RAW: in
      // half j % 2 of word j / 2, the loaded vectors as they are)
      const u32x4* vp = reinterpret_cast<const u32x4*>(rp + v0 * Elt<DT>::kSize);
      u32x4 q[KP / EPV > 0 ? KP / EPV : 1];
#pragma unroll
      for (int j = 0; j < KP / EPV; ++j) q[j] = __builtin_nontemporal_load(vp + j * BLOCK + tid);
#pragma unroll
      for (int j = 0; j < KP / EPV; ++j) {
        if constexpr (RAW) {
#pragma unroll
          for (int e = 0; e < 4; ++e) okey[j * 4 + e] = q[j][e];
        } else {
          float v[EPV];
          unpack_vec<DT>(q[j], v);
#pragma unroll
          for (int e = 0; e < EPV; ++e)
            okey[j * EPV + e] = order_key(CAP ? softcap_fn(v[e], cap, inv_cap) : v[e]);
        }
      }
    } else {
      if constexpr (RAW) {
#pragma unroll
        for (int w = 0; w < NWORD; ++w) okey[w] = 0u;
      }
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        // RAW: the vector path's element order (one index formula for both paths; groups
        // of min(KP, EPV) consecutive elements per lane)
        const int i = RAW ? (j / RG * BLOCK + tid) * RG + j % RG : tid + BLOCK * j;
        if constexpr (RAW) {
          const uint32_t b = i < n ? reinterpret_cast<const uint16_t*>(rp)[v0 + i] : 0u;
          okey[j >> 1] |= b << ((j & 1) * 16);
        } else {
          float x = 0.0f;
          if (i < n) x = load_one<DT>(rp, v0 + i);
          okey[j] = order_key(CAP ? softcap_fn(x, cap, inv_cap) : x);
        }
      }
    }
    auto key32 = [&](int j) -> uint32_t {   // the order key of element j
      if constexpr (RAW) {
        const uint32_t b = (okey[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
        float x;
        if constexpr (DT == CS_BF16) x = __uint_as_float(b << 16);
        else x = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(b)));
        return order_key(CAP ? softcap_fn(x, cap, inv_cap) : x);
      } else {
        return okey[j];
      }
    };
    // RAW: before each pass over the keys the raw words are named as modified (an empty
    // asm), so the compiler recomputes the keys per pass instead of hoisting all KP of them
    // out of the radix loop into registers (which spills at 64 VGPRs)
    int lbase = tid * RG;    // RAW: element j of this lane is lbase + (j / RG) * BLOCK * RG + j % RG
    auto fresh = [&]() {
      if constexpr (RAW) {
#pragma unroll
        for (int w = 0; w < NWORD; ++w) asm volatile("" : "+v"(okey[w]));
        asm volatile("" : "+v"(lbase));   // nor the KP element indices
      }
    };
    auto local = [&](int j) -> int {   // element of okey[j] within the chunk
      if constexpr (RAW) return lbase + (j / RG) * (BLOCK * RG) + j % RG;
      return vec ? (j / EPV * BLOCK + tid) * EPV + j % EPV : tid + BLOCK * j;
    };
    auto key_of = [&](int j) -> unsigned long long {
      return (static_cast<unsigned long long>(key32(j)) << 32) |
             static_cast<unsigned long long>(0xffffffffu - static_cast<uint32_t>(v0 + local(j)));
    };
    if (tid == 0) sm_n = 0u;
    DEC_T(if (tid == 0) atomicMax(&g_dec_ts[10], wall_clock64());)
    bool have = false;   // candidates collected (block-uniform)
    // (256-thread variants only: in the 1024-thread ones the extra code's registers slow
    // the agent-row stream more than the bound saves; profiles/r01h_decode_wave_bound.jsonl)
    if (CS_WB_ON(BLOCK, K)) {
      uint32_t lm = 0u;
      fresh();
#pragma unroll
      for (int j = 0; j < KP; ++j)
        if (local(j) < n) lm = max(lm, key32(j));
      const uint32_t t = wave_bound<BLOCK>(lm, K, sm_tw);
      fresh();
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        if (local(j) < n && key32(j) >= t) {
          const uint32_t at = atomicAdd(&sm_n, 1u);
          if (at < kTopkCand) sel_cand[at] = key_of(j);
        }
      }
      __syncthreads();
      have = sm_n <= static_cast<uint32_t>(kTopkCand);
      if (!have) {   // massive ties at the bound: the radix path below
        __syncthreads();
        if (tid == 0) sm_n = 0u;
      }
    }
    if (!have) {
      const RadixCut cut = radix_select<BLOCK>(
          [&](auto f) {
            fresh();
#pragma unroll
            for (int j = 0; j < KP; ++j)
              if (local(j) < n) f(key_of(j));
          },
          static_cast<uint32_t>(K), static_cast<uint32_t>(2 * K + 64), hist, sm_tw, sm_res);
      fresh();
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        if (local(j) < n) {
          const unsigned long long kj = key_of(j);
          if ((kj >> cut.shift) >= cut.prefix) sel_cand[atomicAdd(&sm_n, 1u)] = kj;
        }
      }
      __syncthreads();
    }
    DEC_T(if (tid == 0) atomicMax(&g_dec_ts[11], wall_clock64());)
    const int32_t nkeys = nchunk_p * K;
    unsigned long long* pr = ppart + static_cast<int64_t>(b) * pad_line(nkeys, 8);
    unsigned long long* out = pr + static_cast<int64_t>(chunk) * K;
    const int nc = static_cast<int>(sm_n);
    rank_candidates<BLOCK>(sel_cand, nc, K, [&](int r, unsigned long long kc) { st_sc1(out + r, kc); });
    for (int r = nc + tid; r < K; r += BLOCK) st_sc1(out + r, 0ull);
    wait_stores();
    __syncthreads();
    DEC_T(if (tid == 0) { const unsigned long long q = wall_clock64(); atomicMax(&g_dec_ts[2], q);
                          atomicMin(&g_dec_ts[12], q); })
    if (tid == 0) {
      sm_last = arrive(&prop_cnt[b]) == static_cast<uint32_t>(nchunk_p - 1);
      sm_n = 0u;
    }
    __syncthreads();
    if (!sm_last) return;  // block-uniform
    if (tid == 0) st_sc1(prop_cnt + b, 0u);
    // the beam's K best among the chunk winners -> its candidate ids.  The winners are
    // read once (all loads in flight together) into registers when they fit, not again
    // per radix level and for the collection.
    constexpr int MR = 4;
    unsigned long long mk[MR];
    const bool cached = nkeys <= MR * BLOCK;
    if (cached) {
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const int i = tid + r * BLOCK;
        mk[r] = i < nkeys ? ld_sc1(pr + i) : 0ull;
      }
    }
    auto each_key = [&](auto f) {
      if (cached) {
#pragma unroll
        for (int r = 0; r < MR; ++r)
          if (mk[r]) f(mk[r]);
      } else {
        for (int i = tid; i < nkeys; i += BLOCK) {
          const unsigned long long c = ld_sc1(pr + i);
          if (c) f(c);
        }
      }
    };
    bool mhave = false;
    if (CS_WB_ON(BLOCK, K) && cached) {
      uint32_t lm = 0u;
#pragma unroll
      for (int r = 0; r < MR; ++r) lm = max(lm, static_cast<uint32_t>(mk[r] >> 32));
      const uint32_t t = wave_bound<BLOCK>(lm, K, sm_tw);
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        if (mk[r] && static_cast<uint32_t>(mk[r] >> 32) >= t) {
          const uint32_t at = atomicAdd(&sm_n, 1u);
          if (at < kTopkCand) sel_cand[at] = mk[r];
        }
      }
      __syncthreads();
      mhave = sm_n <= static_cast<uint32_t>(kTopkCand);
      if (!mhave) {
        __syncthreads();
        if (tid == 0) sm_n = 0u;
      }
    }
    if (!mhave) {
      const RadixCut mcut = radix_select<BLOCK>(
          each_key, static_cast<uint32_t>(K), static_cast<uint32_t>(2 * K + 64), hist, sm_tw, sm_res);
      each_key([&](unsigned long long c) {
        if ((c >> mcut.shift) >= mcut.prefix) sel_cand[atomicAdd(&sm_n, 1u)] = c;
      });
      __syncthreads();
    }
    const int mc = static_cast<int>(sm_n);
    // the ids also stay in LDS: when this block gathers the beam it reads them there
    uint32_t* sm_ids = reinterpret_cast<uint32_t*>(sm_ord);
    rank_candidates<BLOCK>(sel_cand, mc, K, [&](int r, unsigned long long c) {
      const uint32_t id = 0xffffffffu - static_cast<uint32_t>(c & 0xffffffffull);
      st_sc1(ids_ws + b * pad_line(K, 4) + r, id);
      sm_ids[r] = id;
      out_ids[b * K + r] = static_cast<int32_t>(id);
    });
    for (int r = mc + tid; r < K; r += BLOCK) {
      st_sc1(ids_ws + b * pad_line(K, 4) + r, 0xffffffffu);
      sm_ids[r] = 0xffffffffu;
      out_ids[b * K + r] = -1;
    }
    ids_in_lds = true;
    DEC_T(if (tid == 0) atomicMax(&g_dec_ts[3], wall_clock64());)
    gb = b;
  } else {
    // ---- agent row stream ----
    const int64_t item = rblk;
    const int32_t per_row = nsplit > 1 ? split_items(nsplit, BLOCK) : 1;
    const int32_t row = static_cast<int32_t>(item / per_row);
    const int32_t sitem = static_cast<int32_t>(item - static_cast<int64_t>(row) * per_row);
    const char* rp = logits + row * ld_bytes;
    if constexpr (TAB) {
      build_cap_table<BLOCK>(ctab, cap, inv_cap);
      __syncthreads();
    }
    int32_t split = 0;
    bool valid = true;
    // split rows: the canonical split arithmetic of cs_logsoftmax_gather / cs_beam_step
    // (split_partial), so a 1024-thread launch (proposer chunks of 16 * 1024 elements) takes
    // split rows four splits per block with the same bits as 256-thread splits
    const float2 ms =
        nsplit > 1 ? split_partial<DT, CAP, FIXED, BLOCK, true>(rp, sitem, nsplit, split_len, vocab, cap,
                                                          inv_cap, sm_m, sm_s, ctab, split, valid)
                   : block_lse_partial<DT, CAP, FIXED, BLOCK, UNROLL, true>(rp, 0, vocab, cap, inv_cap,
                                                                      sm_m, sm_s, ctab);
    if (nsplit > 1) {
      if (valid && tid % kSplitSub == 0) {
        st_sc1(part + static_cast<int64_t>(row) * pad_line(nsplit, 8) + split,
               (static_cast<unsigned long long>(__float_as_uint(ms.y)) << 32) |
                                __float_as_uint(ms.x));
        wait_stores();
      }
      __syncthreads();
      if (tid == 0) {
        const uint32_t nv = static_cast<uint32_t>(split_count(sitem, nsplit, BLOCK));
        sm_last = arrive(&row_cnt[row], nv) + nv == static_cast<uint32_t>(nsplit);
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
    DEC_T(if (tid == 0) { const unsigned long long q = wall_clock64(); atomicMax(&g_dec_ts[4], q0);
                          atomicMin(&g_dec_ts[5], q); atomicMax(&g_dec_ts[6], q); })
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
    const int32_t t = static_cast<int32_t>(ids_in_lds ? reinterpret_cast<const uint32_t*>(sm_ord)[j]
                                                      : ld_sc1(ids_ws + gb * pad_line(K, 4) + j));
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
  DEC_T(if (tid == 0) atomicMax(&g_dec_ts[7], wall_clock64());)
  if (tid == 0) sm_last = arrive(done_cnt) == static_cast<uint32_t>(B - 1);
  __syncthreads();
  if (!sm_last) return;  // block-uniform
  if (tid == 0) st_sc1(done_cnt, 0u);
  DEC_T(if (tid == 0) g_dec_ts[8] = wall_clock64();)
  beam_tail<BLOCK>(L, Uw, wkey, W, A, C, kind, eps, n_order, n2, out_order, out_val, out_kept);
  DEC_T(if (tid == 0) g_dec_ts[9] = wall_clock64();)
}

}  // namespace

namespace {
// cs_beam_select: one workgroup orders C <= kFusedSort welfare values and keeps the
// rewards of the n_order best columns (beam_order), after the agent-sharded all-reduce.
constexpr int kSelectBlock = 256;
__global__ __launch_bounds__(kSelectBlock) void beam_select_kernel(
    const float* __restrict__ Win, int32_t C, int unfill, uint32_t* __restrict__ Uw, int32_t A,
    float* __restrict__ W_out, int32_t n_order, int32_t n2, int32_t* __restrict__ out_order,
    float* __restrict__ out_val, float* __restrict__ out_kept) {
  __shared__ __attribute__((aligned(16))) unsigned long long pool[2 * kFusedSort + kTopkCand + kFusedSort];
  __shared__ uint32_t sm_tw[2 * kSelectBlock / 64];
  __shared__ int sm_res[2];
  __shared__ uint32_t sm_n;
  unsigned long long* sel_cand = pool + 2 * kFusedSort;
  float* sm_w = reinterpret_cast<float*>(sel_cand + kTopkCand);
  int32_t* sm_ord = reinterpret_cast<int32_t*>(sm_w + kFusedSort);
  const BeamLds L{pool, pool + kFusedSort, sel_cand, sm_w, sm_ord, sm_tw, sm_res, &sm_n};
  for (int32_t c = threadIdx.x; c < C; c += kSelectBlock) {
    float w = Win[c];
    if ((unfill == CS_UNFILL_POSINF && w == INFINITY) || (unfill == CS_UNFILL_NEGINF && w == -INFINITY))
      w = __builtin_nanf("");
    sm_w[c] = w;
    if (W_out) W_out[c] = w;
  }
  beam_order<kSelectBlock>(L, Uw, A, C, n_order, n2, out_order, out_val, out_kept);
}
}  // namespace

extern "C" {

int cs_beam_select(const float* W, int32_t C, int unfill, const float* U, int32_t A,
                   int32_t n_order, float* out_W, int32_t* out_order, float* out_order_val,
                   float* out_kept, cs_stream_t stream) {
  const char* w = "cs_beam_select: ";
  if (C <= 0 || C > kFusedSort) return fail(CS_ERR_INVALID, std::string(w) + "need 0 < C <= 1024");
  if (n_order <= 0 || n_order > C) return fail(CS_ERR_INVALID, std::string(w) + "need 0 < n_order <= C");
  if (unfill != CS_UNFILL_NONE && unfill != CS_UNFILL_POSINF && unfill != CS_UNFILL_NEGINF)
    return fail(CS_ERR_INVALID, std::string(w) + "unknown unfill mode");
  if (A < 0) return fail(CS_ERR_INVALID, std::string(w) + "need A >= 0");
  if (!W || !out_order || (out_kept && A > 0 && !U))
    return fail(CS_ERR_INVALID, std::string(w) + "NULL pointer");
  int32_t n2 = 2;
  while (n2 < C) n2 <<= 1;
  hipLaunchKernelGGL(beam_select_kernel, dim3(1), dim3(kSelectBlock), 0,
                     static_cast<hipStream_t>(stream), W, C, unfill,
                     reinterpret_cast<uint32_t*>(const_cast<float*>(U)), out_kept ? A : 0, out_W,
                     n_order, n2, out_order, out_order_val, out_kept);
  return check_launch("cs_beam_select");
}

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
  // the same streaming arithmetic as cs_logsoftmax_gather (bit-identical lse): unsplit rows
  // one 1024-thread block x 2 vectors per lane, split rows the canonical split form
  // (split_partial), four splits per 1024-thread block
  const dim3 grid(static_cast<uint32_t>(rows * (plan.nsplit > 1 ? split_items(plan.nsplit, 1024) : 1)));
#define CS_BEAM_LAUNCH(DTV, CAPV, FIXV)                                                           \
  hipLaunchKernelGGL((beam_step_kernel<DTV, CAPV, FIXV, 1024, 2>), grid, dim3(1024), 0, st, lg,     \
                     vocab, ld_bytes, plan.nsplit, plan.split_len, A, B, K, targets, rewards_in,  \
                     softcap, inv_cap, welfare_kind, static_cast<double>(eps), part, row_cnt,     \
                     done_cnt, wkey, out_U, out_W, n_order, n2, out_order, out_order_val, out_kept)
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
  // 1024-thread blocks: split rows take four canonical splits per block (split_partial), so
  // the proposer keeps its 16 * 1024-element chunks (per-rank C3: 43.98 -> 26.4 us,
  // profiles/r05e_beam_ab_*.jsonl).  256-thread blocks (one split each, wave-bound proposer
  // selection for K <= 16) measured slower at C1 too: 17.8 vs 16.9 us (r05f_beam_ab.jsonl)
  d.block = 1024;
  static const int env_block = [] {    // A/B: 256 or 1024 whatever the split (read once)
    const char* e = getenv("CS_DECODE_BLOCK");
    return e ? atoi(e) : 0;
  }();
  if (env_block == 256 || env_block == 1024) d.block = env_block;
  d.kp = decode_kp(B, vocab, d.block, K, dtype);
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

#ifdef CS_TRACE_DECODE
// diagnostics build only: copy the phase timestamps of the last launch and reset them
int cs_trace_read(unsigned long long* out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dec_ts), sizeof(g_dec_ts));
  unsigned long long init[16];
  for (int i = 0; i < 16; ++i) init[i] = (i == 0 || i == 5 || i == 12) ? ~0ull : 0ull;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dec_ts), init, sizeof(init));
  return 0;
}
#endif

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
  const int64_t row_blocks = rows * (d.plan.nsplit > 1 ? split_items(d.plan.nsplit, d.block) : 1);
  const int64_t grid = static_cast<int64_t>(B) * d.nchunk_p + row_blocks;
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
  const int32_t rows_first = decode_rows_first(row_blocks, d.block);
  // 16-byte vector loads in the proposer when every reference row starts 16-B aligned
  const int32_t ref_vec = (reinterpret_cast<uintptr_t>(ref_logits) % 16 == 0 &&
                           (ld_ref * esz) % 16 == 0) ? 1 : 0;
#define CS_DECODE_GO(DTV, CAPV, FIXV, BL, UN, KPV)                                                 \
  hipLaunchKernelGGL((beam_decode_kernel<DTV, CAPV, FIXV, BL, UN, KPV>), dim3(grid), dim3(BL), 0,  \
                     st, rg, ld_ref * esz, d.nchunk_p, rows_first, ref_vec, lg, vocab, ld * esz,   \
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
      if (d.kp == 4) CS_DECODE_GO(DTV, CAPV, FIXV, 1024, CS_DECODE_UN1024, 4);                    \
      else CS_DECODE_GO(DTV, CAPV, FIXV, 1024, CS_DECODE_UN1024, kp1024(DTV));                   \
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

}  // extern "C"
