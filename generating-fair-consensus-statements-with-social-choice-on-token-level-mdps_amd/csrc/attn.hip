// attn.hip — the transformer side of the batched agent x candidate decode:
//
//   prefix_attn_kernel   cascade attention over SHARED per-agent prefix K/V.  Every
//                        candidate stream of an agent (a beam, a Best-of-N candidate) reads
//                        its agent's prefix keys through one workgroup that holds ALL of
//                        that agent's query rows of one K/V head, so a prefix key block is
//                        fetched from HBM once per (agent, head), not once per stream (the
//                        reference re-encodes the whole ~150-800-token prompt per call:
//                        src/utils.py:249-259, driven per candidate at
//                        src/methods/beam_search.py:495-538, best_of_n.py:266-321).  Each
//                        stream's own tokens (history + causal self) live in a per-stream
//                        buffer and are attended in the same pass.  bf16 MFMA
//                        (v_mfma_f32_16x16x32_bf16), fp32 online softmax.
//   attn_merge_kernel    fixed-order merge of the key splits (no float atomics).
//   rope_place_kernel    RoPE on the fused q|k|v projection + placement of the new K (row
//                        layout) and V (transposed layout) into the per-stream buffers;
//                        positions come from device memory (prefix length + history base),
//                        so a captured decode step replays with no host input but ids.
//
// Layouts (all bf16, D = head_dim in {64, 128, 256}):
//   q       [n_tok, H, D], token tok = s*T + t of stream s = grp*n_str + b
//   k_pfx   [Hkv, Lp, D]                vt_pfx [Hkv, Lp/32, D, 32] (ragged prefixes: prefix p's
//           keys are rows off[p] .. off[p] + len[p], off[p] % 32 == 0, padded to 32 keys)
//   k_hist  [S, Hkv, ldh, D]            vt_hist [S, Hkv, ldh/32, D, 32]  (ldh % 32 == 0)
// V is stored TRANSPOSED IN 32-KEY TILES: the tile of keys 32c .. 32c+31 is D rows of 32
// keys, contiguous (64 B per row): a key block's V^T is one 2-16 KB span, read as 16 rows
// of 64 B per load instruction (a plain [D][keys] transpose puts the rows a whole key axis
// apart — tens of KB — and the scattered 64-byte reads ran 10x below the HBM rate).
//   out     [n_tok, H, D]
// Query token t of stream s sees prefix keys [0, plen[pfx]) and history keys
// [0, hist_base + t] (its own key is history slot hist_base + t).
//
// Operand orientation (MI355X 16x16x32 bf16 maps, cdna_hip_programming.md §3): the score
// tile is computed transposed, S^T = K . Q^T (A = 16 keys x 32 d, B = Q^T), so lane l ends
// with query l&15's scores for keys 4(l>>4)+i of each 16-key tile.  Those scores become the
// B operand of O^T = V^T . P^T for a 32-key block without any lane movement, by ordering the
// k slots as key(h, j) = 16(j>>2) + 4h + (j&3): V^T rows are key-contiguous (hence the
// transposed V layout) and give the matching 2 x 8-byte A fragments.  Every lane keeps ONE
// query column throughout, so the softmax rescale needs no shuffle; the row max needs two
// xor-shuffles across the four lane groups.
#include "cs_kernels.cuh"

#include <algorithm>
#include <vector>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kAttnThreads = 256;   // 4 waves
constexpr int kGroupRows = 64;      // query rows per workgroup (4 tiles of 16)
constexpr int kKeyBlock = 32;
constexpr int kMaxSplit = 32;       // key splits of one (group, head, query group)
constexpr int kPlanMinBase = 1024;  // from this many (group, head, query group) workgroups on,
                                    // the chip is full without key splits: no plan
constexpr int kMergeRows = 8;       // query rows per merge workgroup (2 per wave)
#ifndef CS_ATTN_LAZY
#define CS_ATTN_LAZY 8.0f           // attend_block's lazy-rescale threshold (log2 units; 0: every block)
#endif
constexpr float kLazyRescale = CS_ATTN_LAZY;
constexpr int64_t kPlanImbalance = 4;   // ... or from a longest cell 4x the mean on (T = 1)
constexpr int kTargetWgsDefault = 512;    // plan: split cells until about this many workgroups
constexpr int kMinItemsDefault = 3;       // ... but never below this many key blocks per wave

// Work plan entries (int32 x 4, device memory), attention entries first:
//   attention  {pg = group * Hkv + head, query group, split | n_used << 8, partial slot}
//   merge      {pg, query group, first partial slot, row chunk | n_used << 8}
struct AttnParams {
  const __bf16* q;
  const __bf16* kp;
  const __bf16* vtp;
  const int64_t* poff;
  const int32_t* plen;
  const int32_t* gpfx;      // group -> prefix index (nullable: identity)
  const __bf16* kh;
  const __bf16* vth;
  const int32_t* hist_base;
  const int32_t* hrow;      // row-layout history (cs_prefix_attention_rows): [S][ldh] stream
                            // row holding each slot; nullptr: V^T tiles, slot j of stream s in row s
  __bf16* out;
  float* part;              // [slot][kGroupRows][D + 2]: O (unnormalised), m, l
  const int4* plan;         // nullable: one workgroup per (group, head, query group), no split
  int64_t ldp, ldh;
  int32_t n_grp, n_str, T, H, Hkv, rep, n_qg, n_attn;
  float scale, softcap, inv_softcap;
  int32_t window;           // > 0: keys more than window - 1 positions back are masked
  int32_t swizzle;
};


// the workgroup's logical id: consecutive logical ids on one XCD (dispatch is round-robin
// over the 8 XCDs), so the query groups of one (prefix, head) share that XCD's L2
__device__ __forceinline__ int logical_block(int swz) {
  const int b = blockIdx.x;
  if (!swz) return b;
  const int per = gridDim.x >> 3;
  return (b & 7) * per + (b >> 3);
}

// ROWS history V image: the chunk swizzle of key k (even, so 32-byte pairs stay whole; the
// 8 keys of a half-wave's transposed read land in 8 different 8-bank groups)
template <int D>
__device__ __forceinline__ int vimg_swz(int k) {
  return D == 64 ? 2 * ((k >> 1) & 3) : 2 * (k & 7);
}

// One 32-key block's operands for this lane: K rows kb + col and kb + 16 + col (8 bf16 of
// each 32-wide d step), V^T rows (16-row d tiles) of the block's 32-key tile.
template <int D>
struct KeyBlock {
  bf16x8 k0[D / 32], k1[D / 32];
  bf16x4 vlo[D / 16], vhi[D / 16];
};

// where key block `it` of a query tile lives: the prefix blocks first, then the history
// blocks of the tile's streams b_lo .. (nbh blocks each)
struct ItemRef {
  const __bf16* k;   // this lane's first K row
  const __bf16* v;   // this lane's first V^T row
  int kb, lim, pos0;
};

__device__ __forceinline__ ItemRef item_ref(const AttnParams& a, int it, int nbp, int nbh, int b_lo,
                                            int b, int gi, int g, int64_t po, int pl, int hv,
                                            bool vrow, int col, int h4, int D) {
  ItemRef r;
  if (it < nbp) {
    r.kb = it * kKeyBlock;
    const int64_t k0 = static_cast<int64_t>(g) * a.ldp + po;
    r.k = a.kp + (k0 + r.kb + col) * D + 8 * h4;
    r.v = a.vtp + (k0 + r.kb) * D + col * kKeyBlock + 4 * h4;
    r.lim = vrow ? pl : 0;
    r.pos0 = 0;
  } else {
    const int ih = it - nbp;
    const int bb = b_lo + ih / nbh;
    r.kb = (ih % nbh) * kKeyBlock;
    const int64_t sh = (static_cast<int64_t>(gi) * a.n_str + bb) * a.Hkv + g;
    r.k = a.kh + (sh * a.ldh + r.kb + col) * D + 8 * h4;
    r.v = a.vth + (sh * a.ldh + r.kb) * D + col * kKeyBlock + 4 * h4;
    r.lim = (vrow && bb == b) ? hv : 0;
    r.pos0 = pl;
  }
  return r;
}

// all of a block's loads issued back to back (one memory round trip per block)
template <int D>
__device__ __forceinline__ void load_block(KeyBlock<D>& f, const ItemRef& r) {
#pragma unroll
  for (int ds = 0; ds < D / 32; ++ds) {
    f.k0[ds] = *reinterpret_cast<const bf16x8*>(r.k + ds * 32);
    f.k1[ds] = *reinterpret_cast<const bf16x8*>(r.k + 16 * D + ds * 32);
  }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    f.vlo[dt] = *reinterpret_cast<const bf16x4*>(r.v + dt * 16 * kKeyBlock);
    f.vhi[dt] = *reinterpret_cast<const bf16x4*>(r.v + dt * 16 * kKeyBlock + 16);
  }
}

// S^T = K . Q^T for the block's 32 keys, online softmax update, O^T += V^T . P^T
template <int D>
__device__ __forceinline__ void attend_block(const AttnParams& a, const KeyBlock<D>& f,
                                             const ItemRef& r, const bf16x8 (&qf)[D / 32],
                                             int kmin_pos, int h4, f32x4 (&o)[D / 16], float& m,
                                             float& l) {
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ds = 0; ds < D / 32; ++ds) {
    s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.k0[ds], qf[ds], s0, 0, 0, 0);
    s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.k1[ds], qf[ds], s1, 0, 0, 0);
  }
  float y[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    y[i] = s0[i];
    y[4 + i] = s1[i];
  }
  float bm = -INFINITY;
  if constexpr (D <= 128) {
    // the scale into log2 units in one multiply without a soft-cap, and a key k0 + j of the
    // lane's 8 visible iff jlo <= j < jhi: fewer vector instructions per block (the online
    // softmax, not the MFMA, paces these kernels; D = 256 keeps the plain form, whose
    // registers are at the two-waves-per-SIMD limit)
    if (a.softcap > 0.0f) {
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = softcap_fn(y[i] * a.scale, a.softcap, a.inv_softcap) * kLog2e;
    } else {
      const float sl2 = a.scale * kLog2e;
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] *= sl2;
    }
    const int k0 = r.kb + 4 * h4;
    const int jlo = kmin_pos == INT32_MIN ? INT32_MIN : kmin_pos - r.pos0 - k0, jhi = r.lim - k0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = (i >> 2) * 16 + (i & 3);
      y[i] = (j < jhi && j >= jlo) ? y[i] : -INFINITY;
      bm = fmaxf(bm, y[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int key = r.kb + (i >> 2) * 16 + 4 * h4 + (i & 3);
      float x = y[i] * a.scale;
      if (a.softcap > 0.0f) x = softcap_fn(x, a.softcap, a.inv_softcap);
      x *= kLog2e;
      y[i] = (key < r.lim && r.pos0 + key >= kmin_pos) ? x : -INFINITY;
      bm = fmaxf(bm, y[i]);
    }
  }
  bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
  bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
  // lazy rescale: the running max moves (and l, O are rescaled) only when some query column
  // of the wave sees a block max more than kLazyRescale (log2 units) above its own — until
  // then the stale max stands and p = 2^(s - m) stays <= 2^kLazyRescale (exact in the final
  // O / l, which share it).  Most blocks after the first few skip the rescale's vector work.
  float mn = m;
  if (__ballot(bm > m + kLazyRescale) != 0) {   // wave-uniform
    mn = fmaxf(m, bm);
    const float alpha = mn == -INFINITY ? 1.0f : __builtin_amdgcn_exp2f(m - mn);
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) o[dt] *= alpha;
  }
  const bool none = mn == -INFINITY;
  float ps = 0.0f;
  bf16x8 pb;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float pv = none ? 0.0f : __builtin_amdgcn_exp2f(y[i] - mn);
    ps += pv;
    pb[i] = static_cast<__bf16>(pv);
  }
  l += ps;
  m = mn;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    const bf16x8 va = {f.vlo[dt][0], f.vlo[dt][1], f.vlo[dt][2], f.vlo[dt][3],
                       f.vhi[dt][0], f.vhi[dt][1], f.vhi[dt][2], f.vhi[dt][3]};
    o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[dt], 0, 0, 0);
  }
}

// PF: register double buffering (the next block's loads in flight while the current one
// is attended) for the latency-bound decode launches (few workgroups, a plan); without it
// the kernel holds fewer registers and more waves per SIMD, which serves the many-workgroup
// scoring launches (T > 1) better.
template <int D, bool PF>
__global__ __launch_bounds__(kAttnThreads, PF ? (D <= 128 ? 2 : 1) : (D <= 128 ? 3 : 2))
void prefix_attn_kernel(AttnParams a) {
  constexpr int NDS = D / 32;   // 32-wide d steps of S^T = K . Q^T
  constexpr int NDT = D / 16;   // 16-row d tiles of O^T
  constexpr int LDSW = D + 2;   // per query row: O[D], m, l
  __shared__ float sm[3][16][LDSW];

  int pg, qg, split, n_used, slot;
  if (a.plan) {
    const int4 e = a.plan[blockIdx.x];
    pg = e.x;
    qg = e.y;
    split = e.z & 255;
    n_used = e.z >> 8;
    slot = e.w;
  } else {
    const int bid = logical_block(a.swizzle);
    qg = bid % a.n_qg;
    pg = bid / a.n_qg;
    split = 0;
    n_used = 1;
    slot = 0;
  }
  const int gi = pg / a.Hkv, g = pg % a.Hkv;
  const int p = a.gpfx ? a.gpfx[gi] : gi;
  const int M = a.n_str * a.T * a.rep;
  const int r0 = qg * kGroupRows;
  const int nrows = min(kGroupRows, M - r0);
  const int n_qt = (nrows + 15) >> 4;
  const int kw = n_qt == 1 ? 4 : (n_qt == 2 ? 2 : 1);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qt = w % n_qt, ks = w / n_qt;
  const bool active = ks < kw;
  const int col = lane & 15, h4 = lane >> 4;

  const int row = r0 + qt * 16 + col;
  const bool vrow = active && row < M;
  const int rr = row < M ? row : M - 1;
  const int jh = rr % a.rep, bt = rr / a.rep;
  const int t = bt % a.T, b = bt / a.T;
  const int64_t s = static_cast<int64_t>(gi) * a.n_str + b;
  const int64_t tok = s * a.T + t;
  const int head = g * a.rep + jh;
  const int hb = *a.hist_base;
  const int pl = a.plen[p];
  const int64_t po = a.poff[p];
  const int hv = min(hb + t + 1, static_cast<int>(a.ldh));
  // sliding window (Gemma-2 even layers): key position > qpos - window; prefix key j sits at
  // position j, history slot j at pl + j, the query at pl + hb + t
  const int kmin_pos = a.window > 0 ? pl + hb + t - a.window + 1 : INT32_MIN;

  // the tile's streams (wave-uniform)
  const int rt0 = r0 + qt * 16, rt1 = min(rt0 + 15, M - 1);
  const int b_lo = (rt0 / a.rep) / a.T, b_hi = (rt1 / a.rep) / a.T;
  const int t_hi = b_lo == b_hi ? (rt1 / a.rep) % a.T : a.T - 1;
  const int nbh = (min(hb + t_hi + 1, static_cast<int>(a.ldh)) + kKeyBlock - 1) / kKeyBlock;
  const int nbp = (pl + kKeyBlock - 1) / kKeyBlock;
  const int n_items = nbp + (b_hi - b_lo + 1) * nbh;

  bf16x8 qf[NDS];
  {
    const __bf16* qrow = a.q + (tok * a.H + head) * D + 8 * h4;
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds) {
      if (vrow) {
        qf[ds] = *reinterpret_cast<const bf16x8*>(qrow + ds * 32);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[ds][e] = static_cast<__bf16>(0.0f);
      }
    }
  }

  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.0f;

  // the wave's blocks it0, it0 + nslot, ...: two register buffers, the next block's loads
  // in flight while the current one is attended (a wave issues ONE round trip per block,
  // overlapped with the previous block's MFMA / softmax work).  The last block's
  // "next" is itself again (an L2 hit) so the loop body has no branch around the loads.
  const int nslot = n_used * kw;
  int it = split * kw + ks;
  if (!PF && active) {
    for (; it < n_items; it += nslot) {
      KeyBlock<D> f;
      const ItemRef r = item_ref(a, it, nbp, nbh, b_lo, b, gi, g, po, pl, hv, vrow, col, h4, D);
      load_block<D>(f, r);
      attend_block<D>(a, f, r, qf, kmin_pos, h4, o, m, l);
    }
  } else if (active && it < n_items) {
    KeyBlock<D> fa, fb;
    ItemRef ra = item_ref(a, it, nbp, nbh, b_lo, b, gi, g, po, pl, hv, vrow, col, h4, D), rb;
    load_block<D>(fa, ra);
    while (true) {
      int itn = it + nslot < n_items ? it + nslot : it;
      rb = item_ref(a, itn, nbp, nbh, b_lo, b, gi, g, po, pl, hv, vrow, col, h4, D);
      load_block<D>(fb, rb);
      __builtin_amdgcn_sched_barrier(0);
      attend_block<D>(a, fa, ra, qf, kmin_pos, h4, o, m, l);
      it += nslot;
      if (it >= n_items) break;
      itn = it + nslot < n_items ? it + nslot : it;
      ra = item_ref(a, itn, nbp, nbh, b_lo, b, gi, g, po, pl, hv, vrow, col, h4, D);
      load_block<D>(fa, ra);
      __builtin_amdgcn_sched_barrier(0);
      attend_block<D>(a, fb, rb, qf, kmin_pos, h4, o, m, l);
      it += nslot;
      if (it >= n_items) break;
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);

  // waves that share a query tile combine through LDS (fixed order: ks = 0, 1, ...)
  if (kw > 1) {
    if (active && ks > 0) {
      const int sl = w - n_qt;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sm[sl][col][dt * 16 + 4 * h4 + i] = o[dt][i];
      if (h4 == 0) {
        sm[sl][col][D] = m;
        sm[sl][col][D + 1] = l;
      }
    }
    __syncthreads();
    if (active && ks == 0) {
      float mt = m;
      for (int k = 1; k < kw; ++k) mt = fmaxf(mt, sm[qt + n_qt * k - n_qt][col][D]);
      const float c0 = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m - mt);
      l *= c0;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] *= c0;
      for (int k = 1; k < kw; ++k) {
        const int sl = qt + n_qt * k - n_qt;
        const float mk = sm[sl][col][D];
        const float ck = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(mk - mt);
        l = fmaf(sm[sl][col][D + 1], ck, l);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[dt][i] = fmaf(sm[sl][col][dt * 16 + 4 * h4 + i], ck, o[dt][i]);
      }
      m = mt;
    }
  }
  if (!vrow || ks != 0) return;
  if (n_used == 1) {
    const float inv = l > 0.0f ? 1.0f / l : 0.0f;
    __bf16* orow = a.out + (tok * a.H + head) * D + 4 * h4;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = static_cast<__bf16>(o[dt][i] * inv);
      *reinterpret_cast<bf16x4*>(orow + dt * 16) = v;
    }
  } else {
    float* pr = a.part + (static_cast<int64_t>(slot) * kGroupRows + qt * 16 + col) * LDSW;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
      *reinterpret_cast<f32x4*>(pr + dt * 16 + 4 * h4) = o[dt];
    if (h4 == 0) {
      pr[D] = m;
      pr[D + 1] = l;
    }
  }
}

// Scoring chunks and prompt prefill (no plan, T > 1, >= 1024 cells): the workgroup's four
// 16-row query tiles walk ONE key-block list — the agent's prefix blocks, then the history
// blocks of every stream the 64 rows touch, up to the furthest query's causal limit — and
// each 32-key block is staged through LDS once per workgroup (K rows padded to D + 8, V^T
// rows to 40 keys: conflict-free fragment reads), double-buffered: the next block's 16-byte
// global loads are in flight while the current one is attended from LDS.  The per-wave
// kernel above loads every block once per tile (4x the L2 traffic for 64 rows of one
// stream).  Blocks outside a tile's own stream or causal range are masked per lane, as
// there; the arithmetic of a block is attend_block's, so the result matches the per-wave
// kernel up to the order of the key blocks within a split (one split here).
template <int D>
struct LdsTile {
  static constexpr int KROW = D + 8;                 // bf16 per staged K row
  static constexpr int VROW = 40;                    // bf16 per staged V^T row (32 keys + pad)
  static constexpr int KELEMS = kKeyBlock * KROW;
  static constexpr int VELEMS = D * VROW;
  static constexpr int ELEMS = KELEMS + VELEMS;      // one buffer
  static constexpr int NCH = D / 64;                 // 16-byte chunks per thread per operand
};

#ifndef CS_ATTN_LDS_W256
#define CS_ATTN_LDS_W256 1   // waves per SIMD of the D = 256 variant (2: 208 B/lane of spills)
#endif
template <int D>
__global__ __launch_bounds__(kAttnThreads, D <= 128 ? 2 : CS_ATTN_LDS_W256)
void prefix_attn_lds_kernel(AttnParams a) {
  using LT = LdsTile<D>;
  constexpr int NDS = D / 32;
  constexpr int NDT = D / 16;
  constexpr int LDSW = D + 2;
  constexpr int kBufBytes = 2 * LT::ELEMS * 2;
  constexpr int kCombBytes = 3 * 16 * LDSW * 4;
  __shared__ __attribute__((aligned(16))) char lds[kBufBytes > kCombBytes ? kBufBytes : kCombBytes];
  __bf16* buf = reinterpret_cast<__bf16*>(lds);
  auto sm = reinterpret_cast<float (*)[16][LDSW]>(lds);   // the wave combine, after the loop

  const int bid = logical_block(a.swizzle);
  const int qg = bid % a.n_qg, pg = bid / a.n_qg;
  const int gi = pg / a.Hkv, g = pg % a.Hkv;
  const int p = a.gpfx ? a.gpfx[gi] : gi;
  const int M = a.n_str * a.T * a.rep;
  const int r0 = qg * kGroupRows;
  const int nrows = min(kGroupRows, M - r0);
  const int n_qt = (nrows + 15) >> 4;
  const int kw = n_qt == 1 ? 4 : (n_qt == 2 ? 2 : 1);
  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int qt = w % n_qt, ks = w / n_qt;
  const bool active = ks < kw;
  const int col = lane & 15, h4 = lane >> 4;

  const int row = r0 + qt * 16 + col;
  const bool vrow = active && row < M;
  const int rr = row < M ? row : M - 1;
  const int jh = rr % a.rep, bt = rr / a.rep;
  const int t = bt % a.T, b = bt / a.T;
  const int64_t tok = (static_cast<int64_t>(gi) * a.n_str + b) * a.T + t;
  const int head = g * a.rep + jh;
  const int hb = *a.hist_base;
  const int pl = a.plen[p];
  const int64_t po = a.poff[p];
  const int hv = min(hb + t + 1, static_cast<int>(a.ldh));
  const int kmin_pos = a.window > 0 ? pl + hb + t - a.window + 1 : INT32_MIN;

  // the workgroup's key blocks (uniform): prefix, then nbh history blocks per stream b_lo..b_hi
  const int rw1 = r0 + nrows - 1;
  const int b_lo = (r0 / a.rep) / a.T, b_hi = (rw1 / a.rep) / a.T;
  const int t_hi = b_lo == b_hi ? (rw1 / a.rep) % a.T : a.T - 1;
  const int nbh = (min(hb + t_hi + 1, static_cast<int>(a.ldh)) + kKeyBlock - 1) / kKeyBlock;
  const int nbp = (pl + kKeyBlock - 1) / kKeyBlock;
  const int n_items = nbp + (b_hi - b_lo + 1) * nbh;

  // item it: global K rows / V^T tile of 32 keys (contiguous) and this lane's mask data
  auto item_src = [&](int it, const __bf16*& ks_, const __bf16*& vs_) {
    if (it < nbp) {
      const int64_t k0 = static_cast<int64_t>(g) * a.ldp + po + it * kKeyBlock;
      ks_ = a.kp + k0 * D;
      vs_ = a.vtp + k0 * D;
    } else {
      const int ih = it - nbp;
      const int bb = b_lo + ih / nbh;
      const int64_t sh = (static_cast<int64_t>(gi) * a.n_str + bb) * a.Hkv + g;
      const int64_t k0 = sh * a.ldh + (ih % nbh) * kKeyBlock;
      ks_ = a.kh + k0 * D;
      vs_ = a.vth + k0 * D;
    }
  };
  auto item_mask = [&](int it) {
    ItemRef r;
    r.k = nullptr;
    r.v = nullptr;
    if (it < nbp) {
      r.kb = it * kKeyBlock;
      r.lim = vrow ? pl : 0;
      r.pos0 = 0;
    } else {
      const int ih = it - nbp;
      const int bb = b_lo + ih / nbh;
      r.kb = (ih % nbh) * kKeyBlock;
      r.lim = (vrow && bb == b) ? hv : 0;
      r.pos0 = pl;
    }
    return r;
  };
  // staging: thread tid copies 16-byte chunks c = tid + 256 j of K (row c / (D/8)) and of
  // V^T (d row c / 4, keys 8 (c % 4) ..)
  u32x4 rk[LT::NCH], rv[LT::NCH];
  auto fetch = [&](int it) {
    const __bf16 *ksrc, *vsrc;
    item_src(it, ksrc, vsrc);
#pragma unroll
    for (int j = 0; j < LT::NCH; ++j) {
      const int c = tid + kAttnThreads * j;
      rk[j] = *reinterpret_cast<const u32x4*>(ksrc + c * 8);
      rv[j] = *reinterpret_cast<const u32x4*>(vsrc + c * 8);
    }
  };
  auto stage = [&](int sbuf) {
    __bf16* kd = buf + sbuf * LT::ELEMS;
    __bf16* vd = kd + LT::KELEMS;
#pragma unroll
    for (int j = 0; j < LT::NCH; ++j) {
      const int c = tid + kAttnThreads * j;
      *reinterpret_cast<u32x4*>(kd + (c / (D / 8)) * LT::KROW + (c % (D / 8)) * 8) = rk[j];
      *reinterpret_cast<u32x4*>(vd + (c >> 2) * LT::VROW + (c & 3) * 8) = rv[j];
    }
  };

  bf16x8 qf[NDS];
  {
    const __bf16* qrow = a.q + (tok * a.H + head) * D + 8 * h4;
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds) {
      if (vrow) {
        qf[ds] = *reinterpret_cast<const bf16x8*>(qrow + ds * 32);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[ds][e] = static_cast<__bf16>(0.0f);
      }
    }
  }
  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.0f;

  if (n_items > 0) {
    fetch(0);
    stage(0);
  }
  __syncthreads();
  for (int it = 0; it < n_items; ++it) {
    const bool more = it + 1 < n_items;
    if (more) fetch(it + 1);
    if (active && (it % kw) == ks) {
      const __bf16* kd = buf + (it & 1) * LT::ELEMS;
      const __bf16* vd = kd + LT::KELEMS;
      KeyBlock<D> f;
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds) {
        f.k0[ds] = *reinterpret_cast<const bf16x8*>(kd + col * LT::KROW + ds * 32 + 8 * h4);
        f.k1[ds] = *reinterpret_cast<const bf16x8*>(kd + (16 + col) * LT::KROW + ds * 32 + 8 * h4);
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        f.vlo[dt] = *reinterpret_cast<const bf16x4*>(vd + (dt * 16 + col) * LT::VROW + 4 * h4);
        f.vhi[dt] = *reinterpret_cast<const bf16x4*>(vd + (dt * 16 + col) * LT::VROW + 16 + 4 * h4);
      }
      attend_block<D>(a, f, item_mask(it), qf, kmin_pos, h4, o, m, l);
    }
    if (more) stage((it + 1) & 1);   // buffer (it + 1) & 1 was last read in iteration it - 1
    __syncthreads();
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);

  // waves that share a query tile combine through LDS (fixed order: ks = 0, 1, ...)
  if (kw > 1) {
    if (active && ks > 0) {
      const int sl = w - n_qt;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sm[sl][col][dt * 16 + 4 * h4 + i] = o[dt][i];
      if (h4 == 0) {
        sm[sl][col][D] = m;
        sm[sl][col][D + 1] = l;
      }
    }
    __syncthreads();
    if (active && ks == 0) {
      float mt = m;
      for (int k = 1; k < kw; ++k) mt = fmaxf(mt, sm[qt + n_qt * k - n_qt][col][D]);
      const float c0 = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m - mt);
      l *= c0;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] *= c0;
      for (int k = 1; k < kw; ++k) {
        const int sl = qt + n_qt * k - n_qt;
        const float mk = sm[sl][col][D];
        const float ck = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(mk - mt);
        l = fmaf(sm[sl][col][D + 1], ck, l);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[dt][i] = fmaf(sm[sl][col][dt * 16 + 4 * h4 + i], ck, o[dt][i]);
      }
      m = mt;
    }
  }
  if (!vrow || ks != 0) return;
  const float inv = l > 0.0f ? 1.0f / l : 0.0f;
  __bf16* orow = a.out + (tok * a.H + head) * D + 4 * h4;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    bf16x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = static_cast<__bf16>(o[dt][i] * inv);
    *reinterpret_cast<bf16x4*>(orow + dt * 16) = v;
  }
}

#ifdef CS_TRACE_ATTN
// diagnostics build only (tools/attn_trace.py): wall_clock64 ticks (100 MHz) per workgroup of
// the last decode-step launch, plain stores (no atomics: those serialise and distort):
// attention [wg][0 start, 1 prologue loads in, 2 prefix loop done, 3 history loop done
// (wave 0), 4 partial stored (wave 0)], merge [wg][5 start, 6 done]
constexpr int kAttTraceWgs = 4096;
__device__ unsigned long long g_attn_ts[kAttTraceWgs][8];
#define ATT_T(...) __VA_ARGS__
__device__ __forceinline__ void att_at(int i) {
  if (blockIdx.x < kAttTraceWgs) g_attn_ts[blockIdx.x][i] = wall_clock64();
}
#else
#define ATT_T(...)
#endif

// Decode steps (a plan: few (group, head) cells, key splits): the agent's PREFIX blocks
// are shared by the workgroup's four 16-row tiles, so the split's prefix blocks (split,
// split + n_used, ...) are staged through LDS once per workgroup and attended by every
// tile (the per-wave kernel loads each one per tile: 4x the load instructions, 68 % issue
// stalls at C5); each tile's own streams' history blocks are then loaded per wave as
// there.  Every key block is attended exactly once per (query row, split) as in the
// per-wave assignment, so the split partials and the merge are unchanged.
// two waves per SIMD at every D (D = 256: 237 VGPRs, no spills; 1 wave/SIMD before)
//
// ROWS (cs_prefix_attention_rows): the history is row-major for K AND V ([S][Hkv][ldh][D])
// and slot j of stream s lives in stream row hrow[s][j] -- a beam inherits its parent's
// slots through the table (cs_hist_rows_update), no K / V is copied.  A history block's 32
// V rows are gathered by LDS DMA into the wave's own 1 KB-per-16-d image [d/16][key][16 d]
// (lane l loads key l / 2, 8 d of d-tile i: one table entry per lane) and read back
// transposed (ds_read_b64_tr_b16: lane 4q + p of group h reads key 4h + q, d 16 dt + 4p) as
// the V^T operand the V^T-tile layout gives; every 32-lane half reads 8 keys x 32 B at
// 32-B key pitch: 64 distinct banks, conflict-free.
template <int D, bool ROWS = false>
__global__ __launch_bounds__(kAttnThreads, 2)
void prefix_attn_plan_lds_kernel(AttnParams a) {
  using LT = LdsTile<D>;
  constexpr int NDS = D / 32;
  constexpr int NDT = D / 16;
  constexpr int LDSW = D + 2;
  constexpr int kBufBytes = 2 * LT::ELEMS * 2;
  constexpr int kCombBytes = 3 * 16 * LDSW * 4;
  constexpr int kVImg = kKeyBlock * D * 2;            // ROWS: one wave's V image of a block
  static_assert(kAttnThreads / 64 * kVImg <= kBufBytes, "the V images fit the prefix buffers");
  __shared__ __attribute__((aligned(16))) char lds[kBufBytes > kCombBytes ? kBufBytes : kCombBytes];
  __bf16* buf = reinterpret_cast<__bf16*>(lds);
  auto sm = reinterpret_cast<float (*)[16][LDSW]>(lds);

  ATT_T(if (threadIdx.x == 0) att_at(0);)
  // no plan (ROWS only): one workgroup per (group, head, query group), unsplit
  const int4 e = a.plan ? a.plan[blockIdx.x]
                        : int4{static_cast<int>(blockIdx.x) / a.n_qg, static_cast<int>(blockIdx.x) % a.n_qg,
                               1 << 8, 0};
  const int pg = e.x, qg = e.y, split = e.z & 255, n_used = e.z >> 8, slot = e.w;
  const int gi = pg / a.Hkv, g = pg % a.Hkv;
  const int p = a.gpfx ? a.gpfx[gi] : gi;
  const int M = a.n_str * a.T * a.rep;
  const int r0 = qg * kGroupRows;
  const int nrows = min(kGroupRows, M - r0);
  const int n_qt = (nrows + 15) >> 4;
  const int kw = n_qt == 1 ? 4 : (n_qt == 2 ? 2 : 1);
  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int qt = w % n_qt, ks = w / n_qt;
  const bool active = ks < kw;
  const int col = lane & 15, h4 = lane >> 4;

  const int row = r0 + qt * 16 + col;
  const bool vrow = active && row < M;
  const int rr = row < M ? row : M - 1;
  const int jh = rr % a.rep, bt = rr / a.rep;
  const int t = bt % a.T, b = bt / a.T;
  const int64_t tok = (static_cast<int64_t>(gi) * a.n_str + b) * a.T + t;
  const int head = g * a.rep + jh;
  const int hb = *a.hist_base;
  const int pl = a.plen[p];
  const int64_t po = a.poff[p];
  const int hv = min(hb + t + 1, static_cast<int>(a.ldh));
  const int kmin_pos = a.window > 0 ? pl + hb + t - a.window + 1 : INT32_MIN;

  const int nbp = (pl + kKeyBlock - 1) / kKeyBlock;
  // this split's prefix blocks: split, split + n_used, ...  (workgroup-uniform)
  const int npi = nbp > split ? (nbp - split + n_used - 1) / n_used : 0;
  ATT_T(if (tid == 0 && npi + hb + po >= 0) att_at(1);)
  // the tile's own streams' history blocks, per wave (split * kw + ks, + nslot, ...)
  const int rt0 = r0 + qt * 16, rt1 = min(rt0 + 15, M - 1);
  const int b_lo = (rt0 / a.rep) / a.T, b_hi = (rt1 / a.rep) / a.T;
  const int t_hi = b_lo == b_hi ? (rt1 / a.rep) % a.T : a.T - 1;
  const int nbh = (min(hb + t_hi + 1, static_cast<int>(a.ldh)) + kKeyBlock - 1) / kKeyBlock;
  const int n_hist = (b_hi - b_lo + 1) * nbh;
  const int nslot = n_used * kw;
  // ROWS: lane l's table entry (key l % 32) of history block ih; the first block's entry is
  // loaded here, its round trip hidden behind the prefix blocks, each later one during the
  // block before it
  auto hrow_of = [&](int ih) -> int32_t {
    const int64_t sg = static_cast<int64_t>(gi) * a.n_str + b_lo + ih / nbh;
    return a.hrow[sg * a.ldh + (ih % nbh) * kKeyBlock + (lane & 31)];
  };
  int32_t hcur = 0;
  if constexpr (ROWS) {
    if (active && split * kw + ks < n_hist) hcur = hrow_of(split * kw + ks);
  }

  bf16x8 qf[NDS];
  {
    const __bf16* qrow = a.q + (tok * a.H + head) * D + 8 * h4;
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds) {
      if (vrow) {
        qf[ds] = *reinterpret_cast<const bf16x8*>(qrow + ds * 32);
      } else {
#pragma unroll
        for (int e2 = 0; e2 < 8; ++e2) qf[ds][e2] = static_cast<__bf16>(0.0f);
      }
    }
  }
  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.0f;

  // ---- prefix blocks through LDS ----
  u32x4 rk[LT::NCH], rv[LT::NCH];
  auto fetch = [&](int j) {
    const int64_t k0 = static_cast<int64_t>(g) * a.ldp + po + (split + j * n_used) * kKeyBlock;
    const __bf16* ksrc = a.kp + k0 * D;
    const __bf16* vsrc = a.vtp + k0 * D;
#pragma unroll
    for (int i = 0; i < LT::NCH; ++i) {
      const int c = tid + kAttnThreads * i;
      rk[i] = *reinterpret_cast<const u32x4*>(ksrc + c * 8);
      rv[i] = *reinterpret_cast<const u32x4*>(vsrc + c * 8);
    }
  };
  auto stage = [&](int sbuf) {
    __bf16* kd = buf + sbuf * LT::ELEMS;
    __bf16* vd = kd + LT::KELEMS;
#pragma unroll
    for (int i = 0; i < LT::NCH; ++i) {
      const int c = tid + kAttnThreads * i;
      *reinterpret_cast<u32x4*>(kd + (c / (D / 8)) * LT::KROW + (c % (D / 8)) * 8) = rk[i];
      *reinterpret_cast<u32x4*>(vd + (c >> 2) * LT::VROW + (c & 3) * 8) = rv[i];
    }
  };
  if (npi > 0) {
    fetch(0);
    stage(0);
  }
  __syncthreads();
  for (int j = 0; j < npi; ++j) {
    const bool more = j + 1 < npi;
    if (more) fetch(j + 1);
    if (active && (j % kw) == ks) {
      const __bf16* kd = buf + (j & 1) * LT::ELEMS;
      const __bf16* vd = kd + LT::KELEMS;
      KeyBlock<D> f;
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds) {
        f.k0[ds] = *reinterpret_cast<const bf16x8*>(kd + col * LT::KROW + ds * 32 + 8 * h4);
        f.k1[ds] = *reinterpret_cast<const bf16x8*>(kd + (16 + col) * LT::KROW + ds * 32 + 8 * h4);
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        f.vlo[dt] = *reinterpret_cast<const bf16x4*>(vd + (dt * 16 + col) * LT::VROW + 4 * h4);
        f.vhi[dt] = *reinterpret_cast<const bf16x4*>(vd + (dt * 16 + col) * LT::VROW + 16 + 4 * h4);
      }
      ItemRef r;
      r.k = nullptr;
      r.v = nullptr;
      r.kb = (split + j * n_used) * kKeyBlock;
      r.lim = vrow ? pl : 0;
      r.pos0 = 0;
      attend_block<D>(a, f, r, qf, kmin_pos, h4, o, m, l);
    }
    if (more) stage((j + 1) & 1);
    __syncthreads();
  }

  ATT_T(if (tid == 0) att_at(2);)
  if constexpr (!ROWS) {
    if (active) {
      for (int ih = split * kw + ks; ih < n_hist; ih += nslot) {
        KeyBlock<D> f;
        const ItemRef r = item_ref(a, nbp + ih, nbp, nbh, b_lo, b, gi, g, po, pl, hv, vrow, col, h4, D);
        load_block<D>(f, r);
        attend_block<D>(a, f, r, qf, kmin_pos, h4, o, m, l);
      }
    }
  } else {
    unsigned char* vimg = reinterpret_cast<unsigned char*>(lds) + w * kVImg;
    // the wave's V image of a block: key-major, key k's 2D bytes at 2D k, its 16-byte chunk c
    // at chunk c ^ sw(k) (sw even: 32-byte pairs stay whole).  A transposed read (lane 4q + p
    // of group h4: key 4 h4 + q, d 16 dt + 4 p) of one half-wave then touches 8 keys whose
    // pairs sit in 8 different 8-bank groups: conflict-free.  A DMA instruction writes KPI
    // whole keys, so only the keys the block's rows can see are gathered
    constexpr int CPK = D / 8;          // 16-byte chunks per key
    constexpr int KPI = 64 / CPK;       // keys per 1 KB DMA instruction
    const int kq = 4 * h4 + ((lane & 15) >> 2);          // this lane's vlo key (vhi: + 16)
    const uint32_t tr_base = static_cast<uint32_t>(kq * 2 * D + 8 * (lane & 3));
    const int s2 = vimg_swz<D>(kq) >> 1;
    // this lane's DMA chunk: key i KPI + lane / CPK of instruction i, chunk lane % CPK
    const int dkey = lane / CPK, dch = lane % CPK;
    typedef __attribute__((address_space(3))) bf16x4* lds_b4_ptr;
    if (active && split * kw + ks < n_hist) {
      // the image starts zeroed: a key the block's rows cannot see is not gathered, and its
      // V row must still be finite (its probability is 0; 0 x NaN is not): zeros, or an
      // earlier block's rows
#pragma unroll
      for (int i = 0; i < kVImg / 1024; ++i)
        *reinterpret_cast<u32x4*>(vimg + 1024 * i + 16 * lane) = u32x4{0u, 0u, 0u, 0u};
    }
    if (active) {
      for (int ih = split * kw + ks; ih < n_hist; ih += nslot) {
        const int bb = b_lo + ih / nbh;
        const int kb = (ih % nbh) * kKeyBlock;
        // keys the tile's rows can see (wave-uniform): only those are gathered
        const int nvalid = min(kKeyBlock, min(hb + t_hi + 1, static_cast<int>(a.ldh)) - kb);
        const int n_instr = (nvalid + KPI - 1) / KPI;
        auto row_ptr = [&](const __bf16* base, int64_t srow, int key) {
          return base + ((srow * a.Hkv + g) * a.ldh + kb + key) * D;
        };
        // stream rows of keys col, 16 + col (K fragments)
        const int64_t rk0 = __shfl(hcur, col, 64), rk1 = __shfl(hcur, 16 + col, 64);
        KeyBlock<D> f;
        const __bf16* kp0 = row_ptr(a.kh, rk0, col) + 8 * h4;
        const __bf16* kp1 = row_ptr(a.kh, rk1, 16 + col) + 8 * h4;
        // K first, then the V gather (the DMA issue never waits), then the next block's
        // table entry: every load of the block in flight before the one wait
#pragma unroll
        for (int ds = 0; ds < NDS; ++ds) {
          f.k0[ds] = *reinterpret_cast<const bf16x8*>(kp0 + ds * 32);
          f.k1[ds] = *reinterpret_cast<const bf16x8*>(kp1 + ds * 32);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the last block's reads are done
#pragma unroll 1
        for (int i = 0; i < n_instr; ++i) {
          const int k = i * KPI + dkey;
          const int64_t rv = __shfl(hcur, k, 64);
          const __bf16* vsrc = row_ptr(a.vth, rv, k) + 8 * (dch ^ vimg_swz<D>(k));
          __builtin_amdgcn_global_load_lds(vsrc, (__attribute__((address_space(3))) void*)(vimg + 1024 * i),
                                           16, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        const int ihn = ih + nslot < n_hist ? ih + nslot : ih;
        const int32_t hnext = hrow_of(ihn);
        __builtin_amdgcn_sched_barrier(0);
        // the V image landed (the compiler drains every VMEM op before an LDS read that
        // follows an LDS DMA: the next table entry, an L2 hit issued after the HBM-bound
        // gather, is in by then too)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const uint32_t o2 = tr_base + 32 * (((dt & 7) ^ s2) + (dt & ~7));
          f.vlo[dt] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4_ptr)(vimg + o2));
          f.vhi[dt] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4_ptr)(vimg + o2 + 32 * D));
        }
        ItemRef r;
        r.k = nullptr;
        r.v = nullptr;
        r.kb = kb;
        r.lim = (vrow && bb == b) ? hv : 0;
        r.pos0 = pl;
        attend_block<D>(a, f, r, qf, kmin_pos, h4, o, m, l);
        hcur = hnext;
      }
    }
    __syncthreads();   // every wave's V image read before the combine reuses the LDS
  }
  ATT_T(if (tid == 0 && l >= 0.0f) att_at(3);)
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);

  if (kw > 1) {
    if (active && ks > 0) {
      const int sl = w - n_qt;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sm[sl][col][dt * 16 + 4 * h4 + i] = o[dt][i];
      if (h4 == 0) {
        sm[sl][col][D] = m;
        sm[sl][col][D + 1] = l;
      }
    }
    __syncthreads();
    if (active && ks == 0) {
      float mt = m;
      for (int k = 1; k < kw; ++k) mt = fmaxf(mt, sm[qt + n_qt * k - n_qt][col][D]);
      const float c0 = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m - mt);
      l *= c0;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] *= c0;
      for (int k = 1; k < kw; ++k) {
        const int sl = qt + n_qt * k - n_qt;
        const float mk = sm[sl][col][D];
        const float ck = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(mk - mt);
        l = fmaf(sm[sl][col][D + 1], ck, l);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[dt][i] = fmaf(sm[sl][col][dt * 16 + 4 * h4 + i], ck, o[dt][i]);
      }
      m = mt;
    }
  }
  if (!vrow || ks != 0) return;
  if (n_used == 1) {
    const float inv = l > 0.0f ? 1.0f / l : 0.0f;
    __bf16* orow = a.out + (tok * a.H + head) * D + 4 * h4;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = static_cast<__bf16>(o[dt][i] * inv);
      *reinterpret_cast<bf16x4*>(orow + dt * 16) = v;
    }
  } else {
    float* pr = a.part + (static_cast<int64_t>(slot) * kGroupRows + qt * 16 + col) * LDSW;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
      *reinterpret_cast<f32x4*>(pr + dt * 16 + 4 * h4) = o[dt];
    if (h4 == 0) {
      pr[D] = m;
      pr[D + 1] = l;
    }
  }
  ATT_T(if (tid == 0) { __builtin_amdgcn_s_waitcnt(0); att_at(4); })
}

// One workgroup per merge entry (kMergeRows rows of a split (group, head, query group)),
// each wave two rows, one per 32-lane half: the half's lanes fold the splits' (m, l) into
// per-split weights, then the wave sums the weighted partial outputs (f32x4 columns).
// Fixed split order: deterministic.
template <int D>
__global__ __launch_bounds__(kAttnThreads) void attn_merge_kernel(AttnParams a) {
  constexpr int LDSW = D + 2;
  constexpr int NC = D / 4;
  __shared__ float wsm[kAttnThreads / 64][2][kMaxSplit];
  __shared__ float linv[kAttnThreads / 64][2];
  ATT_T(if (threadIdx.x == 0) att_at(5);)
  const int4 e = a.plan[a.n_attn + blockIdx.x];
  const int pg = e.x, qg = e.y, slot0 = e.z, chunk = e.w & 255, nu = e.w >> 8;
  const int gi = pg / a.Hkv, g = pg % a.Hkv;
  const int M = a.n_str * a.T * a.rep;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const float* base = a.part + static_cast<int64_t>(slot0) * kGroupRows * LDSW;
  {
    const int rl = chunk * kMergeRows + 2 * w + half;
    const bool vr = qg * kGroupRows + rl < M && l32 < nu;
    float ms = -INFINITY, ls = 0.0f;
    if (vr) {
      const float* pm = base + (static_cast<int64_t>(l32) * kGroupRows + rl) * LDSW + D;
      ms = pm[0];
      ls = pm[1];
    }
    float mt = ms;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) mt = fmaxf(mt, __shfl_xor(mt, o, 64));
    const float wt = (vr && mt != -INFINITY) ? __builtin_amdgcn_exp2f(ms - mt) : 0.0f;
    float lt = wt * ls;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) lt += __shfl_xor(lt, o, 64);
    if (l32 < kMaxSplit) wsm[w][half][l32] = wt;
    if (l32 == 0) linv[w][half] = lt > 0.0f ? 1.0f / lt : 0.0f;
  }
  __syncthreads();
  for (int item = lane; item < 2 * NC; item += 64) {
    const int hr = item / NC, c4 = item % NC;
    const int rl = chunk * kMergeRows + 2 * w + hr;
    const int row = qg * kGroupRows + rl;
    if (row >= M) continue;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int sp = 0; sp < nu; ++sp) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(
          base + (static_cast<int64_t>(sp) * kGroupRows + rl) * LDSW + 4 * c4);
      acc += v * wsm[w][hr][sp];
    }
    const float inv = linv[w][hr];
    const int jh = row % a.rep, bt = row / a.rep;
    const int t = bt % a.T, b = bt / a.T;
    const int64_t tok = (static_cast<int64_t>(gi) * a.n_str + b) * a.T + t;
    bf16x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = static_cast<__bf16>(acc[i] * inv);
    *reinterpret_cast<bf16x4*>(a.out + (tok * a.H + g * a.rep + jh) * D + 4 * c4) = v;
  }
  ATT_T(if (threadIdx.x == 0) { __builtin_amdgcn_s_waitcnt(0); att_at(6); })
}

// RoPE (half-rotation convention) + placement.  One thread per (token, head, pair i < D/2).
struct RopeParams {
  const __bf16* qkv;
  int64_t ldqkv;
  const float* part;        // rope_place_kernel<P, true>: fp32 K-split partials [splits][n_tok][ldqkv]
  int32_t splits;
  const float* inv_freq;
  const int32_t* plen;
  const int32_t* gpfx;
  const int32_t* hist_base;
  __bf16* q_out;
  __bf16* kh;
  __bf16* vth;
  int64_t ldh;
  int64_t n_tok;
  int32_t n_str, T, H, Hkv, D;
  int32_t skip_v;           // V placed by v_tile_place_kernel instead
  int32_t v_rows;           // V row-major like K ([S][Hkv][ldh][D], cs_rope_place_rows)
};

// n_split workgroups per token (kRopeItems (head, P-pair group) items each): the token's D/2
// angles' sincos into LDS, then every item of the workgroup (q, k rotated; v placed) by its
// own thread with 2P-byte loads / stores.  A decode step's few hundred tokens give over a
// thousand workgroups (one workgroup per token left most CUs with one: 18 us per C3 layer);
// a per-thread loop over the heads serialised one memory round trip per head.
constexpr int kRopeItems = 256;

// fp32 -> bf16, round to nearest even, quiet NaN: the rounding of cs_gemm_bf16's split-K
// fold (gemm.hip gto_bf), so a fold done here is bitwise the fold done there
__device__ __forceinline__ __bf16 rope_to_bf(float f) {
  const uint32_t u = __float_as_uint(f);
  const uint16_t h = (u & 0x7fffffffu) > 0x7f800000u
                         ? static_cast<uint16_t>((u >> 16) | 0x40)
                         : static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  return __builtin_bit_cast(__bf16, h);
}

// FOLD: the projection arrives as a K-split GEMM's unfolded fp32 partials (r.part), summed
// here in split order and rounded as cs_gemm_bf16's own fold would -- one launch and one
// bf16 round trip fewer per layer, bitwise the same q / K / V.  NSP splits' loads are issued
// together (surplus ones re-read the last split and are not summed): one memory round trip
// per NSP splits, not one per split.
template <int P, bool FOLD = false, int NSP = 1>
__global__ __launch_bounds__(256) void rope_place_kernel(RopeParams r, int32_t n_split) {
  typedef __bf16 vec_t __attribute__((ext_vector_type(P)));
  __shared__ float cs[128], sn[128];                // D / 2 <= 128
  const int half = r.D >> 1;
  const int nq = half / P;                          // P-pair groups per head
  const int nh = r.H + 2 * r.Hkv;
  const int64_t tok = blockIdx.x / n_split;
  const int split = static_cast<int>(blockIdx.x % n_split);
  const int64_t s = tok / r.T;
  const int t = static_cast<int>(tok % r.T);
  const int gi = static_cast<int>(s / r.n_str);
  const int p = r.gpfx ? r.gpfx[gi] : gi;
  const int slot = *r.hist_base + t;
  const float pos = static_cast<float>(r.plen[p] + slot);
  for (int i = threadIdx.x; i < half; i += 256) sincosf(pos * r.inv_freq[i], &sn[i], &cs[i]);
  __syncthreads();
  const __bf16* __restrict__ row = r.qkv + tok * r.ldqkv;
  __bf16* __restrict__ qo = r.q_out;
  __bf16* __restrict__ kh = r.kh;
  __bf16* __restrict__ vth = r.vth;
  const int lim = min(nh * nq, (split + 1) * kRopeItems);
  for (int item = split * kRopeItems + threadIdx.x; item < lim; item += 256) {
    const int hh = item / nq;
    const int i0 = P * (item - hh * nq);
    vec_t a, b;
    if constexpr (FOLD) {
      const int64_t off = tok * r.ldqkv + static_cast<int64_t>(hh) * r.D + i0;
      const int64_t sstride = r.n_tok * r.ldqkv;
      float fa[P], fb[P];
      for (int c0 = 0; c0 < r.splits; c0 += NSP) {
        f32x4 la[NSP][P / 4], lb[NSP][P / 4];
#pragma unroll
        for (int j = 0; j < NSP; ++j) {
          const int sp = min(c0 + j, r.splits - 1);
#pragma unroll
          for (int e = 0; e < P; e += 4) {
            la[j][e / 4] = *reinterpret_cast<const f32x4*>(r.part + sp * sstride + off + e);
            lb[j][e / 4] = *reinterpret_cast<const f32x4*>(r.part + sp * sstride + off + half + e);
          }
        }
        __builtin_amdgcn_sched_barrier(0);   // every load of the chunk issued before the sums
#pragma unroll
        for (int j = 0; j < NSP; ++j) {
          const bool first = c0 + j == 0, use = c0 + j < r.splits;
#pragma unroll
          for (int e = 0; e < P; e += 4)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float xa = la[j][e / 4][c], xb = lb[j][e / 4][c];
              fa[e + c] = first ? xa : (use ? fa[e + c] + xa : fa[e + c]);
              fb[e + c] = first ? xb : (use ? fb[e + c] + xb : fb[e + c]);
            }
        }
      }
#pragma unroll
      for (int e = 0; e < P; ++e) {
        a[e] = rope_to_bf(fa[e]);
        b[e] = rope_to_bf(fb[e]);
      }
    } else {
      const __bf16* src = row + static_cast<int64_t>(hh) * r.D + i0;
      a = *reinterpret_cast<const vec_t*>(src);
      b = *reinterpret_cast<const vec_t*>(src + half);
    }
    if (hh >= r.H + r.Hkv) {                         // v: transposed placement, no rotation
      if (r.skip_v) continue;
      const int g = hh - r.H - r.Hkv;
      if (r.v_rows) {
        __bf16* dst = vth + ((s * r.Hkv + g) * r.ldh + slot) * r.D;
        *reinterpret_cast<vec_t*>(dst + i0) = a;
        *reinterpret_cast<vec_t*>(dst + half + i0) = b;
        continue;
      }
      __bf16* dst = vth + ((s * r.Hkv + g) * r.ldh + (slot & ~31)) * r.D +
                    static_cast<int64_t>(i0) * 32 + (slot & 31);
#pragma unroll
      for (int e = 0; e < P; ++e) {
        dst[e * 32] = a[e];
        dst[(half + e) * 32] = b[e];
      }
      continue;
    }
    vec_t y1, y2;
#pragma unroll
    for (int e = 0; e < P; ++e) {
      const float x1 = static_cast<float>(a[e]), x2 = static_cast<float>(b[e]);
      y1[e] = static_cast<__bf16>(fmaf(x1, cs[i0 + e], -x2 * sn[i0 + e]));
      y2[e] = static_cast<__bf16>(fmaf(x2, cs[i0 + e], x1 * sn[i0 + e]));
    }
    __bf16* dst = hh < r.H ? qo + (tok * r.H + hh) * r.D
                           : kh + ((s * r.Hkv + (hh - r.H)) * r.ldh + slot) * r.D;
    *reinterpret_cast<vec_t*>(dst + i0) = y1;
    *reinterpret_cast<vec_t*>(dst + half + i0) = y2;
  }
}

// Multi-token streams (T >= 32: scoring chunks, prompt prefill): V placed by 32-slot tiles,
// one workgroup per (stream, K/V head, slot tile): the tile's tokens' V rows (16-byte loads)
// into LDS, then the tile's D rows of 32 slots written with 16-byte stores — the per-token
// placement of rope_place_kernel writes 2-byte pieces 64 B apart, from workgroups on every
// XCD.  Slots outside [hist_base, hist_base + T) are left as they are.
__global__ __launch_bounds__(256) void v_tile_place_kernel(RopeParams r, int32_t n_tiles) {
  __shared__ __attribute__((aligned(16))) __bf16 tile[32][256 + 8];   // [slot][d], D <= 256
  const int D = r.D;
  const int tid = threadIdx.x;
  const int c = static_cast<int>(blockIdx.x % n_tiles);
  const int64_t sg = blockIdx.x / n_tiles;            // s * Hkv + g
  const int g = static_cast<int>(sg % r.Hkv);
  const int64_t s = sg / r.Hkv;
  const int hb = *r.hist_base;
  const int slot0 = 32 * c;
  if (slot0 + 32 <= hb || slot0 >= hb + r.T) return;  // no token of this stream lands here
  const int dch = D >> 3;                              // 16-byte chunks per V row
  for (int ch = tid; ch < 32 * dch; ch += 256) {
    const int sl = ch / dch, dc = ch - sl * dch;
    const int t = slot0 + sl - hb;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (t >= 0 && t < r.T)
      v = *reinterpret_cast<const u32x4*>(r.qkv + (s * r.T + t) * r.ldqkv +
                                          static_cast<int64_t>(r.H + r.Hkv + g) * D + dc * 8);
    *reinterpret_cast<u32x4*>(&tile[sl][dc * 8]) = v;
  }
  __syncthreads();
  __bf16* base = r.vth + ((s * r.Hkv + g) * r.ldh + slot0) * D;   // the tile's [D][32]
  for (int ch = tid; ch < 4 * D; ch += 256) {
    const int d = ch >> 2, q = ch & 3;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[q * 8 + e][d];
    const int t0 = slot0 + q * 8 - hb;
    __bf16* dst = base + d * 32 + q * 8;
    if (t0 >= 0 && t0 + 8 <= r.T) {
      *reinterpret_cast<bf16x8*>(dst) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (t0 + e >= 0 && t0 + e < r.T) dst[e] = v[e];
    }
  }
}

// Row-layout history (cs_hist_rows_update): stream s inherits its parent's slots by table,
// dst[s][j] = src[parent[s]][j] for j < hist_base, and owns the rest (dst[s][j] = row_base +
// s: the slots this step and later ones write into its own row).  One thread per (s, j).
__global__ __launch_bounds__(256) void hist_rows_kernel(const int32_t* __restrict__ src,
                                                        int32_t* __restrict__ dst,
                                                        const int64_t* __restrict__ parent,
                                                        const int32_t* __restrict__ hist_base,
                                                        int64_t S, int32_t ldh, int64_t row_base) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= S * ldh) return;
  const int64_t s = i / ldh;
  const int j = static_cast<int>(i - s * ldh);
  dst[i] = j < *hist_base ? src[parent[s] * ldh + j] : static_cast<int32_t>(row_base + s);
}

// plan tunables (CS_ATTN_TARGET_WGS, CS_ATTN_MIN_ITEMS override; read once)
int env_int(const char* name, int dflt, int lo, int hi) {
  if (const char* e = getenv(name)) {
    const int y = atoi(e);
    if (y >= lo && y <= hi) return y;
  }
  return dflt;
}
int attn_target_wgs() {
  static const int v = env_int("CS_ATTN_TARGET_WGS", kTargetWgsDefault, 1, 1 << 20);
  return v;
}
// scoring chunks / prompt prefill on the LDS-staged kernel (CS_ATTN_LDS=0: the per-wave one)
bool attn_lds() {
  static const bool v = env_int("CS_ATTN_LDS", 1, 0, 1) != 0;
  return v;
}
// decode steps (a plan): the prefix blocks through LDS (CS_ATTN_PLAN_LDS=0: per wave)
bool attn_plan_lds() {
  static const bool v = env_int("CS_ATTN_PLAN_LDS", 1, 0, 1) != 0;
  return v;
}
int attn_min_items() {
  static const int v = env_int("CS_ATTN_MIN_ITEMS", kMinItemsDefault, 1, 4096);
  return v;
}

struct PlanCell {
  int32_t gi, qg, splits, per_wg;
};

}  // namespace

extern "C" {

int64_t cs_prefix_attention_plan(const int32_t* prefix_len, int32_t n_prefix,
                                 const int32_t* group_prefix, int32_t n_groups, int32_t n_str,
                                 int32_t T, int32_t H, int32_t Hkv, int32_t D, int64_t ld_hist,
                                 int32_t* plan, int64_t plan_cap, int32_t* n_attn, int32_t* n_merge,
                                 size_t* workspace_bytes) {
  if (n_attn) *n_attn = 0;
  if (n_merge) *n_merge = 0;
  if (workspace_bytes) *workspace_bytes = 0;
  if (n_groups < 0 || n_str < 0 || T < 0 || n_prefix < 0)
    return fail(CS_ERR_INVALID, "cs_prefix_attention_plan: negative size");
  if (n_groups == 0 || n_str == 0 || T == 0) return 0;
  if (!prefix_len || Hkv <= 0 || H <= 0 || H % Hkv != 0 || ld_hist <= 0 || ld_hist % kKeyBlock != 0 ||
      (D != 64 && D != 128 && D != 256))
    return fail(CS_ERR_INVALID, "cs_prefix_attention_plan: bad shape");
  const int64_t rep = H / Hkv;
  const int64_t M = static_cast<int64_t>(n_str) * T * rep;
  const int64_t n_qg = (M + kGroupRows - 1) / kGroupRows;
  const int64_t base = static_cast<int64_t>(n_groups) * Hkv * n_qg;
  // enough workgroups without key splits -- unless (single-token streams) some cells are
  // far longer than the rest: a lookahead tree level whose reference prompt lists every
  // opinion (thousands of keys) beside ~250-key agent prompts makes the reference cells
  // the launch's long pole (cells checked below)
  if (base >= kPlanMinBase && T > 1) return 0;
  const int64_t nbh_max = ld_hist / kKeyBlock;
  // every cell's key blocks per query tile (an upper bound: history at capacity)
  struct Cell { int32_t gi, qg; int64_t items, kw, nrows; };
  std::vector<Cell> cl;
  cl.reserve(static_cast<size_t>(n_groups * n_qg));
  for (int32_t gi = 0; gi < n_groups; ++gi) {
    const int32_t p = group_prefix ? group_prefix[gi] : gi;
    if (p < 0 || p >= n_prefix || prefix_len[p] < 0)
      return fail(CS_ERR_INVALID, "cs_prefix_attention_plan: group_prefix / prefix_len out of range");
    const int64_t nbp = (prefix_len[p] + kKeyBlock - 1) / kKeyBlock;
    for (int64_t qg = 0; qg < n_qg; ++qg) {
      const int64_t r0 = qg * kGroupRows;
      const int64_t nrows = std::min<int64_t>(kGroupRows, M - r0);
      const int64_t n_qt = (nrows + 15) / 16;
      const int64_t kw = n_qt == 1 ? 4 : (n_qt == 2 ? 2 : 1);
      int64_t items = 0;
      for (int64_t q = 0; q < n_qt; ++q) {
        const int64_t rt0 = r0 + 16 * q, rt1 = std::min(rt0 + 15, M - 1);
        const int64_t streams = (rt1 / rep) / T - (rt0 / rep) / T + 1;
        items = std::max(items, nbp + streams * nbh_max);
      }
      cl.push_back({gi, static_cast<int32_t>(qg), items, kw, nrows});
    }
  }
  if (base >= kPlanMinBase) {
    int64_t sum = 0, mx = 0;
    for (const Cell& c : cl) {
      sum += c.items;
      mx = std::max(mx, c.items);
    }
    if (mx * static_cast<int64_t>(cl.size()) <= kPlanImbalance * sum) return 0;
  }
  // one per-wave budget q for all cells (a cell of `items` blocks on kw waves takes
  // ceil(items / (q kw)) splits, at most kMaxSplit): the whole launch's wave-serial work
  // spread over about attn_target_wgs() workgroups, never below attn_min_items() blocks per
  // wave — so the split workgroups are about equally long and no cell is the long pole
  auto splits_of = [](const Cell& c, int64_t q) {
    return std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, (c.items + q * c.kw - 1) / (q * c.kw)));
  };
  int64_t work = 0;
  for (const Cell& c : cl) work += (c.items + c.kw - 1) / c.kw;
  work *= Hkv;
  const int64_t q = std::max<int64_t>(attn_min_items(), (work + attn_target_wgs() - 1) / attn_target_wgs());
  std::vector<PlanCell> cells;
  cells.reserve(cl.size());
  int64_t na = 0, nm = 0, slots = 0;
  for (const Cell& c : cl) {
    const int64_t s = splits_of(c, q);
    const int64_t per = (c.items + s * c.kw - 1) / (s * c.kw);
    cells.push_back({c.gi, c.qg, static_cast<int32_t>(s), static_cast<int32_t>(per)});
    na += s * Hkv;
    if (s > 1) {
      slots += s * Hkv;
      nm += (c.nrows + kMergeRows - 1) / kMergeRows * Hkv;
    }
  }
  if (nm == 0) return 0;   // no cell splits: the plain grid
  if (na + nm > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_prefix_attention_plan: plan too large");
  if (n_attn) *n_attn = static_cast<int32_t>(na);
  if (n_merge) *n_merge = static_cast<int32_t>(nm);
  if (workspace_bytes) *workspace_bytes = static_cast<size_t>(slots) * kGroupRows * (D + 2) * sizeof(float);
  const int64_t total = na + nm;
  if (!plan) return total;
  if (plan_cap < total) return fail(CS_ERR_INVALID, "cs_prefix_attention_plan: plan_cap too small");
  // the longest workgroups first (dispatched first: the tail of the launch is short ones)
  std::stable_sort(cells.begin(), cells.end(),
                   [](const PlanCell& x, const PlanCell& y) { return x.per_wg > y.per_wg; });
  int32_t* pa = plan;
  int32_t* pm = plan + 4 * na;
  int32_t slot = 0;
  for (const PlanCell& c : cells) {
    const int64_t r0 = static_cast<int64_t>(c.qg) * kGroupRows;
    const int64_t nrows = std::min<int64_t>(kGroupRows, M - r0);
    for (int32_t g = 0; g < Hkv; ++g) {
      const int32_t pg = c.gi * Hkv + g;
      for (int32_t sp = 0; sp < c.splits; ++sp) {
        pa[0] = pg;
        pa[1] = c.qg;
        pa[2] = sp | (c.splits << 8);
        pa[3] = c.splits > 1 ? slot + sp : 0;
        pa += 4;
      }
      if (c.splits > 1) {
        for (int32_t ch = 0; ch < (nrows + kMergeRows - 1) / kMergeRows; ++ch) {
          pm[0] = pg;
          pm[1] = c.qg;
          pm[2] = slot;
          pm[3] = ch | (c.splits << 8);
          pm += 4;
        }
        slot += c.splits;
      }
    }
  }
  return total;
}

}  // extern "C"

namespace {
// hist_rows == nullptr: cs_prefix_attention (V^T tiles); else cs_prefix_attention_rows
int prefix_attention_impl(const char* name, const void* q, const void* k_prefix, const void* vt_prefix,
                          int64_t ld_prefix, const int64_t* prefix_off, const int32_t* prefix_len,
                          int32_t max_prefix_len, const int32_t* group_prefix, int32_t n_groups,
                          const void* k_hist, const void* vt_hist, const int32_t* hist_rows,
                          int64_t ld_hist, const int32_t* hist_base, int32_t n_str, int32_t T,
                          int32_t H, int32_t Hkv, int32_t D, float scale, float softcap,
                          int32_t window, const void* plan, int32_t n_attn, int32_t n_merge,
                          void* out, void* workspace, size_t workspace_bytes, cs_stream_t stream) {
  const std::string nm(name);
  if (n_groups < 0 || n_str < 0 || T < 0) return fail(CS_ERR_INVALID, nm + ": negative size");
  if (n_groups == 0 || n_str == 0 || T == 0) return CS_OK;
  if (Hkv <= 0 || H <= 0 || H % Hkv != 0 || H / Hkv > 64)
    return fail(CS_ERR_INVALID, nm + ": H must be a multiple of Hkv (<= 64 per group)");
  if (D != 64 && D != 128 && D != 256)
    return fail(CS_ERR_INVALID, nm + ": head_dim must be 64, 128 or 256");
  if (ld_prefix <= 0 || ld_prefix % kKeyBlock != 0 || ld_hist <= 0 || ld_hist % kKeyBlock != 0)
    return fail(CS_ERR_INVALID, nm + ": ld_prefix / ld_hist must be positive multiples of 32");
  if (max_prefix_len < 0 || max_prefix_len > ld_prefix)
    return fail(CS_ERR_INVALID, nm + ": max_prefix_len outside [0, ld_prefix]");
  if (!q || !k_prefix || !vt_prefix || !prefix_off || !prefix_len || !k_hist || !vt_hist ||
      !hist_base || !out || (hist_rows == nullptr) != (nm == "cs_prefix_attention"))
    return fail(CS_ERR_INVALID, nm + ": NULL pointer");
  if (!(scale > 0.0f) || softcap < 0.0f) return fail(CS_ERR_INVALID, nm + ": bad scale / softcap");
  if (plan && (n_attn <= 0 || n_merge <= 0))
    return fail(CS_ERR_INVALID, nm + ": a plan needs n_attn > 0 and n_merge > 0");
  if (plan && !workspace)
    return fail(CS_ERR_WORKSPACE, nm + ": a plan needs the workspace cs_prefix_attention_plan() sized");
  const int64_t M = static_cast<int64_t>(n_str) * T * (H / Hkv);
  const int64_t n_qg = (M + kGroupRows - 1) / kGroupRows;
  const int64_t base = static_cast<int64_t>(n_groups) * Hkv * n_qg;
  if (n_qg > 0x7fffffff || base > 0x7fffffffLL) return fail(CS_ERR_INVALID, nm + ": too many query rows");
  AttnParams a;
  a.q = static_cast<const __bf16*>(q);
  a.kp = static_cast<const __bf16*>(k_prefix);
  a.vtp = static_cast<const __bf16*>(vt_prefix);
  a.poff = prefix_off;
  a.plen = prefix_len;
  a.gpfx = group_prefix;
  a.kh = static_cast<const __bf16*>(k_hist);
  a.vth = static_cast<const __bf16*>(vt_hist);
  a.hist_base = hist_base;
  a.hrow = hist_rows;
  a.out = static_cast<__bf16*>(out);
  a.part = static_cast<float*>(workspace);
  a.plan = static_cast<const int4*>(plan);
  a.ldp = ld_prefix;
  a.ldh = ld_hist;
  a.n_grp = n_groups;
  a.n_str = n_str;
  a.T = T;
  a.H = H;
  a.Hkv = Hkv;
  a.rep = H / Hkv;
  a.n_qg = static_cast<int32_t>(n_qg);
  a.n_attn = plan ? n_attn : 0;
  a.scale = scale;
  a.softcap = softcap;
  a.inv_softcap = softcap > 0.0f ? 1.0f / softcap : 0.0f;
  a.window = window > 0 ? window : 0;
  (void)workspace_bytes;   // sized by cs_prefix_attention_plan for this plan
  const int64_t nwg = plan ? n_attn : base;
  a.swizzle = (!plan && nwg % 8 == 0 && nwg >= 64) ? 1 : 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<uint32_t>(nwg));
  const dim3 merge_grid(static_cast<uint32_t>(plan ? n_merge : 0));
#define CS_ATTN_LAUNCH(DV)                                                              \
  do {                                                                                  \
    if (hist_rows)                                                                      \
      hipLaunchKernelGGL((prefix_attn_plan_lds_kernel<DV, true>), grid, dim3(kAttnThreads), 0, st, a); \
    else if (plan && attn_plan_lds())                                                        \
      hipLaunchKernelGGL(prefix_attn_plan_lds_kernel<DV>, grid, dim3(kAttnThreads), 0, st, a); \
    else if (plan)                                                                      \
      hipLaunchKernelGGL((prefix_attn_kernel<DV, true>), grid, dim3(kAttnThreads), 0, st, a); \
    else if (attn_lds())                                                                \
      hipLaunchKernelGGL(prefix_attn_lds_kernel<DV>, grid, dim3(kAttnThreads), 0, st, a); \
    else                                                                                \
      hipLaunchKernelGGL((prefix_attn_kernel<DV, false>), grid, dim3(kAttnThreads), 0, st, a); \
    if (plan)                                                                           \
      hipLaunchKernelGGL(attn_merge_kernel<DV>, merge_grid, dim3(kAttnThreads), 0, st, a); \
  } while (0)
  if (D == 64) {
    CS_ATTN_LAUNCH(64);
  } else if (D == 128) {
    CS_ATTN_LAUNCH(128);
  } else {
    CS_ATTN_LAUNCH(256);
  }
#undef CS_ATTN_LAUNCH
  return check_launch(name);
}
}  // namespace

extern "C" {

int cs_prefix_attention(const void* q, const void* k_prefix, const void* vt_prefix,
                        int64_t ld_prefix, const int64_t* prefix_off, const int32_t* prefix_len,
                        int32_t max_prefix_len, const int32_t* group_prefix, int32_t n_groups,
                        const void* k_hist, const void* vt_hist, int64_t ld_hist,
                        const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H, int32_t Hkv,
                        int32_t D, float scale, float softcap, int32_t window, const void* plan,
                        int32_t n_attn, int32_t n_merge, void* out, void* workspace,
                        size_t workspace_bytes, cs_stream_t stream) {
  return prefix_attention_impl("cs_prefix_attention", q, k_prefix, vt_prefix, ld_prefix, prefix_off,
                               prefix_len, max_prefix_len, group_prefix, n_groups, k_hist, vt_hist,
                               nullptr, ld_hist, hist_base, n_str, T, H, Hkv, D, scale, softcap,
                               window, plan, n_attn, n_merge, out, workspace, workspace_bytes, stream);
}

int cs_prefix_attention_rows(const void* q, const void* k_prefix, const void* vt_prefix,
                             int64_t ld_prefix, const int64_t* prefix_off, const int32_t* prefix_len,
                             int32_t max_prefix_len, const int32_t* group_prefix, int32_t n_groups,
                             const void* k_hist, const void* v_hist, const int32_t* hist_rows,
                             int64_t ld_hist, const int32_t* hist_base, int32_t n_str, int32_t T,
                             int32_t H, int32_t Hkv, int32_t D, float scale, float softcap,
                             int32_t window, const void* plan, int32_t n_attn, int32_t n_merge,
                             void* out, void* workspace, size_t workspace_bytes, cs_stream_t stream) {
  if (!hist_rows) return fail(CS_ERR_INVALID, "cs_prefix_attention_rows: NULL hist_rows");
  return prefix_attention_impl("cs_prefix_attention_rows", q, k_prefix, vt_prefix, ld_prefix,
                               prefix_off, prefix_len, max_prefix_len, group_prefix, n_groups,
                               k_hist, v_hist, hist_rows, ld_hist, hist_base, n_str, T, H, Hkv, D,
                               scale, softcap, window, plan, n_attn, n_merge, out, workspace,
                               workspace_bytes, stream);
}

#ifdef CS_TRACE_ATTN
// diagnostics build only: copy the per-workgroup timestamps [kAttTraceWgs][8] and clear them
int cs_attn_trace_read(unsigned long long* out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_attn_ts), sizeof(g_attn_ts));
  static unsigned long long zero[kAttTraceWgs][8];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_ts), zero, sizeof(zero));
  return 0;
}
#endif

int cs_hist_rows_update(const int32_t* src_rows, int32_t* dst_rows, const int64_t* parent,
                        const int32_t* hist_base, int64_t S, int32_t ld_hist, int64_t row_base,
                        int64_t n_rows, cs_stream_t stream) {
  if (S < 0 || ld_hist <= 0 || row_base < 0) return fail(CS_ERR_INVALID, "cs_hist_rows_update: bad shape");
  if (row_base + S > n_rows)
    return fail(CS_ERR_INVALID, "cs_hist_rows_update: rows row_base .. row_base + S - 1 exceed the buffer's n_rows");
  if (S == 0) return CS_OK;
  if (!src_rows || !dst_rows || !parent || !hist_base)
    return fail(CS_ERR_INVALID, "cs_hist_rows_update: NULL pointer");
  if (src_rows == dst_rows) return fail(CS_ERR_INVALID, "cs_hist_rows_update: source and destination must differ");
  if (S > 0x7fffffffLL || row_base + S > 0x7fffffffLL || (S * ld_hist + 255) / 256 > 0x7fffffffLL)
    return fail(CS_ERR_INVALID, "cs_hist_rows_update: table too large");
  hipLaunchKernelGGL(hist_rows_kernel, dim3(static_cast<uint32_t>((S * ld_hist + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), src_rows, dst_rows, parent, hist_base, S, ld_hist,
                     row_base);
  return check_launch("cs_hist_rows_update");
}

}  // extern "C"

namespace {
int rope_place_impl(const void* qkv, int64_t ld_qkv, const float* part, int32_t splits,
                    const float* inv_freq, const int32_t* prefix_len, const int32_t* group_prefix,
                    int32_t n_groups, const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H,
                    int32_t Hkv, int32_t D, void* q_out, void* k_hist, void* vt_hist,
                    int64_t ld_hist, int32_t v_rows, cs_stream_t stream);
}  // namespace

extern "C" {

int cs_rope_place(const void* qkv, int64_t ld_qkv, const float* inv_freq, const int32_t* prefix_len,
                  const int32_t* group_prefix, int32_t n_groups, const int32_t* hist_base,
                  int32_t n_str, int32_t T, int32_t H, int32_t Hkv, int32_t D, void* q_out,
                  void* k_hist, void* vt_hist, int64_t ld_hist, cs_stream_t stream) {
  if (!qkv) return fail(CS_ERR_INVALID, "cs_rope_place: NULL pointer");
  return rope_place_impl(qkv, ld_qkv, nullptr, 1, inv_freq, prefix_len, group_prefix, n_groups,
                         hist_base, n_str, T, H, Hkv, D, q_out, k_hist, vt_hist, ld_hist, 0, stream);
}

int cs_rope_place_rows(const void* qkv, int64_t ld_qkv, const float* inv_freq,
                       const int32_t* prefix_len, const int32_t* group_prefix, int32_t n_groups,
                       const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H, int32_t Hkv,
                       int32_t D, void* q_out, void* k_hist, void* v_hist, int64_t ld_hist,
                       cs_stream_t stream) {
  if (!qkv) return fail(CS_ERR_INVALID, "cs_rope_place_rows: NULL pointer");
  return rope_place_impl(qkv, ld_qkv, nullptr, 1, inv_freq, prefix_len, group_prefix, n_groups,
                         hist_base, n_str, T, H, Hkv, D, q_out, k_hist, v_hist, ld_hist, 1, stream);
}

int cs_rope_place_splitk(const float* part, int32_t splits, const float* inv_freq,
                         const int32_t* prefix_len, const int32_t* group_prefix, int32_t n_groups,
                         const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H,
                         int32_t Hkv, int32_t D, void* q_out, void* k_hist, void* vt_hist,
                         int64_t ld_hist, cs_stream_t stream) {
  if (!part || splits < 1) return fail(CS_ERR_INVALID, "cs_rope_place_splitk: need partials, splits >= 1");
  if (T >= 32) return fail(CS_ERR_INVALID, "cs_rope_place_splitk: T < 32 only (fold first for chunks)");
  if (reinterpret_cast<uintptr_t>(part) % 16 || D % 16)
    return fail(CS_ERR_INVALID, "cs_rope_place_splitk: partials 16-byte aligned, head_dim % 16 == 0");
  return rope_place_impl(nullptr, static_cast<int64_t>(H + 2 * Hkv) * D, part, splits, inv_freq,
                         prefix_len, group_prefix, n_groups, hist_base, n_str, T, H, Hkv, D, q_out,
                         k_hist, vt_hist, ld_hist, 0, stream);
}

int cs_rope_place_splitk_rows(const float* part, int32_t splits, const float* inv_freq,
                              const int32_t* prefix_len, const int32_t* group_prefix,
                              int32_t n_groups, const int32_t* hist_base, int32_t n_str, int32_t T,
                              int32_t H, int32_t Hkv, int32_t D, void* q_out, void* k_hist,
                              void* v_hist, int64_t ld_hist, cs_stream_t stream) {
  if (!part || splits < 1) return fail(CS_ERR_INVALID, "cs_rope_place_splitk_rows: need partials, splits >= 1");
  if (T >= 32) return fail(CS_ERR_INVALID, "cs_rope_place_splitk_rows: T < 32 only (fold first for chunks)");
  if (reinterpret_cast<uintptr_t>(part) % 16 || D % 16)
    return fail(CS_ERR_INVALID, "cs_rope_place_splitk_rows: partials 16-byte aligned, head_dim % 16 == 0");
  return rope_place_impl(nullptr, static_cast<int64_t>(H + 2 * Hkv) * D, part, splits, inv_freq,
                         prefix_len, group_prefix, n_groups, hist_base, n_str, T, H, Hkv, D, q_out,
                         k_hist, v_hist, ld_hist, 1, stream);
}

}  // extern "C"

namespace {
int rope_place_impl(const void* qkv, int64_t ld_qkv, const float* part, int32_t splits,
                    const float* inv_freq, const int32_t* prefix_len, const int32_t* group_prefix,
                    int32_t n_groups, const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H,
                    int32_t Hkv, int32_t D, void* q_out, void* k_hist, void* vt_hist,
                    int64_t ld_hist, int32_t v_rows, cs_stream_t stream) {
  if (n_groups < 0 || n_str < 0 || T < 0) return fail(CS_ERR_INVALID, "cs_rope_place: negative size");
  if (n_groups == 0 || n_str == 0 || T == 0) return CS_OK;
  if (H <= 0 || Hkv <= 0 || D <= 0 || D % 2 != 0 || ld_qkv < static_cast<int64_t>(H + 2 * Hkv) * D)
    return fail(CS_ERR_INVALID, "cs_rope_place: bad head layout");
  if (ld_hist < T) return fail(CS_ERR_INVALID, "cs_rope_place: ld_hist < T");
  if (!inv_freq || !prefix_len || !hist_base || !q_out || !k_hist || !vt_hist)
    return fail(CS_ERR_INVALID, "cs_rope_place: NULL pointer");
  RopeParams r;
  r.qkv = static_cast<const __bf16*>(qkv);
  r.ldqkv = ld_qkv;
  r.part = part;
  r.splits = splits;
  r.inv_freq = inv_freq;
  r.plen = prefix_len;
  r.gpfx = group_prefix;
  r.hist_base = hist_base;
  r.q_out = static_cast<__bf16*>(q_out);
  r.kh = static_cast<__bf16*>(k_hist);
  r.vth = static_cast<__bf16*>(vt_hist);
  r.ldh = ld_hist;
  r.v_rows = v_rows;
  r.n_tok = static_cast<int64_t>(n_groups) * n_str * T;
  r.n_str = n_str;
  r.T = T;
  r.H = H;
  r.Hkv = Hkv;
  r.D = D;
  if (D % 8 != 0 || D > 256) return fail(CS_ERR_INVALID, "cs_rope_place: head_dim must be a multiple of 8, <= 256");
  if (r.n_tok > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_rope_place: too many tokens");
  // V by 32-slot tiles when the streams carry many tokens (CS_ROPE_VTILE=0: per token)
  const int64_t n_tiles = ld_hist / 32;
  const int64_t n_vwg = static_cast<int64_t>(n_groups) * n_str * Hkv * n_tiles;
  {
    static const bool vtile = env_int("CS_ROPE_VTILE", 1, 0, 1) != 0;   // read once
    r.skip_v = (!part && !v_rows && T >= 32 && ld_hist % 32 == 0 && ld_qkv % 8 == 0 &&
                reinterpret_cast<uintptr_t>(qkv) % 16 == 0 && n_vwg <= 0x7fffffffLL &&
                vtile) ? 1 : 0;
  }
  // 8-pair (16-byte) items when every head's halves are 16-byte aligned, else 4-pair
  const bool p8 = part ? true
                       : (ld_qkv % 8 == 0 && reinterpret_cast<uintptr_t>(qkv) % 16 == 0 && D % 16 == 0);
  const int64_t n_items = static_cast<int64_t>(H + 2 * Hkv) * (D / 2) / (p8 ? 8 : 4);
  const int64_t n_split = (n_items + kRopeItems - 1) / kRopeItems;
  if (r.n_tok * n_split > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_rope_place: too many tokens");
  const dim3 grid(static_cast<uint32_t>(r.n_tok * n_split));
  if (part && splits <= 2)
    hipLaunchKernelGGL((rope_place_kernel<8, true, 2>), grid, dim3(256), 0, static_cast<hipStream_t>(stream),
                       r, static_cast<int32_t>(n_split));
  else if (part && splits <= 4)
    hipLaunchKernelGGL((rope_place_kernel<8, true, 4>), grid, dim3(256), 0, static_cast<hipStream_t>(stream),
                       r, static_cast<int32_t>(n_split));
  else if (part)
    hipLaunchKernelGGL((rope_place_kernel<8, true, 8>), grid, dim3(256), 0, static_cast<hipStream_t>(stream),
                       r, static_cast<int32_t>(n_split));
  else if (p8)
    hipLaunchKernelGGL(rope_place_kernel<8>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), r,
                       static_cast<int32_t>(n_split));
  else
    hipLaunchKernelGGL(rope_place_kernel<4>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), r,
                       static_cast<int32_t>(n_split));
  if (r.skip_v)
    hipLaunchKernelGGL(v_tile_place_kernel, dim3(static_cast<uint32_t>(n_vwg)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), r, static_cast<int32_t>(n_tiles));
  return check_launch("cs_rope_place");
}
}  // namespace
