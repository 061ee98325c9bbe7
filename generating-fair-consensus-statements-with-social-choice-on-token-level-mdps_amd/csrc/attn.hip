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

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kAttnThreads = 256;   // 4 waves
constexpr int kGroupRows = 64;      // query rows per workgroup (4 tiles of 16)
constexpr int kKeyBlock = 32;
constexpr int kMaxSplit = 32;
constexpr int kItemsPerWave = 4;   // key blocks a wave walks before the work is split further

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
  __bf16* out;
  float* part;
  int64_t ldp, ldh;
  int32_t n_grp, n_str, T, H, Hkv, rep, n_qg, n_split;
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

// key blocks ("items") a 16-row query tile visits: the prefix blocks plus the history blocks
// of every stream with rows in the tile
__device__ __forceinline__ int tile_items(const AttnParams& a, int M, int rt0, int nbp, int hb) {
  const int rt1 = min(rt0 + 15, M - 1);
  const int b_lo = (rt0 / a.rep) / a.T, b_hi = (rt1 / a.rep) / a.T;
  const int t_hi = b_lo == b_hi ? (rt1 / a.rep) % a.T : a.T - 1;
  const int nbh = (min(hb + t_hi + 1, static_cast<int>(a.ldh)) + kKeyBlock - 1) / kKeyBlock;
  return nbp + (b_hi - b_lo + 1) * nbh;
}

// splits a (group, head, query group) uses: enough that no wave walks more than
// kItemsPerWave blocks, at most the grid's n_split (device-side, from the actual prefix
// length and history size; the merge recomputes the same number)
__device__ __forceinline__ int splits_used(const AttnParams& a, int M, int r0, int nbp, int hb) {
  const int nrows = min(kGroupRows, M - r0);
  const int n_qt = (nrows + 15) >> 4;
  const int kw = n_qt == 1 ? 4 : (n_qt == 2 ? 2 : 1);
  int items = 0;
  for (int q = 0; q < n_qt; ++q) items = max(items, tile_items(a, M, r0 + 16 * q, nbp, hb));
  const int per = kItemsPerWave * kw;
  return max(1, min(a.n_split, (items + per - 1) / per));
}

template <int D>
__global__ __launch_bounds__(kAttnThreads) void prefix_attn_kernel(AttnParams a) {
  constexpr int NDS = D / 32;   // 32-wide d steps of S^T = K . Q^T
  constexpr int NDT = D / 16;   // 16-row d tiles of O^T
  constexpr int LDSW = D + 2;   // per query row: O[D], m, l
  __shared__ float sm[3][16][LDSW];

  const int bid = logical_block(a.swizzle);
  const int split = bid % a.n_split;
  const int rest = bid / a.n_split;
  const int qg = rest % a.n_qg;
  const int pg = rest / a.n_qg;
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
  const int n_used = a.n_split == 1 ? 1 : splits_used(a, M, r0, nbp, hb);
  if (split >= n_used) return;                       // whole workgroup: uniform

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

  if (active) {
    const int nslot = n_used * kw;
    for (int it = split * kw + ks; it < n_items; it += nslot) {
      const __bf16* kbase;
      const __bf16* vbase;
      int64_t ldv;
      int kb, lim, pos0;
      if (it < nbp) {
        kb = it * kKeyBlock;
        const int64_t po = a.poff[p];
        kbase = a.kp + (static_cast<int64_t>(g) * a.ldp + po) * D;
        vbase = a.vtp + (static_cast<int64_t>(g) * a.ldp + po + kb) * D;   // the key block's tile
        ldv = kKeyBlock;
        lim = vrow ? pl : 0;
        pos0 = 0;
      } else {
        const int ih = it - nbp;
        const int bb = b_lo + ih / nbh;
        kb = (ih % nbh) * kKeyBlock;
        const int64_t sh = (static_cast<int64_t>(gi) * a.n_str + bb) * a.Hkv + g;
        kbase = a.kh + sh * a.ldh * D;
        vbase = a.vth + (sh * a.ldh + kb) * D;                              // the key block's tile
        ldv = kKeyBlock;
        lim = (vrow && bb == b) ? hv : 0;
        pos0 = pl;
      }
      // S^T tiles: keys kb + [0, 16) and kb + [16, 32)
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
      const __bf16* k0 = kbase + static_cast<int64_t>(kb + col) * D + 8 * h4;
      const __bf16* k1 = k0 + 16 * D;
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds) {
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(k0 + ds * 32);
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(k1 + ds * 32);
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, qf[ds], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, qf[ds], s1, 0, 0, 0);
      }
      float y[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[i] = s0[i];
        y[4 + i] = s1[i];
      }
      float bm = -INFINITY;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key = kb + (i >> 2) * 16 + 4 * h4 + (i & 3);
        float x = y[i] * a.scale;
        if (a.softcap > 0.0f) x = softcap_fn(x, a.softcap, a.inv_softcap);
        x *= kLog2e;
        y[i] = (key < lim && pos0 + key >= kmin_pos) ? x : -INFINITY;
        bm = fmaxf(bm, y[i]);
      }
      bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mn = fmaxf(m, bm);
      const bool none = mn == -INFINITY;
      const float alpha = none ? 1.0f : __builtin_amdgcn_exp2f(m - mn);
      float ps = 0.0f;
      bf16x8 pb;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float pv = none ? 0.0f : __builtin_amdgcn_exp2f(y[i] - mn);
        ps += pv;
        pb[i] = static_cast<__bf16>(pv);
      }
      l = fmaf(l, alpha, ps);
      m = mn;
      const __bf16* vrow0 = vbase + static_cast<int64_t>(col) * ldv + 4 * h4;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const __bf16* vp = vrow0 + static_cast<int64_t>(dt * 16) * ldv;
        const bf16x4 lo = *reinterpret_cast<const bf16x4*>(vp);
        const bf16x4 hi = *reinterpret_cast<const bf16x4*>(vp + 16);
        const bf16x8 va = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[dt] *= alpha;
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[dt], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);

  // waves that share a query tile combine through LDS (fixed order: ks = 0, 1, ...)
  if (kw > 1) {
    if (active && ks > 0) {
      const int slot = w - n_qt;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sm[slot][col][dt * 16 + 4 * h4 + i] = o[dt][i];
      if (h4 == 0) {
        sm[slot][col][D] = m;
        sm[slot][col][D + 1] = l;
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
        const int slot = qt + n_qt * k - n_qt;
        const float mk = sm[slot][col][D];
        const float ck = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(mk - mt);
        l = fmaf(sm[slot][col][D + 1], ck, l);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[dt][i] = fmaf(sm[slot][col][dt * 16 + 4 * h4 + i], ck, o[dt][i]);
      }
      m = mt;
    }
  }
  if (!vrow || ks != 0) return;
  if (a.n_split == 1) {
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
    float* pr = a.part + ((static_cast<int64_t>(pg) * a.n_qg + qg) * a.n_split + split) *
                             kGroupRows * LDSW +
                static_cast<int64_t>(qt * 16 + col) * LDSW;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
      *reinterpret_cast<f32x4*>(pr + dt * 16 + 4 * h4) = o[dt];
    if (h4 == 0) {
      pr[D] = m;
      pr[D + 1] = l;
    }
  }
}

// one workgroup per (group, head, query group): first one thread per row folds the splits'
// (m, l) into per-split weights (LDS), then every (row, 4-column chunk) sums the weighted
// partial outputs — all loads of a phase independent, fixed split order (deterministic)
template <int D>
__global__ __launch_bounds__(kAttnThreads) void attn_merge_kernel(AttnParams a) {
  constexpr int LDSW = D + 2;
  constexpr int NC = D / 4;
  __shared__ float wgt[kMaxSplit][kGroupRows];
  __shared__ float inv_l[kGroupRows];
  const int qg = blockIdx.x % a.n_qg;
  const int pg = blockIdx.x / a.n_qg;
  const int gi = pg / a.Hkv, g = pg % a.Hkv;
  const int M = a.n_str * a.T * a.rep;
  const int r0 = qg * kGroupRows;
  const int nrows = min(kGroupRows, M - r0);
  const int p = a.gpfx ? a.gpfx[gi] : gi;
  const int nbp = (a.plen[p] + kKeyBlock - 1) / kKeyBlock;
  const int n_used = splits_used(a, M, r0, nbp, *a.hist_base);
  const float* base = a.part + (static_cast<int64_t>(pg) * a.n_qg + qg) * a.n_split * kGroupRows * LDSW;
  for (int rl = threadIdx.x; rl < nrows; rl += kAttnThreads) {
    float mt = -INFINITY;
#pragma unroll 8
    for (int sp = 0; sp < n_used; ++sp) mt = fmaxf(mt, base[(sp * kGroupRows + rl) * LDSW + D]);
    float l = 0.0f;
#pragma unroll 8
    for (int sp = 0; sp < n_used; ++sp) {
      const float m = base[(sp * kGroupRows + rl) * LDSW + D];
      const float c = mt == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m - mt);
      wgt[sp][rl] = c;
      l = fmaf(base[(sp * kGroupRows + rl) * LDSW + D + 1], c, l);
    }
    inv_l[rl] = l > 0.0f ? 1.0f / l : 0.0f;
  }
  __syncthreads();
  for (int item = threadIdx.x; item < nrows * NC; item += kAttnThreads) {
    const int rl = item / NC, c4 = item % NC;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int sp = 0; sp < n_used; ++sp) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(base + (sp * kGroupRows + rl) * LDSW + 4 * c4);
      acc += v * wgt[sp][rl];
    }
    const float inv = inv_l[rl];
    const int row = r0 + rl;
    const int jh = row % a.rep, bt = row / a.rep;
    const int t = bt % a.T, b = bt / a.T;
    const int64_t tok = (static_cast<int64_t>(gi) * a.n_str + b) * a.T + t;
    bf16x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = static_cast<__bf16>(acc[i] * inv);
    *reinterpret_cast<bf16x4*>(a.out + (tok * a.H + g * a.rep + jh) * D + 4 * c4) = v;
  }
}

// RoPE (half-rotation convention) + placement.  One thread per (token, head, pair i < D/2).
struct RopeParams {
  const __bf16* qkv;
  int64_t ldqkv;
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
};

// one thread per (token, 4 consecutive rotation pairs): the 4 angles' sincos once, then
// every head of the token (q, k rotated; v placed) with 8-byte loads / stores
__global__ __launch_bounds__(256) void rope_place_kernel(RopeParams r) {
  const int half = r.D >> 1;
  const int nq = half >> 2;                         // 4-pair quads per head
  const int nh = r.H + 2 * r.Hkv;
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= r.n_tok * nq) return;
  const int i0 = 4 * static_cast<int>(idx % nq);
  const int64_t tok = idx / nq;
  const int64_t s = tok / r.T;
  const int t = static_cast<int>(tok % r.T);
  const int gi = static_cast<int>(s / r.n_str);
  const int p = r.gpfx ? r.gpfx[gi] : gi;
  const int slot = *r.hist_base + t;
  const float pos = static_cast<float>(r.plen[p] + slot);
  float cs[4], sn[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) sincosf(pos * r.inv_freq[i0 + e], &sn[e], &cs[e]);
  const __bf16* row = r.qkv + tok * r.ldqkv;
  for (int hh = 0; hh < nh; ++hh) {
    const __bf16* src = row + static_cast<int64_t>(hh) * r.D + i0;
    const bf16x4 a = *reinterpret_cast<const bf16x4*>(src);
    const bf16x4 b = *reinterpret_cast<const bf16x4*>(src + half);
    if (hh >= r.H + r.Hkv) {                         // v: transposed placement, no rotation
      const int g = hh - r.H - r.Hkv;
      __bf16* dst = r.vth + ((s * r.Hkv + g) * r.ldh + (slot & ~31)) * r.D +
                    static_cast<int64_t>(i0) * 32 + (slot & 31);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dst[e * 32] = a[e];
        dst[(half + e) * 32] = b[e];
      }
      continue;
    }
    bf16x4 y1, y2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x1 = static_cast<float>(a[e]), x2 = static_cast<float>(b[e]);
      y1[e] = static_cast<__bf16>(fmaf(x1, cs[e], -x2 * sn[e]));
      y2[e] = static_cast<__bf16>(fmaf(x2, cs[e], x1 * sn[e]));
    }
    __bf16* dst = hh < r.H ? r.q_out + (tok * r.H + hh) * r.D
                           : r.kh + ((s * r.Hkv + (hh - r.H)) * r.ldh + slot) * r.D;
    *reinterpret_cast<bf16x4*>(dst + i0) = y1;
    *reinterpret_cast<bf16x4*>(dst + half + i0) = y2;
  }
}

// Beam reordering of the per-stream history: dst[l][s] = src[l][parent[s]] for the filled
// slots only (j < *hist_base; V tiles rounded up to 32 slots).  One workgroup per (layer,
// stream), 16-byte vectors; the unfilled capacity is never moved.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void hist_gather_kernel(
    const __bf16* __restrict__ src_k, __bf16* __restrict__ dst_k, const __bf16* __restrict__ src_v,
    __bf16* __restrict__ dst_v, const int64_t* __restrict__ parent, const int32_t* __restrict__ hist_base,
    int64_t S, int32_t Hkv, int32_t ldh, int32_t D) {
  // one workgroup per (layer, stream, head)
  const int64_t lsg = blockIdx.x;
  const int g = static_cast<int>(lsg % Hkv);
  const int64_t ls = lsg / Hkv;
  const int64_t l = ls / S, s = ls % S;
  const int hb = min(*hist_base, ldh);
  if (hb <= 0) return;
  const int64_t p = parent[s];
  const int64_t per = static_cast<int64_t>(ldh) * D;                 // elements per (l, s, g)
  const int64_t so = ((l * S + p) * Hkv + g) * per, dn = ((l * S + s) * Hkv + g) * per;
  // K: hb * D contiguous elements
  const int kv = hb * D / 8;
  for (int i = threadIdx.x; i < kv; i += 256)
    reinterpret_cast<u32x4_t*>(dst_k + dn)[i] = reinterpret_cast<const u32x4_t*>(src_k + so)[i];
  // V^T tiles: the first ceil32(hb) slots are ceil32(hb) * D contiguous elements
  const int vv = ((hb + 31) & ~31) * D / 8;
  for (int i = threadIdx.x; i < vv; i += 256)
    reinterpret_cast<u32x4_t*>(dst_v + dn)[i] = reinterpret_cast<const u32x4_t*>(src_v + so)[i];
}

int attn_plan(int32_t n_grp, int32_t n_str, int32_t T, int32_t Hkv, int32_t rep, int64_t max_plen,
              int64_t ldh, int32_t* n_qg, int32_t* n_split) {
  const int64_t M = static_cast<int64_t>(n_str) * T * rep;
  const int64_t qg = (M + kGroupRows - 1) / kGroupRows;
  const int64_t base = static_cast<int64_t>(n_grp) * Hkv * qg;
  if (qg > 0x7fffffff || base > 0x7fffffff) return -1;
  *n_qg = static_cast<int32_t>(qg);
  int64_t ns = 1;
  if (base < 1024) {
    // an upper bound of the splits any (group, head, query group) uses: every prefix
    // block plus the history blocks of the <= 16 streams of a tile, kItemsPerWave per wave
    const int64_t streams = std::min<int64_t>(16, std::max<int64_t>(1, 16 / std::max<int64_t>(1, static_cast<int64_t>(T) * rep)));
    const int64_t items = (max_plen + kKeyBlock - 1) / kKeyBlock + streams * (ldh / kKeyBlock);
    ns = std::min<int64_t>((items + kItemsPerWave - 1) / kItemsPerWave, kMaxSplit);
  }
  *n_split = static_cast<int32_t>(std::max<int64_t>(ns, 1));
  return 0;
}

}  // namespace

extern "C" {

size_t cs_prefix_attention_workspace_size(int32_t n_groups, int32_t n_str, int32_t T, int32_t H,
                                          int32_t Hkv, int32_t D, int32_t max_prefix_len,
                                          int64_t ld_hist) {
  if (n_groups <= 0 || n_str <= 0 || T <= 0 || Hkv <= 0 || H % Hkv != 0) return 0;
  int32_t nqg = 0, ns = 0;
  if (attn_plan(n_groups, n_str, T, Hkv, H / Hkv, max_prefix_len, ld_hist, &nqg, &ns) != 0 || ns == 1)
    return 0;
  return static_cast<size_t>(n_groups) * Hkv * nqg * ns * kGroupRows * (D + 2) * sizeof(float);
}

int cs_prefix_attention(const void* q, const void* k_prefix, const void* vt_prefix,
                        int64_t ld_prefix, const int64_t* prefix_off, const int32_t* prefix_len,
                        int32_t max_prefix_len, const int32_t* group_prefix, int32_t n_groups,
                        const void* k_hist, const void* vt_hist, int64_t ld_hist,
                        const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H, int32_t Hkv,
                        int32_t D, float scale, float softcap, int32_t window, void* out,
                        void* workspace, size_t workspace_bytes, cs_stream_t stream) {
  if (n_groups < 0 || n_str < 0 || T < 0) return fail(CS_ERR_INVALID, "cs_prefix_attention: negative size");
  if (n_groups == 0 || n_str == 0 || T == 0) return CS_OK;
  if (Hkv <= 0 || H <= 0 || H % Hkv != 0 || H / Hkv > 64)
    return fail(CS_ERR_INVALID, "cs_prefix_attention: H must be a multiple of Hkv (<= 64 per group)");
  if (D != 64 && D != 128 && D != 256)
    return fail(CS_ERR_INVALID, "cs_prefix_attention: head_dim must be 64, 128 or 256");
  if (ld_prefix <= 0 || ld_prefix % kKeyBlock != 0 || ld_hist <= 0 || ld_hist % kKeyBlock != 0)
    return fail(CS_ERR_INVALID, "cs_prefix_attention: ld_prefix / ld_hist must be positive multiples of 32");
  if (max_prefix_len < 0 || max_prefix_len > ld_prefix)
    return fail(CS_ERR_INVALID, "cs_prefix_attention: max_prefix_len outside [0, ld_prefix]");
  if (!q || !k_prefix || !vt_prefix || !prefix_off || !prefix_len || !k_hist || !vt_hist ||
      !hist_base || !out)
    return fail(CS_ERR_INVALID, "cs_prefix_attention: NULL pointer");
  if (!(scale > 0.0f) || softcap < 0.0f) return fail(CS_ERR_INVALID, "cs_prefix_attention: bad scale / softcap");
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
  a.out = static_cast<__bf16*>(out);
  a.ldp = ld_prefix;
  a.ldh = ld_hist;
  a.n_grp = n_groups;
  a.n_str = n_str;
  a.T = T;
  a.H = H;
  a.Hkv = Hkv;
  a.rep = H / Hkv;
  a.scale = scale;
  a.softcap = softcap;
  a.inv_softcap = softcap > 0.0f ? 1.0f / softcap : 0.0f;
  a.window = window > 0 ? window : 0;
  if (attn_plan(n_groups, n_str, T, Hkv, a.rep, max_prefix_len, ld_hist, &a.n_qg, &a.n_split) != 0)
    return fail(CS_ERR_INVALID, "cs_prefix_attention: too many query rows");
  const int64_t nwg = static_cast<int64_t>(n_groups) * Hkv * a.n_qg * a.n_split;
  if (nwg > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_prefix_attention: grid too large");
  a.part = nullptr;
  if (a.n_split > 1) {
    const size_t need =
        cs_prefix_attention_workspace_size(n_groups, n_str, T, H, Hkv, D, max_prefix_len, ld_hist);
    if (!workspace || workspace_bytes < need)
      return fail(CS_ERR_WORKSPACE, "cs_prefix_attention: workspace smaller than "
                                    "cs_prefix_attention_workspace_size()");
    a.part = static_cast<float*>(workspace);
  }
  a.swizzle = (nwg % 8 == 0 && nwg >= 64) ? 1 : 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<uint32_t>(nwg));
  const dim3 merge_grid(static_cast<uint32_t>(static_cast<int64_t>(n_groups) * Hkv * a.n_qg));
#define CS_ATTN_LAUNCH(DV)                                                              \
  do {                                                                                  \
    hipLaunchKernelGGL(prefix_attn_kernel<DV>, grid, dim3(kAttnThreads), 0, st, a);      \
    if (a.n_split > 1)                                                                  \
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
  return check_launch("cs_prefix_attention");
}

int cs_hist_gather(const void* src_k, void* dst_k, const void* src_vt, void* dst_vt,
                   const int64_t* parent, const int32_t* hist_base, int64_t L, int64_t S,
                   int32_t Hkv, int32_t ld_hist, int32_t D, cs_stream_t stream) {
  if (L < 0 || S < 0 || Hkv <= 0 || D <= 0) return fail(CS_ERR_INVALID, "cs_hist_gather: bad shape");
  if (L == 0 || S == 0) return CS_OK;
  if (!src_k || !dst_k || !src_vt || !dst_vt || !parent || !hist_base)
    return fail(CS_ERR_INVALID, "cs_hist_gather: NULL pointer");
  if (ld_hist <= 0 || ld_hist % 8 || D % 8)
    return fail(CS_ERR_INVALID, "cs_hist_gather: ld_hist and D must be positive multiples of 8");
  if (src_k == dst_k || src_vt == dst_vt)
    return fail(CS_ERR_INVALID, "cs_hist_gather: source and destination must differ (ping-pong)");
  if (L * S * Hkv > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_hist_gather: grid too large");
  hipLaunchKernelGGL(hist_gather_kernel, dim3(static_cast<uint32_t>(L * S * Hkv)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const __bf16*>(src_k),
                     static_cast<__bf16*>(dst_k), static_cast<const __bf16*>(src_vt),
                     static_cast<__bf16*>(dst_vt), parent, hist_base, S, Hkv, ld_hist, D);
  return check_launch("cs_hist_gather");
}

int cs_rope_place(const void* qkv, int64_t ld_qkv, const float* inv_freq, const int32_t* prefix_len,
                  const int32_t* group_prefix, int32_t n_groups, const int32_t* hist_base,
                  int32_t n_str, int32_t T, int32_t H, int32_t Hkv, int32_t D, void* q_out,
                  void* k_hist, void* vt_hist, int64_t ld_hist, cs_stream_t stream) {
  if (n_groups < 0 || n_str < 0 || T < 0) return fail(CS_ERR_INVALID, "cs_rope_place: negative size");
  if (n_groups == 0 || n_str == 0 || T == 0) return CS_OK;
  if (H <= 0 || Hkv <= 0 || D <= 0 || D % 2 != 0 || ld_qkv < static_cast<int64_t>(H + 2 * Hkv) * D)
    return fail(CS_ERR_INVALID, "cs_rope_place: bad head layout");
  if (ld_hist < T) return fail(CS_ERR_INVALID, "cs_rope_place: ld_hist < T");
  if (!qkv || !inv_freq || !prefix_len || !hist_base || !q_out || !k_hist || !vt_hist)
    return fail(CS_ERR_INVALID, "cs_rope_place: NULL pointer");
  RopeParams r;
  r.qkv = static_cast<const __bf16*>(qkv);
  r.ldqkv = ld_qkv;
  r.inv_freq = inv_freq;
  r.plen = prefix_len;
  r.gpfx = group_prefix;
  r.hist_base = hist_base;
  r.q_out = static_cast<__bf16*>(q_out);
  r.kh = static_cast<__bf16*>(k_hist);
  r.vth = static_cast<__bf16*>(vt_hist);
  r.ldh = ld_hist;
  r.n_tok = static_cast<int64_t>(n_groups) * n_str * T;
  r.n_str = n_str;
  r.T = T;
  r.H = H;
  r.Hkv = Hkv;
  r.D = D;
  if (D % 8 != 0) return fail(CS_ERR_INVALID, "cs_rope_place: head_dim must be a multiple of 8");
  const int64_t total = r.n_tok * (D / 8);
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_rope_place: too many elements");
  hipLaunchKernelGGL(rope_place_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), r);
  return check_launch("cs_rope_place");
}

}  // extern "C"
