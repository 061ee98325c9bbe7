// gemm.hip — the projection GEMMs of a decode step, Y[M, N] = X[M, K] · W[N, K]^T in bf16
// with fp32 accumulation, for the row counts a step has (M = agents x beams + reference
// rows: C1 20, C3 272, C5 520): too many rows for a GEMV, too few for a square tile.
//
// What it replaces: the remote forward behind every get_prompt_logprobs call
// (src/utils.py:249-259) re-encodes each (agent, candidate) text; here one step of all
// (agent, beam) streams runs the weights of every layer once, so the layer's time is a
// weight stream (C3: 397 MB per layer) with M MACs per weight element — balanced between
// HBM (8 TB/s) and MFMA (2.5 PF dense) at M ~ 272.
//
// ws_gemm_kernel<MW>: one workgroup (8 waves: 2 row groups x 4 column groups) owns 128
// output features x 32*MW rows (all of a step's rows up to 288) over a K range:
//   * W (the streamed operand, read from HBM exactly once per row block) goes straight
//     from global memory into MFMA A-fragments (16 B per lane, 16 rows x 64 B per wave
//     instruction), a three-stage register ring per 64-deep K step;
//   * X (L2-resident: 2-8 MB, re-read by every column tile) is staged through LDS in
//     three buffers by plain 16-byte loads + ds_write_b128, 128-B rows with a 16-B chunk
//     XOR swizzle (chunk ^ (row >> 1) & 7) so the B-fragment ds_read_b128 of 16 rows is
//     bank-conflict free;
//   * v_mfma_f32_16x16x32_bf16 computes the transposed tile D[n][m] (A = W rows, B = X^T):
//     each lane ends with 4 consecutive features of one row -> one 8-byte store.
// Split-K (grid splits x column tiles) writes fp32 partials [split][M][N], folded in split
// order by splitk_reduce_kernel: the result does not depend on scheduling.  The gated
// variant (GATED = 1) pairs gate feature f with up feature F + f in the same wave and
// writes act(gate) * up (the rounding of cs_gated_act) instead of both halves.
#include "cs_kernels.cuh"

#include <utility>

namespace {

typedef __bf16 gbf16x8 __attribute__((ext_vector_type(8)));
typedef float gf32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t gu32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t gu16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t gu16x8 __attribute__((ext_vector_type(8)));

constexpr int kGemmThreads = 512;   // 8 waves: 2 row groups x 4 column groups
constexpr int kGemmBN = 128;        // output features (W rows) per workgroup
constexpr int kGemmBK = 64;         // K per stage (one 128-B row of X per stage)
constexpr int kGemmMaxMW = 9;       // 16-row tiles per wave: up to 288 rows per workgroup

__device__ __forceinline__ float gbf(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }

__device__ __forceinline__ uint16_t gto_bf(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);
  return static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ float g_silu(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float g_gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

// byte offset of 16-B chunk c (0..7) of X-tile row r in one LDS stage
__device__ __forceinline__ int x_swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int MW>
struct WsShape {
  static constexpr int kRows = 32 * MW;
  static constexpr int kStageBytes = kRows * 128;
  static constexpr int kChunks = kRows * 8;
  static constexpr int kCPT = (kChunks + kGemmThreads - 1) / kGemmThreads;
};

// grid: n_tiles x splits x m_blocks (flattened, column tile fastest).  nk = K steps per split.
// GATED: W rows [0, F) gate, [F, 2F) up (F = N / 2 = gate_off); a tile covers 64 features of
// each; Y is [M, F].  P != nullptr: fp32 partial [split][M][n_out] instead of Y.
template <int MW, int GATED>
__global__ __launch_bounds__(kGemmThreads, 1) void ws_gemm_kernel(
    const uint16_t* __restrict__ X, int64_t ldx, const uint16_t* __restrict__ W, int64_t ldw,
    uint16_t* __restrict__ Y, int64_t ldy, float* __restrict__ P, int64_t M, int64_t n_out,
    int64_t gate_off, int nk, int n_tiles, int splits, int act) {
  using S = WsShape<MW>;
  __shared__ __align__(16) unsigned char lds[3 * S::kStageBytes];

  const int bid = blockIdx.x;
  const int nt = bid % n_tiles;
  const int sp = (bid / n_tiles) % splits;
  const int mb = bid / (n_tiles * splits);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int wm = wv >> 2;          // row group (MW tiles of 16 rows)
  const int wn = wv & 3;           // column group
  const int64_t m0 = static_cast<int64_t>(mb) * S::kRows;
  const int64_t kbase = static_cast<int64_t>(sp) * nk * kGemmBK;

  // this lane's two W rows (A-fragment rows) and its k offset inside a 32-deep sub-step
  int64_t wrow[2];
  if (GATED) {
    const int64_t f = static_cast<int64_t>(nt) * 64 + wn * 16 + (lane & 15);
    wrow[0] = f;
    wrow[1] = gate_off + f;
  } else {
    const int64_t n = static_cast<int64_t>(nt) * kGemmBN + wn * 32 + (lane & 15);
    wrow[0] = n;
    wrow[1] = n + 16;
  }
  const uint16_t* wp0 = W + wrow[0] * ldw + kbase + 8 * (lane >> 4);
  const uint16_t* wp1 = W + wrow[1] * ldw + kbase + 8 * (lane >> 4);

  // X staging: chunk q = tid + u * 512 -> tile row q >> 3, chunk q & 7.  Every lane loads
  // and stores (chunks past the tile repeat its last chunk: the same bytes to the same LDS
  // address), and every load is unconditional (K steps past the end re-read the last one,
  // from cache): straight-line code, so the compiler's counted vmcnt waits keep the loads
  // of later stages in flight instead of draining them at each branch join.
  const uint16_t* xp[S::kCPT];
  int xoff[S::kCPT];
#pragma unroll
  for (int u = 0; u < S::kCPT; ++u) {
    int q = tid + u * kGemmThreads;
    if (q > S::kChunks - 1) q = S::kChunks - 1;
    const int r = q >> 3;
    const int c = q & 7;
    int64_t gr = m0 + r;
    if (gr > M - 1) gr = M - 1;     // padded rows read a real row; their results are dropped
    xp[u] = X + gr * ldx + kbase + c * 8;
    xoff[u] = x_swz(r, c);
  }

  gf32x4 acc[MW][2];
#pragma unroll
  for (int i = 0; i < MW; ++i) {
    acc[i][0] = gf32x4{0.f, 0.f, 0.f, 0.f};
    acc[i][1] = gf32x4{0.f, 0.f, 0.f, 0.f};
  }

  auto load_x = [&](gu32x4 (&xs)[S::kCPT], int kt) {
    kt = kt < nk ? kt : nk - 1;
#pragma unroll
    for (int u = 0; u < S::kCPT; ++u) xs[u] = *reinterpret_cast<const gu32x4*>(xp[u] + kt * kGemmBK);
  };
  auto store_x = [&](const gu32x4 (&xs)[S::kCPT], int buf) {
#pragma unroll
    for (int u = 0; u < S::kCPT; ++u)
      *reinterpret_cast<gu32x4*>(lds + buf * S::kStageBytes + xoff[u]) = xs[u];
  };
  auto load_w = [&](gbf16x8 (&w)[2][2], int kt) {
    kt = kt < nk ? kt : nk - 1;
    const int64_t o = static_cast<int64_t>(kt) * kGemmBK;
    w[0][0] = *reinterpret_cast<const gbf16x8*>(wp0 + o);
    w[0][1] = *reinterpret_cast<const gbf16x8*>(wp0 + o + 32);
    w[1][0] = *reinterpret_cast<const gbf16x8*>(wp1 + o);
    w[1][1] = *reinterpret_cast<const gbf16x8*>(wp1 + o + 32);
  };
  const int xr = wm * 16 * MW + (lane & 15);   // this lane's B-fragment row in tile 0
  auto compute = [&](int buf, const gbf16x8 (&w)[2][2]) {
    const unsigned char* base = lds + buf * S::kStageBytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < MW; ++i) {
        const gbf16x8 xf =
            *reinterpret_cast<const gbf16x8*>(base + x_swz(xr + 16 * i, s * 4 + (lane >> 4)));
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0][s], xf, acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1][s], xf, acc[i][1], 0, 0, 0);
      }
    }
  };

  // Step t computes stage t (LDS buffer t % 3, W register set t % 3), stores X(t + 1)
  // (register set (t + 1) % 3, loaded two steps earlier) into buffer (t + 1) % 3 — last
  // read in step t - 2 — then issues X(t + 3) into set t % 3 (stored by step t - 1) and
  // W(t + 3) into set t % 3; one barrier per step.  W loads (HBM) have three steps to land,
  // X loads (L2) two.
  gbf16x8 w0[2][2], w1[2][2], w2[2][2];
  gu32x4 xs0[S::kCPT], xs1[S::kCPT], xs2[S::kCPT];
  load_x(xs0, 0);
  load_w(w0, 0);
  load_w(w1, 1);
  load_w(w2, 2);
  load_x(xs1, 1);
  load_x(xs2, 2);
  store_x(xs0, 0);
  __syncthreads();
#define CS_WS_STEP(T, B, WB, XST, XLD) \
  compute(B, WB);                      \
  store_x(XST, ((B) + 1) % 3);         \
  load_x(XLD, (T) + 3);                \
  load_w(WB, (T) + 3);                 \
  __syncthreads();
  int t = 0;
  for (; t + 3 <= nk; t += 3) {
    CS_WS_STEP(t, 0, w0, xs1, xs0)
    CS_WS_STEP(t + 1, 1, w1, xs2, xs1)
    CS_WS_STEP(t + 2, 2, w2, xs0, xs2)
  }
#undef CS_WS_STEP
  if (t < nk) {                      // tail: 1 or 2 steps, nothing left to prefetch
    compute(0, w0);
    if (t + 1 < nk) {
      store_x(xs1, 1);
      __syncthreads();
      compute(1, w1);
    }
  }

  // epilogue: D[n][m] -> lane holds rows n = 4 * (lane >> 4) + e (e = 0..3) of column m
#pragma unroll
  for (int i = 0; i < MW; ++i) {
    const int64_t m = m0 + wm * 16 * MW + 16 * i + (lane & 15);
    if (m >= M) continue;
    if (GATED) {
      const int64_t f = static_cast<int64_t>(nt) * 64 + wn * 16 + 4 * (lane >> 4);
      gu16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = gbf(gto_bf(acc[i][0][e]));
        const float u = gbf(gto_bf(acc[i][1][e]));
        const uint16_t a = gto_bf(act ? g_gelu_tanh(g) : g_silu(g));
        o[e] = gto_bf(gbf(a) * u);
      }
      *reinterpret_cast<gu16x4*>(Y + m * ldy + f) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t n = static_cast<int64_t>(nt) * kGemmBN + wn * 32 + 16 * j + 4 * (lane >> 4);
        if (P) {
          *reinterpret_cast<gf32x4*>(P + (static_cast<int64_t>(sp) * M + m) * n_out + n) = acc[i][j];
        } else {
          gu16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = gto_bf(acc[i][j][e]);
          *reinterpret_cast<gu16x4*>(Y + m * ldy + n) = o;
        }
      }
    }
  }
}

typedef __attribute__((address_space(3))) void* gl_lds_ptr;

// f(std::integral_constant<int, 0>) ... f(std::integral_constant<int, N - 1>), in order: an
// unrolled loop whose index is a constant expression (asm immediates, waitcnt counts)
template <typename F, int... Is>
__device__ __forceinline__ void cs_static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void cs_static_for(F&& f) {
  cs_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// one LDS DMA piece: 16 bytes per lane from src into the wave's 1 KB at lds_base
__device__ __forceinline__ void dma16(const uint16_t* src, unsigned char* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (gl_lds_ptr)lds_base, 16, 0, 0);
}

// a 16-byte global load the compiler does not track (its vmcnt is counted by hand).  NT: the
// non-temporal policy (`nt`), for PACKED weights one CU streams once -- the row blocks of
// <= 80 rows (per-rank and C1 shapes), where the weight stream is latency-bound and nt
// shortens a load's issue-to-landed time (MI355X_MICROARCH.md "nt-weights"): per-rank C5
// graph step 29.44 -> 27.14 ms, C3 5.94 -> 5.75 ms.  Kept off (measured slower,
// profiles/r06f_*.jsonl, r06i_*.json): the one-GPU C3 / C5 shapes (two row blocks sharing a
// column tile's weights through L2, compute-leaning: 3 % / 1.5 %), and row-major weights
// (each 16-byte load takes a quarter of a 64-byte line whose rest the next K steps read:
// the per-rank C3 down projection 27.6 -> 32.6 us unpacked, 23.2 -> 21.6 us packed)
template <bool NT = false>
__device__ __forceinline__ gbf16x8 asm_load16(const uint16_t* p) {
  gbf16x8 v;
  if constexpr (NT)
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// ws2_gemm_kernel<MT, NT>: the per-CU traffic of ws_gemm_kernel halved.  The 8 waves split
// only the columns (NT 16-column tiles each, 128 * NT per workgroup) and every wave covers
// all MT row tiles, so each W fragment is loaded by exactly one wave; X is staged by LDS
// DMA (global_load_lds_dwordx4: no staging registers, no ds_write; the chunk swizzle is
// applied to the per-lane SOURCE address, the LDS image is lane-linear) in three stages;
// W goes to registers through inline-asm loads, so the compiler's waits never drain the
// DMA queue: one counted s_waitcnt vmcnt per step (this step's X and W landed, the next
// two steps' loads still in flight) + a raw s_barrier.
template <int MT, int NT, int WAVES>
struct Ws2Shape {
  static constexpr int kRows = 16 * MT;
  static constexpr int kStage = kRows * 128;
  static constexpr int kPieces = kRows / 8;            // 1 KB DMA pieces (8 rows) per stage
  static constexpr int kG = (kPieces + WAVES - 1) / WAVES;   // DMA instructions per wave per stage
  static constexpr int kBN = 16 * NT * WAVES;
  static constexpr int kHalf = NT / 2;                 // gated: tiles [0, kHalf) gate, [kHalf, NT) up
  // loads issued after the older of X(t), W(t) when step t starts: W(t + 1), X(t + 1),
  // W(t + 2) after X(t)
  static constexpr int kWait = kG + 4 * NT;
  static constexpr int kLds = 3 * kStage;
};

// the tile (column tile nt, rows m0 ..) accumulated over nk K steps from kbase into acc:
// the whole software pipeline of a ws2 workgroup (every wave calls it; LDS free on entry)
// PACKED: W in the fragment-major layout of cs_gemm_pack (ldw = K): the 16-row tile T's
// 64-deep K step s is 2 KB at ((T * K / 64 + s) * 2 + sub) * 512 elements, lane-linear (lane
// l's 16 B = row l % 16, k 8 * (l / 16) of half `sub`), so each fragment load is ONE
// contiguous 1 KB and a wave's whole W stream for a tile is one sequential run.
template <int MT, int NT, int GATED, int WAVES, bool PACKED = false>
__device__ __forceinline__ void ws2_accumulate(
    unsigned char* lds, const uint16_t* __restrict__ X, int64_t ldx,
    const uint16_t* __restrict__ W, int64_t ldw, int64_t M, int64_t gate_off, int64_t nt,
    int64_t m0, int64_t kbase, int nk, gf32x4 (&acc)[MT][NT]) {
  using S = Ws2Shape<MT, NT, WAVES>;
  constexpr int kRows = S::kRows;
  constexpr int kStage = S::kStage;
  constexpr int kPieces = S::kPieces;
  constexpr int kG = S::kG;
  constexpr int kBN = S::kBN;
  constexpr int kHalf = S::kHalf;
  constexpr int kWait = S::kWait;
  (void)kRows;
  static_assert(!GATED || NT % 2 == 0, "the gated form pairs gate and up column tiles");
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    int64_t row;
    if (GATED) {
      const int jj = j % kHalf;
      const int64_t f = nt * (kBN / 2) + wv * 16 * kHalf + 16 * jj + (lane & 15);
      row = j < kHalf ? f : gate_off + f;
    } else {
      row = nt * kBN + wv * 16 * NT + 16 * j + (lane & 15);
    }
    if constexpr (PACKED) {
      const int64_t tile = (row - (lane & 15)) >> 4;
      wp[j] = W + ((tile * (ldw / kGemmBK) + kbase / kGemmBK) * 2) * 512 + 8 * lane;
    } else {
      wp[j] = W + row * ldw + kbase + 8 * (lane >> 4);
    }
  }
  const uint16_t* xsrc[kG];
  int xdst[kG];
#pragma unroll
  for (int g = 0; g < kG; ++g) {
    int pc = wv + WAVES * g;
    if (pc > kPieces - 1) pc = kPieces - 1;     // surplus pieces rewrite the last one
    const int r = 8 * pc + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);  // x_swz's involution, applied at the source
    int64_t gr = m0 + r;
    if (gr > M - 1) gr = M - 1;
    xsrc[g] = X + gr * ldx + kbase + 8 * c;
    xdst[g] = pc * 1024;
  }

#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = gf32x4{0.f, 0.f, 0.f, 0.f};

  auto issue_x = [&](int kt, int buf) {
    kt = kt < nk ? kt : nk - 1;
#pragma unroll
    for (int g = 0; g < kG; ++g)
      dma16(xsrc[g] + kt * kGemmBK, lds + buf * kStage + xdst[g]);
  };
  auto load_w = [&](gbf16x8 (&w)[NT][2], int kt) {
    kt = kt < nk ? kt : nk - 1;
    const int64_t o = static_cast<int64_t>(kt) * (PACKED ? 1024 : kGemmBK);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      w[j][0] = asm_load16<(PACKED && MT <= 5)>(wp[j] + o);
      w[j][1] = asm_load16<(PACKED && MT <= 5)>(wp[j] + o + (PACKED ? 512 : 32));
    }
  };
  const int xr = lane & 15;
  constexpr int kQ = 2 * MT;
  auto frag = [&](const unsigned char* base, int q) {
    const int s = q / MT, i = q % MT;
    return *reinterpret_cast<const gbf16x8*>(base + x_swz(xr + 16 * i, s * 4 + (lane >> 4)));
  };
#ifndef CS_WS2_THIN_RING
// W steps in flight for row blocks of <= 80 rows: 6 measured 0-30 % SLOWER than 3 on every
// per-rank / C1 shape (the longer prologue and tail outweigh the deeper stream;
// profiles/r05s_gemm_{old,new}.jsonl), so 3
#define CS_WS2_THIN_RING 3
#endif
#ifndef CS_GEMM_BIG_RING
#define CS_GEMM_BIG_RING 0
#endif
#ifndef CS_GEMM_ASM_LDS
#define CS_GEMM_ASM_LDS 6   // fragment reads in flight on the hand-counted path (0: off)
#endif
  // this lane's B-fragment byte offset (row xr of tile 0, chunk s * 4 + lane / 16) inside a
  // stage: row tile i adds 16 * 128 B (the swizzle term (r >> 1) & 7 is the same for r and
  // r + 16 i), so one address per sub-step serves every row tile as an immediate offset
  const uint32_t lds_u32 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((gl_lds_ptr)lds));
  const uint32_t fa0 = lds_u32 + x_swz(xr, lane >> 4);
  const uint32_t fa1 = lds_u32 + x_swz(xr, 4 + (lane >> 4));
  auto compute = [&](int buf, const gbf16x8 (&w)[NT][2]) {
    const unsigned char* base = lds + buf * kStage;
    if constexpr (CS_GEMM_ASM_LDS > 0 && MT > 9) {
      // hand-counted LDS pipeline for the large row counts (2 waves per SIMD): the fragment
      // reads are inline asm (invisible to the compiler's waitcnt pass, which otherwise
      // drains every read with lgkmcnt(0) before its first use), kR reads in flight; before
      // fragment q's MFMAs one counted lgkmcnt(n) names q's register as read-write, so its
      // MFMAs consume the landed value.  Measured 5-11 % faster at M = 272 / 520 and neutral
      // to 10 % slower at M <= 144 (profiles/r03g_gemm_asm_lds_ab.json), hence MT > 9 only.
      constexpr int kR = CS_GEMM_ASM_LDS > 0 ? CS_GEMM_ASM_LDS : 1;
      const uint32_t a0 = fa0 + buf * kStage, a1 = fa1 + buf * kStage;
      gbf16x8 f[kR];
      auto rd = [a0, a1](gbf16x8 (&fr)[kR], auto qc) {
        constexpr int q = decltype(qc)::value;
        if constexpr (q < kQ) {
          constexpr int off = (q % MT) * 2048;
          gbf16x8 v;
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(q < MT ? a0 : a1), "n"(off));
          fr[q % kR] = v;
        }
      };
      cs_static_for<kR - 1>([&](auto qc) { rd(f, qc); });
      cs_static_for<kQ>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        rd(f, std::integral_constant<int, q + kR - 1>{});
        constexpr int issued_after = (q + kR - 1 < kQ ? q + kR - 1 : kQ - 1) - q;
        gbf16x8 v = f[q % kR];
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(issued_after));
        constexpr int sub = q / MT, i = q % MT;
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][sub], v, acc[i][j], 0, 0, 0);
      });
    } else if constexpr (MT > 9 && CS_GEMM_BIG_RING == 0) {   // 2 waves per SIMD, no registers left for a ring
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        const gbf16x8 xf = frag(base, q);
        const int s = q / MT, i = q % MT;
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][s], xf, acc[i][j], 0, 0, 0);
      }
    } else {
      // B-fragments through a ring of kRing registers, kRing - 1 reads ahead of their
      // MFMAs; the schedule is pinned (ring fill, then one ds_read per NT MFMAs) so the LDS
      // round trip hides behind the MFMAs of earlier fragments
      constexpr int kRing = MT > 9 ? (CS_GEMM_BIG_RING > 1 ? CS_GEMM_BIG_RING : 3) : 4;
      gbf16x8 f[kRing];
#pragma unroll
      for (int q = 0; q < kRing - 1; ++q) f[q] = frag(base, q);
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        if (q + kRing - 1 < kQ) f[(q + kRing - 1) % kRing] = frag(base, q + kRing - 1);
        const int s = q / MT, i = q % MT;
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][s], f[q % kRing], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, kRing - 1, 0);
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        if (q + kRing - 1 < kQ) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);
      }
    }
  };
  // the step's wait names the W set it releases as read-write operands: the MFMAs consume
  // the wait's outputs, so the compiler cannot copy or move an asm-loaded register before
  // its data has landed (cdna_hip_programming.md §5.7 item 1, form (ii))
  auto sync = [&](gbf16x8 (&w)[NT][2]) {
    if constexpr (NT == 1) {
      asm volatile("s_waitcnt vmcnt(%2)" : "+v"(w[0][0]), "+v"(w[0][1]) : "n"(kWait) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%4)"
                   : "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[1][0]), "+v"(w[1][1])
                   : "n"(kWait) : "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // the loads of the last steps are never consumed: their registers stay allocated (named
  // as read-write operands) until the final vmcnt(0), or the compiler hands them to the
  // epilogue while the data is still in flight (a landing load overwrote an address)
  auto hold = [&](gbf16x8 (&w)[NT][2]) {
#pragma unroll
    for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(w[j][0]), "+v"(w[j][1]));
  };

  // Step t: X(t) in LDS buffer t % 3, W(t) in register set t % R.  It waits for X(t) (and
  // the older W(t)) with the loads of steps t - 2 and t - 1 after it still in flight, passes
  // the barrier (every wave done with step t - 1, so buffer (t + 2) % 3 — read in step
  // t - 1 — is free), issues X(t + 2) into it, computes, then loads W(t + R) into the set
  // it used: W (HBM) R steps ahead, X (L2) two.  R = 3 (CS_WS2_THIN_RING for the thin row
  // blocks; the younger loads at step t's wait are the same W(t + R - 2), X(t + 1),
  // W(t + R - 1) for every R, so kWait holds; R % 3 == 0 keeps every step's LDS buffer a
  // constant)
  constexpr int R = MT <= 5 ? CS_WS2_THIN_RING : 3;
  static_assert(R % 3 == 0 && R >= 3, "the W ring: a multiple of the 3 X buffers");
  gbf16x8 wr[R][NT][2];
  cs_static_for<R - 2>([&](auto rc) { load_w(wr[decltype(rc)::value], decltype(rc)::value); });
  issue_x(0, 0);
  load_w(wr[R - 2], R - 2);
  issue_x(1, 1);
  load_w(wr[R - 1], R - 1);
  for (int t = 0; t < nk; t += R) {
    cs_static_for<R>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      sync(wr[r]);
      issue_x(t + r + 2, (r + 2) % 3);
      if (t + r < nk) compute(r % 3, wr[r]);
      load_w(wr[r], t + r + R);
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may outlive the workgroup
  cs_static_for<R>([&](auto rc) { hold(wr[decltype(rc)::value]); });
}

// the accumulated tile to Y (bf16, or act(gate) * up) or, P != nullptr, to the fp32 partial
// of K split sp ([sp][M][n_out])
template <int MT, int NT, int GATED, int WAVES>
__device__ __forceinline__ void ws2_store(const gf32x4 (&acc)[MT][NT], uint16_t* __restrict__ Y,
                                          int64_t ldy, float* __restrict__ P, int64_t M,
                                          int64_t n_out, int64_t nt, int64_t m0, int sp, int act) {
  using S = Ws2Shape<MT, NT, WAVES>;
  constexpr int kBN = S::kBN;
  constexpr int kHalf = S::kHalf;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int64_t m = m0 + 16 * i + (lane & 15);
    if (m >= M) continue;
    if (GATED) {
#pragma unroll
      for (int jj = 0; jj < kHalf; ++jj) {
        const int64_t f = nt * (kBN / 2) + wv * 16 * kHalf + 16 * jj + 4 * (lane >> 4);
        gu16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float g = gbf(gto_bf(acc[i][jj][e]));
          const float u = gbf(gto_bf(acc[i][kHalf + jj][e]));
          const uint16_t a = gto_bf(act ? g_gelu_tanh(g) : g_silu(g));
          o[e] = gto_bf(gbf(a) * u);
        }
        *reinterpret_cast<gu16x4*>(Y + m * ldy + f) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int64_t n = nt * kBN + wv * 16 * NT + 16 * j + 4 * (lane >> 4);
        if (P) {
          *reinterpret_cast<gf32x4*>(P + (static_cast<int64_t>(sp) * M + m) * n_out + n) = acc[i][j];
        } else {
          gu16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = gto_bf(acc[i][j][e]);
          *reinterpret_cast<gu16x4*>(Y + m * ldy + n) = o;
        }
      }
    }
  }
}

// ws2_gemm_kernel<MT, NT>: the per-CU traffic of ws_gemm_kernel halved.  The 8 waves split
// only the columns (NT 16-column tiles each, 128 * NT per workgroup) and every wave covers
// all MT row tiles, so each W fragment is loaded by exactly one wave; X is staged by LDS
// DMA (global_load_lds_dwordx4: no staging registers, no ds_write; the chunk swizzle is
// applied to the per-lane SOURCE address, the LDS image is lane-linear) in three stages;
// W goes to registers through inline-asm loads, so the compiler's waits never drain the
// DMA queue: one counted s_waitcnt vmcnt per step (this step's X and W landed, the next
// two steps' loads still in flight) + a raw s_barrier.
#ifndef CS_WS2_GATED4
#define CS_WS2_GATED4 1   // variant 3 gated: 4 waves x 32 W rows (64 features) per workgroup
#endif
template <int MT, int NT, int GATED, int WAVES, bool PACKED = false>
__global__ __launch_bounds__(64 * WAVES, WAVES == 4 ? 2 : 1) void ws2_gemm_kernel(
    const uint16_t* __restrict__ X, int64_t ldx, const uint16_t* __restrict__ W, int64_t ldw,
    uint16_t* __restrict__ Y, int64_t ldy, float* __restrict__ P, int64_t M, int64_t n_out,
    int64_t gate_off, int nk, int n_tiles, int splits, int act, int m_blocks) {
  using S = Ws2Shape<MT, NT, WAVES>;
  __shared__ __align__(16) unsigned char lds[S::kLds];
  // row blocks of one (column tile, split) cell are 8 block ids apart — dispatched to the
  // same XCD (ids are dealt round-robin over the 8 XCDs) at about the same time, so the
  // second block's W reads hit that XCD's L2; the grid is padded to whole groups of 8 cells
  const int bid = blockIdx.x;
  int cell = bid, mb = 0;
  if (m_blocks > 1) {
    const int g = bid / (8 * m_blocks), r = bid % (8 * m_blocks);
    mb = r / 8;
    cell = g * 8 + (r % 8);
  }
  if (cell >= n_tiles * splits) return;
  const int nt = cell % n_tiles;
  const int sp = cell / n_tiles;
  const int64_t m0 = static_cast<int64_t>(mb) * S::kRows;
  const int64_t kbase = static_cast<int64_t>(sp) * nk * kGemmBK;
  gf32x4 acc[MT][NT];
  ws2_accumulate<MT, NT, GATED, WAVES, PACKED>(lds, X, ldx, W, ldw, M, gate_off, nt, m0, kbase, nk,
                                               acc);
  ws2_store<MT, NT, GATED, WAVES>(acc, Y, ldy, P, M, n_out, nt, m0, sp, act);
}

// Y[m][n] = bf16(sum_s P[s][m][n]) in split order; 8 outputs per thread
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ P, int splits,
                                                            int64_t M, int64_t N,
                                                            uint16_t* __restrict__ Y, int64_t ldy) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int64_t nv = N / 8;
  if (v >= M * nv) return;
  const int64_t m = v / nv;
  const int64_t n = (v - m * nv) * 8;
  gf32x4 a = *reinterpret_cast<const gf32x4*>(P + m * N + n);
  gf32x4 b = *reinterpret_cast<const gf32x4*>(P + m * N + n + 4);
  for (int s = 1; s < splits; ++s) {
    const float* q = P + (static_cast<int64_t>(s) * M + m) * N + n;
    a += *reinterpret_cast<const gf32x4*>(q);
    b += *reinterpret_cast<const gf32x4*>(q + 4);
  }
  gu16x8 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    o[e] = gto_bf(a[e]);
    o[4 + e] = gto_bf(b[e]);
  }
  *reinterpret_cast<gu16x8*>(Y + m * ldy + n) = o;
}

// thin_gemm_kernel<MT, FT, GATED, WAVES, RING>: the per-rank step shapes (M <= 80 rows: C1
// 20, C3 48 at 8 ranks, C5 72), where the weight stream is latency-bound -- the split-K
// kernels above reach 2-5 TB/s there and ~25 % more when the weights sit in the Infinity
// Cache (profiles/r04f_gemm_r8_*.jsonl).  No barrier and no LDS in the main loop: a
// workgroup owns 16 * FT output features (GATED: 16 gate features and their 16 up
// features), its WAVES waves split the K steps (64 deep) evenly, and each wave streams its
// slice of W and of X (L2-resident) straight into MFMA fragments through a RING-deep
// register ring (plain loads; the compiler's counted vmcnt keeps the later slots in flight).
// A lane reads 32 contiguous bytes of its W row per step (4 lanes = one 128-B line) and the
// same k range of its X row; the two 16-B halves feed the step's two 32-deep MFMAs, so k is
// permuted identically in both operands.  At the end the waves' fp32 accumulators meet in
// LDS and are folded in wave order (deterministic), then rounded to bf16 (GATED: act(gate)
// * up with cs_gated_act's roundings).  K % 64 == 0, M <= 16 * MT.
template <int MT, int FT, int GATED, int WAVES, int RING>
__global__ __launch_bounds__(64 * WAVES, 1) void thin_gemm_kernel(
    const uint16_t* __restrict__ X, int64_t ldx, const uint16_t* __restrict__ W, int64_t ldw,
    uint16_t* __restrict__ Y, int64_t ldy, int64_t M, int64_t gate_off, int nsteps, int act) {
  static_assert(!GATED || FT == 2, "the gated form pairs one gate tile with one up tile");
  __shared__ gf32x4 red[WAVES][FT * MT][64];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t f0 = static_cast<int64_t>(blockIdx.x) * (GATED ? 16 : 16 * FT);
  const int s0 = wv * nsteps / WAVES;
  const int s1 = (wv + 1) * nsteps / WAVES;
  const int koff = 16 * (lane >> 4);
  const uint16_t* wp[FT];
#pragma unroll
  for (int j = 0; j < FT; ++j) {
    const int64_t row = GATED ? (j ? gate_off : 0) + f0 + (lane & 15) : f0 + 16 * j + (lane & 15);
    wp[j] = W + row * ldw + koff;
  }
  const uint16_t* xp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int64_t row = 16 * i + (lane & 15);
    if (row > M - 1) row = M - 1;     // padded rows read a real row; their results are dropped
    xp[i] = X + row * ldx + koff;
  }
  gf32x4 acc[FT][MT];
#pragma unroll
  for (int j = 0; j < FT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[j][i] = gf32x4{0.f, 0.f, 0.f, 0.f};

  gbf16x8 wr[RING][FT][2];
  gbf16x8 xr[RING][MT][2];
  const int last = s1 > s0 ? s1 - 1 : s0;
  auto load = [&](int r, int s) {
    s = s < last ? s : last;           // past the slice: re-read its last step (a cache hit)
    const int64_t o = static_cast<int64_t>(s) * 64;
#pragma unroll
    for (int j = 0; j < FT; ++j) {
      wr[r][j][0] = *reinterpret_cast<const gbf16x8*>(wp[j] + o);
      wr[r][j][1] = *reinterpret_cast<const gbf16x8*>(wp[j] + o + 8);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      xr[r][i][0] = *reinterpret_cast<const gbf16x8*>(xp[i] + o);
      xr[r][i][1] = *reinterpret_cast<const gbf16x8*>(xp[i] + o + 8);
    }
  };
  auto compute = [&](int r) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < FT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[r][j][q], xr[r][i][q], acc[j][i], 0, 0, 0);
  };
  cs_static_for<RING>([&](auto r) { load(r, s0 + r); });
  int s = s0;
  for (; s + RING <= s1; s += RING) {
    cs_static_for<RING>([&](auto r) {
      compute(r);
      load(r, s + RING + r);
    });
  }
  cs_static_for<RING>([&](auto r) {
    if (s + r < s1) compute(r);
  });

  // fold the waves' partial sums in wave order; fold unit u (a row tile i and, unless
  // gated, a feature tile j) is finished by wave u % WAVES
#pragma unroll
  for (int j = 0; j < FT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) red[wv][j * MT + i][lane] = acc[j][i];
  __syncthreads();
  constexpr int kUnits = GATED ? MT : FT * MT;
  for (int u = wv; u < kUnits; u += WAVES) {
    if (GATED) {
      const int i = u;
      const int64_t m = 16 * i + (lane & 15);
      gf32x4 g = red[0][i][lane], up = red[0][MT + i][lane];
      for (int w = 1; w < WAVES; ++w) {
        g += red[w][i][lane];
        up += red[w][MT + i][lane];
      }
      if (m < M) {
        gu16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = gbf(gto_bf(g[e]));
          const float uv = gbf(gto_bf(up[e]));
          const uint16_t a = gto_bf(act ? g_gelu_tanh(gv) : g_silu(gv));
          o[e] = gto_bf(gbf(a) * uv);
        }
        *reinterpret_cast<gu16x4*>(Y + m * ldy + f0 + 4 * (lane >> 4)) = o;
      }
    } else {
      const int j = u / MT, i = u - j * MT;
      const int64_t m = 16 * i + (lane & 15);
      gf32x4 a = red[0][u][lane];
      for (int w = 1; w < WAVES; ++w) a += red[w][u][lane];
      if (m < M) {
        gu16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = gto_bf(a[e]);
        *reinterpret_cast<gu16x4*>(Y + m * ldy + f0 + 16 * j + 4 * (lane >> 4)) = o;
      }
    }
  }
}

// thin variants: 5 = 16 features x 8 waves, 6 = 32 features x 8 waves, 7 = 16 features x
// 16 waves (gated: one gate + one up tile, 8 / 8 / 16 waves)
constexpr int kThinMaxRows = 80;
bool thin_variant(int variant) { return variant >= 5 && variant <= 7; }
int thin_ft(int variant, int gated) { return gated || variant == 6 ? 2 : 1; }
int thin_waves(int variant) { return variant == 7 ? 16 : 8; }

template <int MT, int FT, int GATED, int WAVES, int RING>
void launch_thin(int blocks, hipStream_t st, const uint16_t* X, int64_t ldx, const uint16_t* W,
                 int64_t ldw, uint16_t* Y, int64_t ldy, int64_t M, int64_t gate_off, int nsteps,
                 int act) {
  hipLaunchKernelGGL((thin_gemm_kernel<MT, FT, GATED, WAVES, RING>), dim3(blocks), dim3(64 * WAVES),
                     0, st, X, ldx, W, ldw, Y, ldy, M, gate_off, nsteps, act);
}

// row tiles 1..MAXMT (the caller keeps mt <= MAXMT)
template <int FT, int GATED, int WAVES, int RING, int MAXMT>
void dispatch_thin(int mt, int blocks, hipStream_t st, const uint16_t* X, int64_t ldx,
                   const uint16_t* W, int64_t ldw, uint16_t* Y, int64_t ldy, int64_t M,
                   int64_t gate_off, int nsteps, int act) {
  if constexpr (MAXMT > 1) {
    if (mt < MAXMT) {
      dispatch_thin<FT, GATED, WAVES, RING, MAXMT - 1>(mt, blocks, st, X, ldx, W, ldw, Y, ldy, M,
                                                       gate_off, nsteps, act);
      return;
    }
  }
  launch_thin<MAXMT, FT, GATED, WAVES, RING>(blocks, st, X, ldx, W, ldw, Y, ldy, M, gate_off,
                                             nsteps, act);
}

template <int MW, int GATED>
void launch_ws(int blocks, hipStream_t st, const uint16_t* X, int64_t ldx, const uint16_t* W,
               int64_t ldw, uint16_t* Y, int64_t ldy, float* P, int64_t M, int64_t n_out,
               int64_t gate_off, int nk, int n_tiles, int splits, int act) {
  hipLaunchKernelGGL((ws_gemm_kernel<MW, GATED>), dim3(blocks), dim3(kGemmThreads), 0, st, X, ldx, W,
                     ldw, Y, ldy, P, M, n_out, gate_off, nk, n_tiles, splits, act);
}

template <int GATED>
void dispatch_ws(int mw, int blocks, hipStream_t st, const uint16_t* X, int64_t ldx,
                 const uint16_t* W, int64_t ldw, uint16_t* Y, int64_t ldy, float* P, int64_t M,
                 int64_t n_out, int64_t gate_off, int nk, int n_tiles, int splits, int act) {
#define CS_WS_CASE(V) \
  case V: launch_ws<V, GATED>(blocks, st, X, ldx, W, ldw, Y, ldy, P, M, n_out, gate_off, nk, n_tiles, splits, act); break;
  switch (mw) {
    CS_WS_CASE(1) CS_WS_CASE(2) CS_WS_CASE(3) CS_WS_CASE(4) CS_WS_CASE(5)
    CS_WS_CASE(6) CS_WS_CASE(7) CS_WS_CASE(8) CS_WS_CASE(9)
    default: break;
  }
#undef CS_WS_CASE
}

// 16-row tiles per wave for M rows: all rows in one block up to 288
int ws_mw(int64_t M) {
  const int64_t tiles = (M + 15) / 16;
  const int64_t mw = (tiles + 1) / 2;
  return static_cast<int>(mw < kGemmMaxMW ? mw : kGemmMaxMW);
}

// ws2: row tiles per workgroup (instantiated counts) and row blocks for M rows. The 5-tile
// block is taken on packed weights only (per-rank C5, 72 rows: 1-2% over 8 tiles there,
// profiles/r04af_ws2_mt5_ab.jsonl); on row-major weights it measured slower (gate|up 194 -> 224 us).
constexpr int kWs2MT[] = {2, 4, 5, 8, 9, 12, 17, 18};
void ws2_rows(int64_t M, int* mt, int64_t* mblocks, int max_tiles = 18, bool packed = false) {
  const int64_t tiles = (M + 15) / 16;
  const int64_t mb = (tiles + max_tiles - 1) / max_tiles;
  const int64_t per = (tiles + mb - 1) / mb;
  int v = 18;
  for (int c : kWs2MT) {
    if (c == 5 && !packed) continue;
    if (c >= per) { v = c; break; }
  }
  *mt = v;
  *mblocks = (tiles + v - 1) / v;
}

template <int MT, int NT, int GATED, int WAVES, bool PACKED>
void launch_ws2(int blocks, hipStream_t st, const uint16_t* X, int64_t ldx, const uint16_t* W,
                int64_t ldw, uint16_t* Y, int64_t ldy, float* P, int64_t M, int64_t n_out,
                int64_t gate_off, int nk, int n_tiles, int splits, int act, int m_blocks) {
  hipLaunchKernelGGL((ws2_gemm_kernel<MT, NT, GATED, WAVES, PACKED>), dim3(blocks), dim3(64 * WAVES),
                     0, st, X, ldx, W, ldw, Y, ldy, P, M, n_out, gate_off, nk, n_tiles, splits, act,
                     m_blocks);
}

template <int NT, int GATED, int WAVES, bool PACKED>
void dispatch_ws2(int mt, int blocks, hipStream_t st, const uint16_t* X, int64_t ldx,
                  const uint16_t* W, int64_t ldw, uint16_t* Y, int64_t ldy, float* P, int64_t M,
                  int64_t n_out, int64_t gate_off, int nk, int n_tiles, int splits, int act,
                  int m_blocks) {
#define CS_WS2_CASE(V)                                                                          \
  case V:                                                                                       \
    launch_ws2<V, NT, GATED, WAVES, PACKED>(blocks, st, X, ldx, W, ldw, Y, ldy, P, M, n_out,    \
                                            gate_off, nk, n_tiles, splits, act, m_blocks);      \
    break;
  switch (mt) {
    CS_WS2_CASE(2) CS_WS2_CASE(4) CS_WS2_CASE(5) CS_WS2_CASE(8) CS_WS2_CASE(9) CS_WS2_CASE(12)
    CS_WS2_CASE(17)
    CS_WS2_CASE(18)
    default: break;
  }
#undef CS_WS2_CASE
}

// W rows per workgroup of a variant (1: ws 128; 2: ws2 8 waves x 32; 3: ws2 8 x 16, gated
// 4 x 32; 4: as 2 with at most 9 row tiles (144 rows) per workgroup)
int64_t variant_bn(int variant, int gated) {
  if (variant == 1) return 128;
  if (variant == 3) return gated && !CS_WS2_GATED4 ? 256 : 128;
  return 256;
}

int variant_max_tiles(int variant) { return variant == 4 ? 9 : 18; }

int64_t gemm_tiles(int variant, int64_t M, int64_t N, int gated) {
  if (variant == 1) {
    const int mw = ws_mw(M);
    return (gated ? N / 128 : N / kGemmBN) * ((M + 32 * mw - 1) / (32 * mw));
  }
  int mt;
  int64_t mb;
  ws2_rows(M, &mt, &mb, variant_max_tiles(variant));
  return (N / variant_bn(variant, gated)) * mb;
}

// grid of a ws2 launch: (column tile, split) cells padded to groups of 8 when row blocks pair
int64_t ws2_grid(int64_t cells, int64_t mblocks) {
  return mblocks > 1 ? (cells + 7) / 8 * 8 * mblocks : cells;
}

// the packed gated form at <= 80 rows (the per-rank decode steps) with 7 waves x 32 W rows
// (112 features) per workgroup: the 70B gate|up (57,344 rows) is then 256 workgroups on
// the 256 CUs instead of 224 (8 waves x 32 rows)
#ifndef CS_WS2_GATED7
#define CS_WS2_GATED7 1
#endif
bool ws2_gated7(int variant, int64_t M, int64_t N, int gated, bool packed) {
  return CS_WS2_GATED7 && gated && packed && (variant == 2 || variant == 4) && M <= 80 &&
         N % 224 == 0;
}

int resolve_variant(int variant, int64_t N, int gated) {
  if (variant == 0) variant = 2;
  if (thin_variant(variant)) return variant;
  if ((variant == 2 || variant == 4) && N % 256) variant = gated ? 1 : 3;
  if (variant == 3 && gated && (!CS_WS2_GATED4 || N % 128)) variant = 2;
  return variant;
}

}  // namespace

extern "C" {

int64_t cs_gemm_splits(int64_t M, int64_t N, int64_t K, int gated, int variant) {
  if (M <= 0 || N <= 0 || K <= 0 || N % 128) return 0;
  if (gated || thin_variant(variant)) return 1;
  variant = resolve_variant(variant, N, gated);
  const int64_t tiles = gemm_tiles(variant, M, N, gated);
  // fill the 256 CUs (one 512-thread workgroup each) while keeping >= 8 K steps per split
  int64_t s = 1;
  while (tiles * s < 256 && K % (kGemmBK * s * 2) == 0 && K / (kGemmBK * s * 2) >= 8) s *= 2;
  return s;
}

}  // extern "C"

namespace {
// cs_gemm_bf16 (packed = false) and cs_gemm_bf16_packed (W in cs_gemm_pack's layout: the ws2
// variants 2-4 only, ldw = K)
int gemm_impl(const void* x, int64_t ldx, const void* w, int64_t ldw, void* y, int64_t ldy,
              int64_t M, int64_t N, int64_t K, int splits, int gated, int act, int variant,
              float* workspace, cs_stream_t stream, bool packed) {
  if (M < 0 || N <= 0 || K <= 0) return fail(CS_ERR_INVALID, "cs_gemm_bf16: bad shape");
  if (packed) {
    if (variant == 0) variant = 2;
    if (variant < 2 || variant > 4)
      return fail(CS_ERR_INVALID, "cs_gemm_bf16_packed: variants 2-4 (the ws2 kernels) only");
    if (K % kGemmBK) return fail(CS_ERR_INVALID, "cs_gemm_bf16_packed: K must be a multiple of 64");
    ldw = K;
  }
  if (M == 0) return CS_OK;
  if (!x || !w) return fail(CS_ERR_INVALID, "cs_gemm_bf16: NULL pointer");
  if (variant < 0 || variant > 7) return fail(CS_ERR_INVALID, "cs_gemm_bf16: variant must be 0..7");
  if (N % 128) return fail(CS_ERR_INVALID, "cs_gemm_bf16: N must be a multiple of 128");
  if (gated && splits > 1)
    return fail(CS_ERR_INVALID, "cs_gemm_bf16: the gated form takes no K split");
  variant = resolve_variant(variant, N, gated);
  if (packed && variant != 2 && variant != 3 && variant != 4)
    return fail(CS_ERR_INVALID, "cs_gemm_bf16_packed: N must be a multiple of 256 for this variant");
  if (splits <= 0) splits = static_cast<int>(cs_gemm_splits(M, N, K, gated, variant));
  if (!y && (splits <= 1 || gated))
    return fail(CS_ERR_INVALID, "cs_gemm_bf16: y may be NULL only with a K split (partials kept)");
  if (K % (kGemmBK * splits))
    return fail(CS_ERR_INVALID, "cs_gemm_bf16: K must be a multiple of 64 * splits");
  if (ldx % 8 || ldw % 8 || (y && (ldy % 4 || ldy < (gated ? N / 2 : N))) || ldx < K || ldw < K)
    return fail(CS_ERR_INVALID, "cs_gemm_bf16: leading dimensions too small or misaligned");
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w)) & 15 ||
      reinterpret_cast<uintptr_t>(y) & 7)
    return fail(CS_ERR_INVALID, "cs_gemm_bf16: operands must be 16-byte aligned (y 8-byte)");
  if (splits > 1 && !workspace)
    return fail(CS_ERR_INVALID, "cs_gemm_bf16: split K needs a workspace of splits * M * N floats");
  // the split-K fold writes 16-byte vectors of 8 features at y + m * ldy + n
  if (splits > 1 && y && (ldy % 8 || reinterpret_cast<uintptr_t>(y) & 15))
    return fail(CS_ERR_INVALID, "cs_gemm_bf16: a K split needs y 16-byte aligned and ldy % 8 == 0");
  if (thin_variant(variant)) {
    if (M > kThinMaxRows || K % kGemmBK || splits > 1 || !y)
      return fail(CS_ERR_INVALID, "cs_gemm_bf16: variants 5-7 take M <= 80, K % 64 == 0, no K split");
    const int ft = thin_ft(variant, gated);
    const int64_t n_out = gated ? N / 2 : N;
    const int64_t blocks = gated ? n_out / 16 : n_out / (16 * ft);
    const int mt = static_cast<int>((M + 15) / 16);
    const int nsteps = static_cast<int>(K / kGemmBK);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint16_t* X = static_cast<const uint16_t*>(x);
    const uint16_t* Wp = static_cast<const uint16_t*>(w);
    uint16_t* Y = static_cast<uint16_t*>(y);
    const int b = static_cast<int>(blocks);
    if (gated) {
      if (variant == 7 && mt <= 3)    // (16 gated waves spill at 4-5 row tiles: 8 waves there)
        dispatch_thin<2, 1, 16, 2, 3>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, M, n_out, nsteps, act);
      else
        dispatch_thin<2, 1, 8, 3, 5>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, M, n_out, nsteps, act);
    } else if (variant == 5) {
      dispatch_thin<1, 0, 8, 3, 5>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, M, 0, nsteps, 0);
    } else if (variant == 6) {
      dispatch_thin<2, 0, 8, 3, 5>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, M, 0, nsteps, 0);
    } else {
      dispatch_thin<1, 0, 16, 2, 5>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, M, 0, nsteps, 0);
    }
    return check_launch("cs_gemm_bf16");
  }
  const int64_t tiles = gemm_tiles(variant, M, N, gated);
  const int64_t blocks = tiles * splits;
  if (blocks > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_gemm_bf16: grid too large");
  const int nk = static_cast<int>(K / (kGemmBK * splits));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint16_t* X = static_cast<const uint16_t*>(x);
  const uint16_t* Wp = static_cast<const uint16_t*>(w);
  uint16_t* Y = static_cast<uint16_t*>(y);
  float* Pp = splits > 1 ? workspace : nullptr;
  if (variant == 1) {
    const int mw = ws_mw(M);
    const int n_tiles = static_cast<int>(gated ? N / 128 : N / kGemmBN);
    if (gated)
      dispatch_ws<1>(mw, static_cast<int>(blocks), st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2,
                     N / 2, nk, n_tiles, 1, act);
    else
      dispatch_ws<0>(mw, static_cast<int>(blocks), st, X, ldx, Wp, ldw, Y, ldy, Pp, M, N, 0, nk,
                     n_tiles, splits, 0);
  } else {
    int mt;
    int64_t mb;
    ws2_rows(M, &mt, &mb, variant_max_tiles(variant), packed);
    const int n_tiles = static_cast<int>(N / variant_bn(variant, gated));
    const int64_t grid = ws2_grid(static_cast<int64_t>(n_tiles) * splits, mb);
    if (grid > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_gemm_bf16: grid too large");
    const int b = static_cast<int>(grid);
    const int mbi = static_cast<int>(mb);
    if (ws2_gated7(variant, M, N, gated, packed)) {
      const int n7 = static_cast<int>(N / 224);     // (M <= 80: one row block, mt <= 5)
      if (mt == 2)
        launch_ws2<2, 2, 1, 7, true>(n7, st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2, N / 2, nk,
                                     n7, 1, act, 1);
      else if (mt == 4)
        launch_ws2<4, 2, 1, 7, true>(n7, st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2, N / 2, nk,
                                     n7, 1, act, 1);
      else
        launch_ws2<5, 2, 1, 7, true>(n7, st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2, N / 2, nk,
                                     n7, 1, act, 1);
    } else if (gated && variant == 3) {
      if (packed)
        dispatch_ws2<2, 1, 4, true>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2, N / 2, nk,
                                    n_tiles, 1, act, mbi);
      else
        dispatch_ws2<2, 1, 4, false>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2, N / 2, nk,
                                     n_tiles, 1, act, mbi);
    } else if (gated) {
      if (packed)
        dispatch_ws2<2, 1, 8, true>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2, N / 2, nk,
                                    n_tiles, 1, act, mbi);
      else
        dispatch_ws2<2, 1, 8, false>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, nullptr, M, N / 2, N / 2, nk,
                                     n_tiles, 1, act, mbi);
    } else if (variant == 3) {
      if (packed)
        dispatch_ws2<1, 0, 8, true>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, Pp, M, N, 0, nk, n_tiles, splits,
                                    0, mbi);
      else
        dispatch_ws2<1, 0, 8, false>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, Pp, M, N, 0, nk, n_tiles,
                                     splits, 0, mbi);
    } else {
      if (packed)
        dispatch_ws2<2, 0, 8, true>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, Pp, M, N, 0, nk, n_tiles, splits,
                                    0, mbi);
      else
        dispatch_ws2<2, 0, 8, false>(mt, b, st, X, ldx, Wp, ldw, Y, ldy, Pp, M, N, 0, nk, n_tiles,
                                     splits, 0, mbi);
    }
  }
  if (splits > 1 && !gated && Y) {     // y == NULL: the caller folds the partials itself
    const int64_t nv = M * (N / 8);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(static_cast<uint32_t>((nv + 255) / 256)), dim3(256),
                       0, st, workspace, splits, M, N, Y, ldy);
  }
  return check_launch("cs_gemm_bf16");
}

// Wp[((T * ns + s) * 2 + h) * 512 + 8 l + e] = W[16 T + l % 16][64 s + 32 h + 8 (l / 16) + e]
__global__ __launch_bounds__(256) void gemm_pack_kernel(const uint16_t* __restrict__ W, int64_t ldw,
                                                        int64_t n_vec, int64_t ns,
                                                        uint16_t* __restrict__ Wp) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;   // one 16-B vector
  if (v >= n_vec) return;
  const int l = static_cast<int>(v & 63);
  const int64_t blk = v >> 6;                    // (T * ns + s) * 2 + h
  const int h = static_cast<int>(blk & 1);
  const int64_t ts = blk >> 1;
  const int64_t T = ts / ns, st = ts - T * ns;
  const int64_t row = 16 * T + (l & 15);
  const int64_t col = 64 * st + 32 * h + 8 * (l >> 4);
  *reinterpret_cast<gu32x4*>(Wp + 8 * v) = *reinterpret_cast<const gu32x4*>(W + row * ldw + col);
}
}  // namespace

extern "C" {

int cs_gemm_bf16(const void* x, int64_t ldx, const void* w, int64_t ldw, void* y, int64_t ldy,
                 int64_t M, int64_t N, int64_t K, int splits, int gated, int act, int variant,
                 float* workspace, cs_stream_t stream) {
  return gemm_impl(x, ldx, w, ldw, y, ldy, M, N, K, splits, gated, act, variant, workspace, stream,
                   false);
}

int cs_gemm_bf16_packed(const void* x, int64_t ldx, const void* w_packed, void* y, int64_t ldy,
                        int64_t M, int64_t N, int64_t K, int splits, int gated, int act,
                        int variant, float* workspace, cs_stream_t stream) {
  return gemm_impl(x, ldx, w_packed, K, y, ldy, M, N, K, splits, gated, act, variant, workspace,
                   stream, true);
}

int cs_gemm_pack(const void* w, int64_t ldw, int64_t N, int64_t K, void* w_packed,
                 cs_stream_t stream) {
  if (!w || !w_packed) return fail(CS_ERR_INVALID, "cs_gemm_pack: NULL pointer");
  if (N <= 0 || K <= 0 || N % 16 || K % kGemmBK || ldw < K || ldw % 8)
    return fail(CS_ERR_INVALID, "cs_gemm_pack: need N % 16 == 0, K % 64 == 0, ldw >= K, ldw % 8 == 0");
  if ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(w_packed)) & 15)
    return fail(CS_ERR_INVALID, "cs_gemm_pack: operands must be 16-byte aligned");
  const int64_t n_vec = N * K / 8;
  hipLaunchKernelGGL(gemm_pack_kernel, dim3(static_cast<uint32_t>((n_vec + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t*>(w), ldw, n_vec,
                     K / kGemmBK, static_cast<uint16_t*>(w_packed));
  return check_launch("cs_gemm_pack");
}

}  // extern "C"
