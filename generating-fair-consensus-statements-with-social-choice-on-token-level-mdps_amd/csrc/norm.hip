// norm.hip — the per-token elementwise work of the stream forward, fused:
//
//   add_rms_kernel    residual add + RMSNorm in one pass over a row: s = a + b (rounded to
//                     bf16, the residual stream), y = s * rsqrt(mean(s^2) + eps) * w
//                     (Llama-3) or * (1 + w) (Gemma-2), fp32 statistics.  Replaces the
//                     add + 1 (Llama) / 7 (Gemma: cast, pow, mean, add, rsqrt, mul, mul,
//                     cast) launches of the PyTorch layer.
//   gated_act_kernel  act(gate) * up for the gated MLP (SiLU for Llama-3, tanh-GeLU for
//                     Gemma-2) in one pass; the activation is rounded to bf16 before the
//                     product, as the PyTorch pair of launches does.
//
// Both are HBM-streaming (16-byte vector loads, one workgroup per row / per row slice);
// on decode-sized batches what they save is launches (each costs ~4-5 us of GPU time
// even inside a captured graph).
#include "cs_kernels.cuh"

namespace {

typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }

// fp32 -> bf16, round to nearest even (NaN kept quiet)
__device__ __forceinline__ uint16_t to_bf(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);
  return static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

constexpr int kNormThreads = 256;
constexpr int kMaxSplits = 16;      // K-split partials folded by cs_add_rms_norm_splitk

// the row's sum over the workgroup: wave64 butterfly, then the BLOCK / 64 wave sums in wave
// order (the same order everywhere, so a norm is bitwise the same in every kernel that uses it)
template <int BLOCK = kNormThreads>
__device__ __forceinline__ float row_sum(float ss, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.0f;
#pragma unroll
  for (int i = 0; i < BLOCK / 64; ++i) tot += red[i];
  return tot;
}

// one workgroup per row; VPT 16-byte vectors per thread (d <= 256 * 8 * VPT).  s_out may
// alias a (the residual stream updated in place): every element is loaded before the
// barrier and stored after it by the same thread.  wb != nullptr: the branch b is first
// RMS-normalised itself with weight wb (Gemma-2's post-attention / post-MLP norm), with
// the arithmetic and rounding of a separate add_rms launch over b alone.
// FOLD: the K-split partials' count rounded up to a power of two (only those loads issued).
// BLOCK: threads per row -- one 16-byte vector per thread up to d = 8192 (a decode step's
// 48-72 rows are one workgroup each, so the row's loads are spread over as many lanes as
// its vectors: the launch is a few memory round trips, not VPT serial issue batches)
template <int VPT, bool FOLD, int NSP = kMaxSplits, int BLOCK = kNormThreads>
__global__ __launch_bounds__(BLOCK) void add_rms_kernel(
    const uint16_t* a, int64_t lda, const uint16_t* __restrict__ b, int64_t ldb,
    const uint16_t* __restrict__ wb, uint16_t* s_out, int64_t lds,
    const uint16_t* __restrict__ w, int64_t d, float eps, int plus_one,
    uint16_t* __restrict__ y, int64_t ldy, const float* __restrict__ bp, int splits) {
  const int64_t r = blockIdx.x;
  const int nv = static_cast<int>(d >> 3);
  __shared__ float red[2][BLOCK / 64];
  // every load of the row is issued before the first reduction: one memory round trip per
  // row instead of four (b, then wb after b's norm, then a, then w after the second norm);
  // the weights are prefetched only while the registers allow (VPT <= 4)
  constexpr bool kPre = VPT <= 4;
  u16x8 bv[VPT], av[VPT], wv[kPre ? VPT : 1], wbv[kPre ? VPT : 1];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = threadIdx.x + k * BLOCK;
    if (v < nv) {
      av[k] = *reinterpret_cast<const u16x8*>(a + r * lda + 8 * v);
      if constexpr (FOLD) {
        // b = bf16 of the split-K partials [splits][rows][d] folded in split order: the
        // arithmetic of cs_gemm_bf16's own fold (splitk_reduce_kernel), so the fused launch
        // is bitwise the GEMM's bf16 output followed by this norm
        // (all kMaxSplits loads issued unconditionally from clamped splits, so they are in
        // flight together; a select, not an added zero, skips the ones past `splits`)
        const float* q = bp + r * d + 8 * v;
        const int64_t sstride = static_cast<int64_t>(gridDim.x) * d;
        // at 1024 threads (d > 4096) 16 splits in flight would need 128 VGPRs and spill:
        // there the splits go in two batches of 8 (the same additions in the same order)
        constexpr int NB = (BLOCK >= 1024 && NSP > 8) ? 8 : NSP;
        f32x4 x0 = {0.0f, 0.0f, 0.0f, 0.0f}, x1 = x0;
#pragma unroll
        for (int s0 = 0; s0 < NSP; s0 += NB) {
          if (s0 > 0 && s0 >= splits) break;
          f32x4 p0[NB], p1[NB];
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            const int sp = s0 + j;
            const float* qs = q + (sp < splits ? sp : splits - 1) * sstride;
            p0[j] = *reinterpret_cast<const f32x4*>(qs);
            p1[j] = *reinterpret_cast<const f32x4*>(qs + 4);
          }
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            const int sp = s0 + j;
            if (sp == 0) {
              x0 = p0[0];
              x1 = p1[0];
            } else {
              x0 = sp < splits ? x0 + p0[j] : x0;
              x1 = sp < splits ? x1 + p1[j] : x1;
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bv[k][e] = to_bf(x0[e]);
          bv[k][4 + e] = to_bf(x1[e]);
        }
      } else if (b) {
        bv[k] = *reinterpret_cast<const u16x8*>(b + r * ldb + 8 * v);
      }
      if constexpr (kPre) {
        wv[k] = *reinterpret_cast<const u16x8*>(w + 8 * v);
        if (wb) wbv[k] = *reinterpret_cast<const u16x8*>(wb + 8 * v);
      }
    }
  }
  const bool has_b = FOLD || b;
  if (has_b && wb) {
    float sb = 0.0f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int v = threadIdx.x + k * BLOCK;
      if (v < nv) {
#pragma unroll
        for (int e = 0; e < 8; ++e) sb = fmaf(bf(bv[k][e]), bf(bv[k][e]), sb);
      }
    }
    const float inv_b = 1.0f / sqrtf(row_sum<BLOCK>(sb, red[0]) / static_cast<float>(d) + eps);
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int v = threadIdx.x + k * BLOCK;
      if (v < nv) {
        u16x8 g8;
        if constexpr (kPre) g8 = wbv[k];
        else g8 = *reinterpret_cast<const u16x8*>(wb + 8 * v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g = plus_one ? 1.0f + bf(g8[e]) : bf(g8[e]);
          bv[k][e] = to_bf((bf(bv[k][e]) * inv_b) * g);
        }
      }
    }
  }
  float ss = 0.0f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = threadIdx.x + k * BLOCK;
    if (v < nv) {
      if (has_b) {
#pragma unroll
        for (int e = 0; e < 8; ++e) av[k][e] = to_bf(bf(av[k][e]) + bf(bv[k][e]));
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ss = fmaf(bf(av[k][e]), bf(av[k][e]), ss);
    }
  }
  const float inv = 1.0f / sqrtf(row_sum<BLOCK>(ss, red[1]) / static_cast<float>(d) + eps);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = threadIdx.x + k * BLOCK;
    if (v < nv) {
      if (s_out) *reinterpret_cast<u16x8*>(s_out + r * lds + 8 * v) = av[k];
      u16x8 g8;
      if constexpr (kPre) g8 = wv[k];
      else g8 = *reinterpret_cast<const u16x8*>(w + 8 * v);
      u16x8 out;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = plus_one ? 1.0f + bf(g8[e]) : bf(g8[e]);
        // Llama (F.rms_norm): x * inv * w, one rounding; Gemma: (x * inv) * (1 + w)
        out[e] = to_bf((bf(av[k][e]) * inv) * g);
      }
      *reinterpret_cast<u16x8*>(y + r * ldy + 8 * v) = out;
    }
  }
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
}

// grid rows * nb (nb = ceil(F / (8 * 256)) blocks per row): 8 outputs per thread
__global__ __launch_bounds__(kNormThreads) void gated_act_kernel(
    const uint16_t* __restrict__ gate, int64_t ldg, const uint16_t* __restrict__ up, int64_t ldu,
    int64_t F, int nb, int act, uint16_t* __restrict__ out, int64_t ldo) {
  const int64_t r = blockIdx.x / nb;
  const int64_t j = (static_cast<int64_t>(blockIdx.x % nb) * kNormThreads + threadIdx.x) * 8;
  if (j >= F) return;
  const u16x8 g = *reinterpret_cast<const u16x8*>(gate + r * ldg + j);
  const u16x8 u = *reinterpret_cast<const u16x8*>(up + r * ldu + j);
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = bf(g[e]);
    const uint16_t a = to_bf(act ? gelu_tanh_f(x) : silu_f(x));
    o[e] = to_bf(bf(a) * bf(u[e]));
  }
  *reinterpret_cast<u16x8*>(out + r * ldo + j) = o;
}

bool norm_vpt_form() {
  static const bool v = [] {
    const char* e = getenv("CS_NORM_VPT");
    return e && atoi(e) == 1;
  }();
  return v;
}

int add_rms_launch(const char* name, const void* a, int64_t lda, const void* b, int64_t ldb,
                   const float* bp, int splits, const void* b_weight, void* s_out, int64_t lds,
                   const void* weight, int64_t rows, int64_t d, float eps, int plus_one, void* y,
                   int64_t ldy, cs_stream_t stream) {
  if (rows < 0 || d <= 0) return fail(CS_ERR_INVALID, std::string(name) + ": bad shape");
  if (rows == 0) return CS_OK;
  if (!a || !weight || !y) return fail(CS_ERR_INVALID, std::string(name) + ": NULL pointer");
  const bool has_b = b || bp;
  if (b_weight && !has_b) return fail(CS_ERR_INVALID, std::string(name) + ": b_weight without b");
  if (d % 8 != 0 || d > 16 * 8 * kNormThreads)
    return fail(CS_ERR_INVALID, std::string(name) + ": d must be a multiple of 8 and <= 32768");
  if (rows > 0x7fffffffLL) return fail(CS_ERR_INVALID, std::string(name) + ": too many rows");
  if (bp && d > 4 * 8 * kNormThreads)
    return fail(CS_ERR_INVALID, std::string(name) + ": d must be <= 8192 with split partials");
  if (lda < d || ldy < d || (b && ldb < d) || (s_out && lds < d) || lda % 8 || ldy % 8 ||
      (b && ldb % 8) || (s_out && lds % 8))
    return fail(CS_ERR_INVALID, std::string(name) + ": leading dimensions must be >= d and multiples of 8");
  const uint16_t* A = static_cast<const uint16_t*>(a);
  const uint16_t* B = static_cast<const uint16_t*>(b);
  const uint16_t* WB = static_cast<const uint16_t*>(b_weight);
  uint16_t* S = static_cast<uint16_t*>(s_out);
  const uint16_t* W = static_cast<const uint16_t*>(weight);
  uint16_t* Y = static_cast<uint16_t*>(y);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nv = static_cast<int>(d / 8);
  const dim3 grid(static_cast<uint32_t>(rows));
#define CS_ADD_RMS_FOLD(V, BL, NS)                                                                \
  hipLaunchKernelGGL((add_rms_kernel<V, true, NS, BL>), grid, dim3(BL), 0, st, A, lda, B, ldb,     \
                     WB, S, lds, W, d, eps, plus_one, Y, ldy, bp, splits)
#define CS_ADD_RMS(V, BL)                                                                         \
  if (bp) {                                                                                       \
    if (splits <= 2) CS_ADD_RMS_FOLD(V, BL, 2);                                                   \
    else if (splits <= 4) CS_ADD_RMS_FOLD(V, BL, 4);                                              \
    else if (splits <= 8) CS_ADD_RMS_FOLD(V, BL, 8);                                              \
    else CS_ADD_RMS_FOLD(V, BL, 16);                                                              \
  } else                                                                                          \
    hipLaunchKernelGGL((add_rms_kernel<V, false, kMaxSplits, BL>), grid, dim3(BL), 0, st, A, lda, \
                       B, ldb, WB, S, lds, W, d, eps, plus_one, Y, ldy, bp, splits)
  // one vector per thread up to d = 8192 (the block size depends on d only, so a norm's
  // rounding is the same at every row count).  CS_NORM_VPT=1 (A/B only): the round-4 form,
  // 256 threads with up to 4 vectors each
  if (norm_vpt_form()) {
    if (nv <= 256) {
      CS_ADD_RMS(1, 256);
    } else if (nv <= 512) {
      CS_ADD_RMS(2, 256);
    } else if (nv <= 1024) {
      CS_ADD_RMS(4, 256);
    } else {
      hipLaunchKernelGGL((add_rms_kernel<16, false>), grid, dim3(kNormThreads), 0, st, A, lda, B, ldb,
                         WB, S, lds, W, d, eps, plus_one, Y, ldy, nullptr, 0);
    }
  } else if (nv <= 256) {
    CS_ADD_RMS(1, 256);
  } else if (nv <= 512) {
    CS_ADD_RMS(1, 512);
  } else if (nv <= 1024) {
    CS_ADD_RMS(1, 1024);
  } else {       // (d > 8192: the fold is refused above)
    hipLaunchKernelGGL((add_rms_kernel<16, false>), grid, dim3(kNormThreads), 0, st, A, lda, B, ldb,
                       WB, S, lds, W, d, eps, plus_one, Y, ldy, nullptr, 0);
  }
#undef CS_ADD_RMS
#undef CS_ADD_RMS_FOLD
  return check_launch(name);
}

}  // namespace

extern "C" {

int cs_add_rms_norm(const void* a, int64_t lda, const void* b, int64_t ldb, const void* b_weight,
                    void* s_out, int64_t lds, const void* weight, int64_t rows, int64_t d, float eps,
                    int plus_one, void* y, int64_t ldy, cs_stream_t stream) {
  return add_rms_launch("cs_add_rms_norm", a, lda, b, ldb, nullptr, 0, b_weight, s_out, lds, weight,
                        rows, d, eps, plus_one, y, ldy, stream);
}

int cs_add_rms_norm_splitk(const void* a, int64_t lda, const float* partials, int32_t splits,
                           const void* b_weight, void* s_out, int64_t lds, const void* weight,
                           int64_t rows, int64_t d, float eps, int plus_one, void* y, int64_t ldy,
                           cs_stream_t stream) {
  if (!partials || splits < 1 || splits > kMaxSplits)
    return fail(CS_ERR_INVALID, "cs_add_rms_norm_splitk: partials and 1 <= splits <= 16 required");
  if (reinterpret_cast<uintptr_t>(partials) & 15)
    return fail(CS_ERR_INVALID, "cs_add_rms_norm_splitk: partials must be 16-byte aligned");
  return add_rms_launch("cs_add_rms_norm_splitk", a, lda, nullptr, 0, partials, splits, b_weight,
                        s_out, lds, weight, rows, d, eps, plus_one, y, ldy, stream);
}

int cs_gated_act(const void* gate, int64_t ld_gate, const void* up, int64_t ld_up, int64_t rows,
                 int64_t F, int act, void* out, int64_t ld_out, cs_stream_t stream) {
  if (rows < 0 || F <= 0) return fail(CS_ERR_INVALID, "cs_gated_act: bad shape");
  if (rows == 0) return CS_OK;
  if (!gate || !up || !out) return fail(CS_ERR_INVALID, "cs_gated_act: NULL pointer");
  if (act != 0 && act != 1) return fail(CS_ERR_INVALID, "cs_gated_act: act must be 0 (SiLU) or 1 (tanh-GeLU)");
  if (F % 8 || ld_gate % 8 || ld_up % 8 || ld_out % 8 || ld_gate < F || ld_up < F || ld_out < F)
    return fail(CS_ERR_INVALID, "cs_gated_act: F and leading dimensions must be multiples of 8, >= F");
  const int64_t nb = (F / 8 + kNormThreads - 1) / kNormThreads;
  if (rows * nb > 0x7fffffffLL) return fail(CS_ERR_INVALID, "cs_gated_act: grid too large");
  hipLaunchKernelGGL(gated_act_kernel, dim3(static_cast<uint32_t>(rows * nb)), dim3(kNormThreads), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t*>(gate), ld_gate,
                     static_cast<const uint16_t*>(up), ld_up, F, static_cast<int>(nb), act,
                     static_cast<uint16_t*>(out), ld_out);
  return check_launch("cs_gated_act");
}

}  // extern "C"
