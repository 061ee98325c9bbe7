// Microbenchmark: placing one V^T column (one slot of a [D][32] tile) per stream.
// mode 0: 2-byte store per d row (today's rope_place); 1: 16-byte read-modify-write of the
// chunk holding the slot; 2: whole 64-byte row read-modify-write.  Timed with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int D = 128, HKV = 8, LDH = 512;

template <int MODE>
__global__ __launch_bounds__(256) void place(uint16_t* vth, const uint16_t* src, int n_str, int slot) {
  const int64_t i = blockIdx.x * 256LL + threadIdx.x;           // (stream, g, d)
  if (i >= (int64_t)n_str * HKV * D) return;
  const int d = i % D;
  const int64_t sg = i / D;
  const uint16_t v = src[i];
  uint16_t* row = vth + (sg * LDH + (slot & ~31)) * D + (int64_t)d * 32;
  if (MODE == 0) {
    row[slot & 31] = v;
  } else if (MODE == 1) {
    u32x4* c = reinterpret_cast<u32x4*>(row + ((slot & 31) & ~7));
    u32x4 x = *c;
    const int w = (slot & 7) >> 1;
    uint32_t word = x[w];
    word = (slot & 1) ? ((word & 0xffffu) | ((uint32_t)v << 16)) : ((word & 0xffff0000u) | v);
    x[w] = word;
    *c = x;
  } else {
    u32x4* c = reinterpret_cast<u32x4*>(row);
    u32x4 x[4] = {c[0], c[1], c[2], c[3]};
    const int q = (slot & 31) >> 3, w = (slot & 7) >> 1;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k == q) {
        uint32_t word = x[k][w];
        word = (slot & 1) ? ((word & 0xffffu) | ((uint32_t)v << 16)) : ((word & 0xffff0000u) | v);
        x[k][w] = word;
      }
    c[0] = x[0]; c[1] = x[1]; c[2] = x[2]; c[3] = x[3];
  }
}

int main() {
  for (int n_str : {528, 2112}) {
    size_t nv = (size_t)n_str * HKV * LDH * D;
    uint16_t *vth, *src;
    hipMalloc(&vth, nv * 2);
    hipMalloc(&src, (size_t)n_str * HKV * D * 2);
    hipMemset(vth, 0, nv * 2);
    hipMemset(src, 1, (size_t)n_str * HKV * D * 2);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int n = n_str * HKV * D, grid = (n + 255) / 256;
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        for (int it = 0; it < 50; ++it) {
          const int slot = 100 + it;
          if (mode == 0) place<0><<<grid, 256>>>(vth, src, n_str, slot);
          if (mode == 1) place<1><<<grid, 256>>>(vth, src, n_str, slot);
          if (mode == 2) place<2><<<grid, 256>>>(vth, src, n_str, slot);
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep) printf("{\"n_str\": %d, \"mode\": %d, \"us\": %.2f}\n", n_str, mode, ms * 1e3 / 50);
      }
    }
    hipFree(vth);
    hipFree(src);
  }
  return 0;
}
