// Pure-read calibration: how long does the MI355X take to stream N bytes with nothing
// else to do?  (tools/read_floor.py; sets the floor the small beam-shape streams are
// compared against.)
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL>
__global__ void read_kernel(const u32x4* __restrict__ p, int64_t nvec, int64_t per_wg,
                            uint32_t* __restrict__ out) {
  const int64_t v0 = static_cast<int64_t>(blockIdx.x) * per_wg;
  int64_t v1 = v0 + per_wg;
  if (v1 > nvec) v1 = nvec;
  uint32_t acc = 0;
  const int bs = blockDim.x;
  int64_t i = v0 + threadIdx.x;
  for (; i + (UNROLL - 1) * bs < v1; i += UNROLL * bs) {
    u32x4 q[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) q[u] = __builtin_nontemporal_load(p + i + u * bs);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= q[u][0] ^ q[u][1] ^ q[u][2] ^ q[u][3];
  }
  for (; i < v1; i += bs) {
    const u32x4 q = __builtin_nontemporal_load(p + i);
    acc ^= q[0] ^ q[1] ^ q[2] ^ q[3];
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads live
}

extern "C" int rf_read(const void* p, int64_t bytes, int wgs, int block, int unroll, void* out,
                       hipStream_t s) {
  const int64_t nvec = bytes / 16;
  const int64_t per_wg = (nvec + wgs - 1) / wgs;
  const u32x4* q = static_cast<const u32x4*>(p);
  uint32_t* o = static_cast<uint32_t*>(out);
  switch (unroll) {
    case 1: hipLaunchKernelGGL(read_kernel<1>, dim3(wgs), dim3(block), 0, s, q, nvec, per_wg, o); break;
    case 2: hipLaunchKernelGGL(read_kernel<2>, dim3(wgs), dim3(block), 0, s, q, nvec, per_wg, o); break;
    case 4: hipLaunchKernelGGL(read_kernel<4>, dim3(wgs), dim3(block), 0, s, q, nvec, per_wg, o); break;
    case 8: hipLaunchKernelGGL(read_kernel<8>, dim3(wgs), dim3(block), 0, s, q, nvec, per_wg, o); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
