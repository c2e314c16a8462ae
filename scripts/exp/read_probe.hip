// Experiment (not product): read-only streaming (sum of squares) shapes: U float4 per thread,
// B threads per block, default or nontemporal loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U, int B, bool NT>
__global__ __launch_bounds__(B) void rd(const f32x4* __restrict__ x, float* __restrict__ part, int64_t n4) {
  const int64_t b = (int64_t)blockIdx.x * B * U + threadIdx.x;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = min(b + (int64_t)u * B, n4 - 1);
    v[u] = NT ? __builtin_nontemporal_load(x + i) : x[i];
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) acc += v[u][0] * v[u][0] + v[u][1] * v[u][1] + v[u][2] * v[u][2] + v[u][3] * v[u][3];
  for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0 && acc == 1234.5f) part[0] = acc;
}

#define RD(U, B, NT) hipLaunchKernelGGL((rd<U, B, NT>), dim3((unsigned)((n4 + (int64_t)B * U - 1) / ((int64_t)B * U))), dim3(B), 0, st, (const f32x4*)x, (float*)part, n4)

extern "C" int probe_run(int v, const void* x, void* part, int64_t n, void* stream) {
  const int64_t n4 = n / 4;
  hipStream_t st = (hipStream_t)stream;
  switch (v) {
    case 0: RD(1, 256, false); break;
    case 1: RD(2, 256, false); break;
    case 2: RD(4, 256, false); break;
    case 3: RD(8, 256, false); break;
    case 4: RD(16, 256, false); break;
    case 5: RD(1, 256, true); break;
    case 6: RD(4, 256, true); break;
    case 7: RD(16, 256, true); break;
    case 8: RD(4, 512, false); break;
    case 9: RD(4, 1024, false); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
