// Experiment (not product): the cost of a small dependent launch after a streaming pass —
// empty workgroups of various counts, and one or two dependent global loads per thread.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_pass(const f32x4* __restrict__ x, uint32_t* __restrict__ q, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (i + 256 * u < n4) {
      const f32x4 v = __builtin_nontemporal_load(x + i + 256 * u);
      __builtin_nontemporal_store((uint32_t)(v[0] > 0.f) | ((uint32_t)(v[1] > 0.f) << 8), q + i + 256 * u);
    }
  }
}

__global__ __launch_bounds__(256) void empty_k(int* __restrict__ out) {
  if (threadIdx.x == 1000) out[0] = 1;
}

__global__ __launch_bounds__(256) void dep_loads(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                 uint32_t* __restrict__ out, int64_t n, int depth) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t v = a[i];
  if (depth > 1) v = b[v & 0xFFFFF];
  if (v == 0x12345678u) out[i] = v;
}

extern "C" int probe_run(int mode, int64_t wgs, void* x, void* q, int64_t n4, void* a, void* b, void* out,
                         void* stream) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(stream_pass, dim3((unsigned)((n4 + 1023) / 1024)), dim3(256), 0, st, (const f32x4*)x,
                     (uint32_t*)q, n4);
  if (mode == 1) hipLaunchKernelGGL(empty_k, dim3((unsigned)wgs), dim3(256), 0, st, (int*)out);
  if (mode == 2 || mode == 3)
    hipLaunchKernelGGL(dep_loads, dim3((unsigned)wgs), dim3(256), 0, st, (const uint32_t*)a, (const uint32_t*)b,
                       (uint32_t*)out, wgs * 256, mode == 2 ? 1 : 2);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
