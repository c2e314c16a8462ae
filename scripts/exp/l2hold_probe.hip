// Experiment (not product): can each CU's L2 (4 MiB per XCD) hold a chunk between its first read
// (norm partial) and its re-read (quantise) H chunk-steps later?  Persistent grid, one
// 1024-thread workgroup per CU, workgroup g owns chunks g, g + G, ... (64 KiB each).  Step k
// reads chunk k (sum of squares) and re-reads chunk k - H (f32 -> i8 store).  No cross-CU sync.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NT 1024

template <int PER>  // float4 per thread per chunk (4: 64 KiB chunks)
__global__ __launch_bounds__(NT) void hold(const float4* __restrict__ x, uint32_t* __restrict__ q,
                                           float* __restrict__ part, int64_t nchunks, int H) {
  const int t = threadIdx.x;
  const int64_t G = gridDim.x;
  float acc = 0.f;
  for (int64_t s = 0;; ++s) {
    const int64_t ka = (int64_t)blockIdx.x + s * G;        // fresh chunk
    const int64_t kb = (int64_t)blockIdx.x + (s - H) * G;  // chunk read H steps ago
    if (kb >= nchunks) break;
    float4 va[PER], vb[PER];
    if (ka < nchunks) {
      const float4* p = x + ka * (NT * PER);
#pragma unroll
      for (int j = 0; j < PER; ++j) va[j] = p[j * NT + t];
    }
    if (s >= H) {
      const float4* p = x + kb * (NT * PER);
#pragma unroll
      for (int j = 0; j < PER; ++j) vb[j] = p[j * NT + t];
    }
    if (ka < nchunks) {
#pragma unroll
      for (int j = 0; j < PER; ++j)
        acc = fmaf(va[j].x, va[j].x, fmaf(va[j].y, va[j].y, fmaf(va[j].z, va[j].z, fmaf(va[j].w, va[j].w, acc))));
    }
    if (s >= H) {
      uint32_t* d = q + kb * (NT * PER);
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const uint32_t w = (uint32_t)(vb[j].x > 0) | ((uint32_t)(vb[j].y > 0) << 8) | ((uint32_t)(vb[j].z > 0) << 16) |
                           ((uint32_t)(vb[j].w > 0) << 24);
        __builtin_nontemporal_store(w, d + j * NT + t);
      }
    }
  }
  if (acc == 1234.5f) part[0] = acc;
}

extern "C" int hold_run(const void* x, void* q, void* part, int64_t n, int H, int grid, int per, void* stream) {
  const int64_t nchunks = n / (NT * per * 4);
  if (per == 1)
    hipLaunchKernelGGL(hold<1>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, (const float4*)x, (uint32_t*)q,
                       (float*)part, nchunks, H);
  else if (per == 2)
    hipLaunchKernelGGL(hold<2>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, (const float4*)x, (uint32_t*)q,
                       (float*)part, nchunks, H);
  else
    hipLaunchKernelGGL(hold<4>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, (const float4*)x, (uint32_t*)q,
                       (float*)part, nchunks, H);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
