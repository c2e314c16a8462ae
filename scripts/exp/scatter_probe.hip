// Experiment (not product): 4-byte scattered stores (1 % of the elements, random positions)
// into an arena that was just zero-filled, window by window (the window's lines still in the
// Infinity Cache), versus one full fill followed by one full scatter.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void fill_scatter(f32x4* __restrict__ y, int64_t f0, int64_t f1,
                                                    const int64_t* __restrict__ idx, const float* __restrict__ val,
                                                    int64_t s0, int64_t s1, int64_t fill_blocks) {
  if ((int64_t)blockIdx.x < fill_blocks) {  // zero-fill float4 range [f0, f1)
    const int64_t i = f0 + (int64_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < f1) __builtin_nontemporal_store((f32x4){0.f, 0.f, 0.f, 0.f}, y + i + 256 * u);
    return;
  }
  const int64_t j = s0 + ((int64_t)blockIdx.x - fill_blocks) * 256 + threadIdx.x;
  if (j < s1) reinterpret_cast<float*>(y)[idx[j]] = val[j];
}

// window: elements per window (multiple of 4096); the selection is sorted by window (idx
// within each window's range), as the per-tensor packed Top-K selection is.
extern "C" int probe_run(void* y, int64_t n, const int64_t* idx, const float* val, const int64_t* wstart, int64_t nwin,
                         int64_t window, int mode, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  f32x4* Y = (f32x4*)y;
  if (mode == 0) {  // full fill then full scatter
    const int64_t n4 = n / 4, fb = (n4 + 1023) / 1024;
    hipLaunchKernelGGL(fill_scatter, dim3((unsigned)fb), dim3(256), 0, st, Y, (int64_t)0, n4, idx, val, (int64_t)0,
                       (int64_t)0, fb);
    const int64_t m = wstart[nwin];
    hipLaunchKernelGGL(fill_scatter, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, Y, (int64_t)0, (int64_t)0,
                       idx, val, (int64_t)0, m, (int64_t)0);
  } else {  // launch w: fill window w + 1, scatter window w
    const int64_t w4 = window / 4, fb = (w4 + 1023) / 1024;
    for (int64_t w = -1; w < nwin; ++w) {
      const bool f = w + 1 < nwin;
      const int64_t s0 = w >= 0 ? wstart[w] : 0, s1 = w >= 0 ? wstart[w + 1] : 0;
      const int64_t sb = (s1 - s0 + 255) / 256;
      const int64_t nb = (f ? fb : 0) + sb;
      if (nb == 0) continue;
      hipLaunchKernelGGL(fill_scatter, dim3((unsigned)nb), dim3(256), 0, st, Y, (w + 1) * w4, (w + 2) * w4, idx, val,
                         s0, s1, f ? fb : (int64_t)0);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
