// Experiment (not product): the streaming floor of the Top-K error-feedback pass
// r := r + alpha * x (read 8 B, write 4 B per element) under different kernel shapes.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NTS, bool NTL>
__global__ __launch_bounds__(256) void ef_stream(const f32x4* __restrict__ x, f32x4* __restrict__ r, float a,
                                                 int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n4; b += stride) {
    f32x4 xv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = min(b + (int64_t)u * 256, n4 - 1);
      xv[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
      rv[u] = r[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = b + (int64_t)u * 256;
      if (i < n4) {
        const f32x4 t = rv[u] + xv[u] * a;
        if (NTS) __builtin_nontemporal_store(t, r + i);
        else r[i] = t;
      }
    }
  }
}

// one block per 16 Ki-element item, two passes of 8 float4 per thread (topk_fused's shape)
template <bool NTS>
__global__ __launch_bounds__(256) void ef_items(const f32x4* __restrict__ x, f32x4* __restrict__ r, float a,
                                                int64_t n4) {
  const int64_t b0 = (int64_t)blockIdx.x * 4096;
  for (int p = 0; p < 2; ++p) {
    const int64_t b = b0 + p * 2048 + threadIdx.x;
    f32x4 xv[8], rv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = min(b + (int64_t)u * 256, n4 - 1);
      xv[u] = x[i];
      rv[u] = r[i];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = b + (int64_t)u * 256;
      if (i < n4) {
        const f32x4 t = rv[u] + xv[u] * a;
        if (NTS) __builtin_nontemporal_store(t, r + i);
        else r[i] = t;
      }
    }
    __syncthreads();
  }
}

// non-persistent: each thread U float4 of each input (blocks of B threads), then exits
template <int U, int B, bool NTS>
__global__ __launch_bounds__(B) void ef_flat(const f32x4* __restrict__ x, f32x4* __restrict__ r, float a, int64_t n4) {
  const int64_t b = (int64_t)blockIdx.x * B * U + threadIdx.x;
  f32x4 xv[U], rv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = min(b + (int64_t)u * B, n4 - 1);
    xv[u] = x[i];
    rv[u] = r[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b + (int64_t)u * B;
    if (i < n4) {
      const f32x4 t = rv[u] + xv[u] * a;
      if (NTS) __builtin_nontemporal_store(t, r + i);
      else r[i] = t;
    }
  }
}
#define FLAT(U, B, NTS) hipLaunchKernelGGL((ef_flat<U, B, NTS>), dim3((unsigned)((n4 + B * U - 1) / (B * U))), dim3(B), 0, st, X, R, 1.0f, n4)

extern "C" int ef_run(int variant, const void* x, void* r, int64_t n, int grid, void* stream) {
  const int64_t n4 = n / 4;
  hipStream_t st = (hipStream_t)stream;
  const f32x4* X = (const f32x4*)x;
  f32x4* R = (f32x4*)r;
  switch (variant) {
    case 0: hipLaunchKernelGGL((ef_stream<4, false, false>), dim3(grid), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 1: hipLaunchKernelGGL((ef_stream<4, true, false>), dim3(grid), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 2: hipLaunchKernelGGL((ef_stream<4, true, true>), dim3(grid), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 3: hipLaunchKernelGGL((ef_stream<8, false, false>), dim3(grid), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 4: hipLaunchKernelGGL((ef_stream<8, true, false>), dim3(grid), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 5: hipLaunchKernelGGL((ef_stream<2, true, false>), dim3(grid), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 6: hipLaunchKernelGGL((ef_items<false>), dim3((unsigned)((n4 + 4095) / 4096)), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 7: hipLaunchKernelGGL((ef_items<true>), dim3((unsigned)((n4 + 4095) / 4096)), dim3(256), 0, st, X, R, 1.0f, n4); break;
    case 8: FLAT(1, 256, false); break;
    case 9: FLAT(2, 256, false); break;
    case 10: FLAT(4, 256, false); break;
    case 11: FLAT(1, 512, false); break;
    case 12: FLAT(2, 512, false); break;
    case 13: FLAT(4, 512, false); break;
    case 14: FLAT(1, 1024, false); break;
    case 15: FLAT(2, 256, true); break;
    case 16: FLAT(4, 256, true); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
