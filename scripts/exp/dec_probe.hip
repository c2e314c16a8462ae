// Experiment (not product): streaming shapes for the QSGD decoder's traffic (read 1 B, write
// 4 B per element) and the encoder's (read 4 B, write 1 B), with default / nontemporal policy.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 expand(int w, float s) {
  return (f32x4){(float)(int8_t)(w & 0xff), (float)(int8_t)((w >> 8) & 0xff), (float)(int8_t)((w >> 16) & 0xff),
                 (float)(int8_t)(w >> 24)} * s;
}

// decode shape: U int32 (4 elements each) per thread, blocks of 256 threads, grid covers n
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void dec_flat(const int* __restrict__ q, f32x4* __restrict__ y, float s, int64_t n4) {
  const int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  int w[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = min(b + (int64_t)u * 256, n4 - 1);
    w[u] = NTL ? __builtin_nontemporal_load(q + i) : q[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b + (int64_t)u * 256;
    if (i < n4) {
      const f32x4 v = expand(w[u], s);
      if (NTS) __builtin_nontemporal_store(v, y + i);
      else y[i] = v;
    }
  }
}

// decode shape, 16 bytes of q per thread (16 elements -> 4 float4)
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void dec_vec(const i32x4* __restrict__ q, f32x4* __restrict__ y, float s, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n16) return;
  const i32x4 w = NTL ? __builtin_nontemporal_load(q + i) : q[i];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x4 v = expand(w[c], s);
    if (NTS) __builtin_nontemporal_store(v, y + 4 * i + c);
    else y[4 * i + c] = v;
  }
}

// encoder shape: read U float4 per thread, write U int32 (4 x int8)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void enc_flat(const f32x4* __restrict__ x, int* __restrict__ q, float s, int64_t n4) {
  const int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = min(b + (int64_t)u * 256, n4 - 1);
    v[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b + (int64_t)u * 256;
    if (i < n4) {
      const int w = ((int)(v[u][0] * s) & 0xff) | (((int)(v[u][1] * s) & 0xff) << 8) | (((int)(v[u][2] * s) & 0xff) << 16) |
                    ((int)(v[u][3] * s) << 24);
      if (NTS) __builtin_nontemporal_store(w, q + i);
      else q[i] = w;
    }
  }
}

#define DEC(U, L, S) hipLaunchKernelGGL((dec_flat<U, L, S>), dim3((unsigned)((n4 + 256 * U - 1) / (256 * U))), dim3(256), 0, st, (const int*)q, (f32x4*)y, 0.5f, n4)
#define DECV(L, S) hipLaunchKernelGGL((dec_vec<L, S>), dim3((unsigned)((n4 / 4 + 255) / 256)), dim3(256), 0, st, (const i32x4*)q, (f32x4*)y, 0.5f, n4 / 4)
#define ENC(U, L, S) hipLaunchKernelGGL((enc_flat<U, L, S>), dim3((unsigned)((n4 + 256 * U - 1) / (256 * U))), dim3(256), 0, st, (const f32x4*)y, (int*)q, 3.0f, n4)

extern "C" int probe_run(int v, void* q, void* y, int64_t n, void* stream) {
  const int64_t n4 = n / 4;
  hipStream_t st = (hipStream_t)stream;
  switch (v) {
    case 0: DEC(1, false, true); break;
    case 1: DEC(1, true, true); break;
    case 2: DEC(4, false, true); break;
    case 3: DEC(4, true, true); break;
    case 4: DECV(false, true); break;
    case 5: DECV(true, true); break;
    case 6: DEC(1, true, false); break;
    case 7: DEC(1, false, false); break;
    case 10: ENC(1, false, false); break;
    case 11: ENC(1, true, false); break;
    case 12: ENC(1, true, true); break;
    case 13: ENC(4, true, true); break;
    case 14: ENC(2, true, true); break;
    case 15: ENC(1, false, true); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
