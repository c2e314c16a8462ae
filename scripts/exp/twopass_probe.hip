// Experiment (not product): a two-pass encoder's traffic (pass A: read 4 B/elem, sum of squares;
// pass B: read 4 B/elem, write 1 B/elem) with nontemporal vs default load policy, over the
// whole arena or in windows (A on window w + 1, B on window w) that may hit the Infinity Cache.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL>
__global__ __launch_bounds__(256) void pass_a(const f32x4* __restrict__ x, float* __restrict__ part, int64_t b4,
                                              int64_t n4) {
  const int64_t b = b4 + (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = min(b + (int64_t)u * 256, b4 + n4 - 1);
    v[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) acc += v[u][0] * v[u][0] + v[u][1] * v[u][1] + v[u][2] * v[u][2] + v[u][3] * v[u][3];
  for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(part + (blockIdx.x & 1023), acc);
}

template <int U, bool NTL>
__global__ __launch_bounds__(256) void pass_b(const f32x4* __restrict__ x, int* __restrict__ q, int64_t b4, int64_t n4) {
  const int64_t b = b4 + (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = min(b + (int64_t)u * 256, b4 + n4 - 1);
    v[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b + (int64_t)u * 256;
    const int w = ((int)(v[u][0] * 3.f) & 0xff) | (((int)(v[u][1] * 3.f) & 0xff) << 8) |
                  (((int)(v[u][2] * 3.f) & 0xff) << 16) | ((int)(v[u][3] * 3.f) << 24);
    __builtin_nontemporal_store(w, q + i);
  }
}

template <bool A_NT, bool B_NT>
static void launch(const float* x, int* q, float* part, int64_t n, int64_t window, hipStream_t st) {
  constexpr int U = 2;
  const int64_t n4 = n / 4, w4 = window / 4;
  const unsigned gw = (unsigned)(w4 / (256 * U));
  const int64_t nw = n4 / w4;
  for (int64_t w = -1; w < nw; ++w) {
    if (w + 1 < nw)
      hipLaunchKernelGGL((pass_a<U, A_NT>), dim3(gw), dim3(256), 0, st, (const f32x4*)x, part, (w + 1) * w4, w4);
    if (w >= 0) hipLaunchKernelGGL((pass_b<U, B_NT>), dim3(gw), dim3(256), 0, st, (const f32x4*)x, q, w * w4, w4);
  }
}

// window = n: the two full passes.  pol: bit 0 = A nontemporal, bit 1 = B nontemporal.
extern "C" int twopass_run(const void* x, void* q, void* part, int64_t n, int64_t window, int pol, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const float* X = (const float*)x;
  int* Q = (int*)q;
  float* P = (float*)part;
  if (window == n) {  // A over everything, then B over everything
    const int64_t n4 = n / 4;
    const unsigned g = (unsigned)(n4 / 512);
    if (pol & 1) hipLaunchKernelGGL((pass_a<2, true>), dim3(g), dim3(256), 0, st, (const f32x4*)X, P, (int64_t)0, n4);
    else hipLaunchKernelGGL((pass_a<2, false>), dim3(g), dim3(256), 0, st, (const f32x4*)X, P, (int64_t)0, n4);
    if (pol & 2) hipLaunchKernelGGL((pass_b<2, true>), dim3(g), dim3(256), 0, st, (const f32x4*)X, Q, (int64_t)0, n4);
    else hipLaunchKernelGGL((pass_b<2, false>), dim3(g), dim3(256), 0, st, (const f32x4*)X, Q, (int64_t)0, n4);
  } else {
    switch (pol) {
      case 0: launch<false, false>(X, Q, P, n, window, st); break;
      case 1: launch<true, false>(X, Q, P, n, window, st); break;
      case 2: launch<false, true>(X, Q, P, n, window, st); break;
      default: launch<true, true>(X, Q, P, n, window, st); break;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
