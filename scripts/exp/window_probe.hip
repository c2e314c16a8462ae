// Experiment (not product): can a windowed two-pass encoder get its second read from the
// 256 MiB Infinity Cache?  Launch w reads window w+1 (sum of squares, "norm pass") and
// converts window w (f32 -> i8, "quant pass"); the kernel boundary is the only sync.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NT 256
#define PER 16  // float4 per thread per item: 16 Ki elements per item

__global__ __launch_bounds__(NT) void pipe(const float4* __restrict__ x, uint32_t* __restrict__ q,
                                           float* __restrict__ part, int64_t a0, int64_t a_items, int64_t b0,
                                           int64_t b_items, int interleave) {
  int64_t i = blockIdx.x;
  bool is_a;
  int64_t k;
  if (interleave) {
    // alternate A and B items while both last
    const int64_t m = a_items < b_items ? a_items : b_items;
    if (i < 2 * m) { is_a = (i & 1) == 0; k = i >> 1; }
    else { k = m + (i - 2 * m); is_a = a_items > b_items; }
  } else {
    is_a = i < a_items;
    k = is_a ? i : i - a_items;
  }
  const int t = threadIdx.x;
  if (is_a) {
    const float4* p = x + (a0 + k * NT * PER);
    float acc = 0.f;
    float4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) v[j] = p[j * NT + t];
#pragma unroll
    for (int j = 0; j < PER; ++j) acc = fmaf(v[j].x, v[j].x, fmaf(v[j].y, v[j].y, fmaf(v[j].z, v[j].z, fmaf(v[j].w, v[j].w, acc))));
    for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o);
    if ((t & 63) == 0) atomicAdd(part + (k & 1023), acc);
  } else {
    const float4* p = x + (b0 + k * NT * PER);
    uint32_t* d = q + (b0 + k * NT * PER);
    float4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) v[j] = p[j * NT + t];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      uint32_t w = (uint32_t)(v[j].x > 0) | ((uint32_t)(v[j].y > 0) << 8) | ((uint32_t)(v[j].z > 0) << 16) |
                   ((uint32_t)(v[j].w > 0) << 24);
      __builtin_nontemporal_store(w, d + j * NT + t);
    }
  }
}

// window_elems multiple of 16384; n multiple of window
extern "C" int window_run(const void* x, void* q, void* part, int64_t n, int64_t window, int interleave,
                          int reverse_b, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int64_t per_item = (int64_t)NT * PER * 4;  // elements
  const int64_t nw = n / window;
  const int64_t wi = window / per_item;
  if (reverse_b == 2) {  // convert pass alone (floor)
    hipLaunchKernelGGL(pipe, dim3((unsigned)(n / per_item)), dim3(NT), 0, st, (const float4*)x, (uint32_t*)q,
                       (float*)part, (int64_t)0, (int64_t)0, (int64_t)0, n / per_item, 0);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  for (int64_t w = -1; w < nw; ++w) {
    const int64_t a_items = (w + 1 < nw) ? wi : 0;
    const int64_t b_items = (w >= 0) ? wi : 0;
    const int64_t a0 = (w + 1) * window / 4, b0 = w * window / 4;
    hipLaunchKernelGGL(pipe, dim3((unsigned)(a_items + b_items)), dim3(NT), 0, st, (const float4*)x, (uint32_t*)q,
                       (float*)part, a0, a_items, b0 < 0 ? 0 : b0, b_items, interleave);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
