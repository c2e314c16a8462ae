// Philox4x32-10 round products, three bit-identical formulations (a cheaper
// bit-identical Philox for the ResNet-18 encoder, whose Philox is ~3.75 v_mad_u64_u32 per element).
//   0: (uint64_t)M * c    -> v_mad_u64_u32 (omf_common.h's philox4x32_10)
//   1: __umulhi + M * c   -> v_mul_hi_u32 + v_mul_lo_u32
//   2: 16-bit halves      -> four full-rate v_mul_u32_u24 + carries
// Each thread runs `iters` Philox blocks on its own counter; the outputs are xor-folded per
// thread and compared across the variants (bit identity), and each variant is timed with HIP
// events over several launches (after a warm-up).  Build and run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/philox_variants scripts/exp/philox_variants.hip && /tmp/philox_variants
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));            \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;

template <int V>
__device__ __forceinline__ void mulhilo(uint32_t m, uint32_t c, uint32_t& hi, uint32_t& lo) {
  if (V == 0) {
    const uint64_t p = (uint64_t)m * c;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
  } else if (V == 1) {
    hi = __umulhi(m, c);
    lo = m * c;
  } else {
    const uint32_t ml = m & 0xffffu, mh = m >> 16, cl = c & 0xffffu, ch = c >> 16;
    const uint32_t p0 = __umul24(ml, cl), p1 = __umul24(mh, cl);
    const uint32_t p2 = __umul24(ml, ch), p3 = __umul24(mh, ch);
    const uint64_t mid = (uint64_t)p1 + p2;  // 33 bits
    const uint64_t low = (uint64_t)p0 + ((mid & 0xffffu) << 16);
    lo = (uint32_t)low;
    hi = p3 + (uint32_t)(mid >> 16) + (uint32_t)(low >> 32);
  }
}

template <int V>
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint32_t h0, l0, h1, l1;
    mulhilo<V>(M0, c.x, h0, l0);
    mulhilo<V>(M1, c.z, h1, l1);
    c = make_uint4(h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0);
  }
  return c;
}

template <int V>
__global__ __launch_bounds__(256) void bench(uint32_t* out, int iters, uint32_t k0, uint32_t k1) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    const uint4 r = philox<V>(make_uint4(t, (uint32_t)i, 0x1234u, 0u), k0, k1);
    acc ^= r.x ^ (r.y << 1) ^ (r.z << 2) ^ (r.w << 3);
  }
  out[t] = acc;
}

template <int V>
float run(uint32_t* d, int blocks, int iters, std::vector<uint32_t>& h) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(bench<V>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u, 11u);
  CHECK(hipDeviceSynchronize());
  constexpr int reps = 10;
  CHECK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(bench<V>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u, 11u);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipMemcpy(h.data(), d, 4 * h.size(), hipMemcpyDeviceToHost));
  return ms / reps;
}

int main() {
  const int blocks = 256 * 16, iters = 256;
  const size_t n = (size_t)blocks * 256;
  uint32_t* d = nullptr;
  CHECK(hipMalloc(&d, 4 * n));
  std::vector<uint32_t> h0(n), h1(n), h2(n);
  const float t0 = run<0>(d, blocks, iters, h0);
  const float t1 = run<1>(d, blocks, iters, h1);
  const float t2 = run<2>(d, blocks, iters, h2);
  const double blocks_total = (double)n * iters;  // Philox blocks (4 draws each)
  std::printf("{\"philox_blocks\": %.0f, \"mad_u64_ms\": %.4f, \"mulhi_lo_ms\": %.4f, \"u24_split_ms\": %.4f, "
              "\"ns_per_block\": [%.4f, %.4f, %.4f], \"identical_1\": %s, \"identical_2\": %s}\n",
              blocks_total, t0, t1, t2, 1e6 * t0 / blocks_total, 1e6 * t1 / blocks_total, 1e6 * t2 / blocks_total,
              h0 == h1 ? "true" : "false", h0 == h2 ? "true" : "false");
  CHECK(hipFree(d));
  return 0;
}
