// omf_common.h — shared device/host helpers of the MI355X codec (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace omf {

constexpr int kThreads = 256;           // 4 wave64 per workgroup
constexpr int kWaves = kThreads / 64;

// Thread-local error string behind omf_last_error().
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define OMF_HIP(call)                                   \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return ::omf::hip_fail(e_, #call); \
  } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// ---------------------------------------------------------------- device helpers

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Deterministic block sum (fixed butterfly per wave, fixed wave order); result valid in all threads.
__device__ __forceinline__ double block_sum_f64(double v, double* lds /* kWaves */) {
  v = wave_sum_f64(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  double s = lds[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) s += lds[w];
  __syncthreads();
  return s;
}

// Agent-scope relaxed accesses (global_load/store ... sc1): the hand-off protocol of
// cdna_hip_programming.md §6 G16 — payload stored sc1 + drained, consumer loads sc1.
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Philox4x32-10 (Salmon et al., SC'11).  Counter layout: oracle/philox.py.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
  }
  return c;
}

// 24-bit uniform in [0,1): the torch CPU generator's rule.
__device__ __forceinline__ float u24(uint32_t w) { return (float)(w & 0xFFFFFFu) * 5.9604644775390625e-08f; }

}  // namespace omf
