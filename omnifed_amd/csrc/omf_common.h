// omf_common.h — shared device/host helpers of the MI355X codec (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>

namespace omf {

constexpr int kThreads = 256;           // 4 wave64 per workgroup
constexpr int kWaves = kThreads / 64;

// Events that only order launches between streams of one device: no timing and no system-scope
// fence.  Recording an event with the default system-scope release writes back and invalidates
// the caches, and the next kernel on the stream started ~6 us later (rocprofv3 kernel trace, every
// encode call of round 3); the kernels' own completion already releases at device scope.
constexpr unsigned kOrderEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;

// Top-K encoder counters of a plan (omf_topk_stats) that the host knows: calls of the sampled
// path and of the exact path.  Which path a sampled call took (bucket-sort fast path, zero fill,
// the exact tail's fallback, a redo) is decided on the device, which counts it (omf_topk.hip).
struct TopkStats {
  int64_t calls = 0, exact = 0;
};

// Top-K encoder settings of a plan (omf_topk.hip): in experiment builds read from the OMF_TOPK_* environment once, at
// the plan's first Top-K call, and settable by the omf_plan_set_topk test / experiment hook.
struct TopkKnobs {
  TopkStats stats;
  bool init = false;
  int32_t groups = 1;          // two-stream group pipeline (off: measured slower)
  int32_t dbg = 0;             // OMF_TOPK_DBG diagnostics
  int32_t force_fallback = 0;  // 1: always the exact tail's radix sort; 2: and a barrier expiry (tests)
  int64_t sample_runs = 0;     // sampled runs per tensor at most (0: the default, 2 Ki)
  float sure_z = 1.5f, sure_c = 2.0f;  // the "sure" bin's margin below the expected rank-k count
  bool scatter_small = true;   // the bucket scatter's LDS-staged bucket table (OMF_TOPK_SCATTER_SMALL=0 off)
  bool planned_scatter = true; // the bucket plan inside the scatter launch (OMF_TOPK_PLANNED_SCATTER=0 off)
};

// Tuning knobs from the environment (OMF_TOPK_*, OMF_SPEC_*, OMF_RING_*, OMF_ENCODE_STRATEGY,
// OMF_DEC_LDS): read only by experiment builds (-DOMF_EXPERIMENTS, scripts/exp/variant_lib.sh);
// the product library ignores its environment and takes settings through the API alone
// (omf_codec_experimental.h for the test / experiment hooks).
inline const char* knob(const char* name) {
#ifdef OMF_EXPERIMENTS
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

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
// Each round's two 32x32->64 products are single 64-bit multiplies (v_mad_u64_u32).
#ifndef OMF_PHILOX_ROUNDS
#define OMF_PHILOX_ROUNDS 10
#endif
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < OMF_PHILOX_ROUNDS; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    // three-input xor in one v_bitop3_b32 (truth table 0x96)
    c = make_uint4(__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
                   __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0);
  }
  return c;
}

// 24-bit uniform in [0,1): the torch CPU generator's rule.
__device__ __forceinline__ float u24(uint32_t w) { return (float)(w & 0xFFFFFFu) * 5.9604644775390625e-08f; }

// Four 24-bit uniforms from three consecutive 32-bit words (96 bits, little-endian fields).
__device__ __forceinline__ float4 u24x4(uint32_t w0, uint32_t w1, uint32_t w2) {
  return make_float4(u24(w0), u24(__builtin_amdgcn_alignbit(w1, w0, 24)), u24(__builtin_amdgcn_alignbit(w2, w1, 16)),
                     (float)(w2 >> 8) * 5.9604644775390625e-08f);
}

// Correctly rounded x / d from r = RN(1/d): Markstein's theorem (one Newton step brings
// q within 1 ulp, the second fma-corrected step rounds correctly).  Valid for d in
// [2^-100, 2^100] and |x| >= 2^-96 or x == 0; callers take x / d elsewhere
// (scripts/exp/div_check.c: 0 mismatches in 1e9 random and near-halfway cases).
__device__ __forceinline__ float div_markstein(float x, float d, float r) {
  float q = __fmul_rn(x, r);
  float e = fmaf(-q, d, x);
  q = fmaf(e, r, q);
  e = fmaf(-q, d, x);
  return fmaf(e, r, q);
}

__device__ __forceinline__ bool div_needs_exact(float x) {
  const float a = fabsf(x);
  return a != 0.0f && !(a >= 0x1p-96f);  // tiny non-zero (or NaN): exact division
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_nt(float* p, float4 v) {
  f32x4_t t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<f32x4_t*>(p));
}
__device__ __forceinline__ void store_nt(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }
typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_nt(int32_t* p, int4 v) {
  i32x4_t t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<i32x4_t*>(p));
}

}  // namespace omf
