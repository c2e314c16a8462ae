// omf_qsgd_dev.h — QSGD element arithmetic shared by every encoder (gfx950).
//
// Semantics: SURVEY.md §8a "Exact QSGD semantics", restating
//   src/omnifed/hybrid/compression/qsgd.py:50-63 (reference, Python/torch CPU):
//   vn = RN(x / norm); sc = |vn| * L; lo = floor(sc); p = sc - lo;
//   q = clamp(lo + (u < p), 0, L) * sign(vn)   (int64 in the reference, then int8/int32)
// Every step after the division is exact in fp32.  The reference's x86 float->int64
// conversion maps NaN and |sc| >= 2^63 to INT64_MIN, which the clamp turns into 0.
//
// Instruction budget (the encoders are VALU-co-bound with HBM): the
// division is Markstein's correctly rounded form on packed pairs (v_pk_mul/v_pk_fma);
// the level uses a NaN-propagating minimum (v_minimum3) for the clamp, copysign (v_bfi)
// + v_cvt_i32_f32 (NaN -> 0) for the sign, and no integer multiply.
#pragma once

#include "omf_common.h"

namespace omf {

typedef float f32x2_t __attribute__((ext_vector_type(2)));

// Value formats: the dtype the reference computes in (qsgd.py:46-58 runs in the tensor's own
// dtype).  The arena always holds fp32 (a bf16/fp16 tensor upcast exactly); in a reduced
// format the encoder rounds where torch's bf16/fp16 CPU ops round: the weighted input
// (torch.mul(param, batch_samples)), the norm (torch.norm(v).item()) and v / norm.  The
// rest of the chain is exact (|vn| * 2^s, floor, the fp32 fraction: prob_round_up is
// promoted to fp32 by `- lower.float()`).
enum : uint32_t { kFmtF32 = 0, kFmtBF16 = 1, kFmtF16 = 2 };

// Round to nearest even, as c10::BFloat16(float) / c10::Half(float) do (NaN stays NaN).
__device__ __forceinline__ float round_bf16(float f) {
  if (f != f) return f;
  const uint32_t u = __float_as_uint(f);
  return __uint_as_float((u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u);
}
__device__ __forceinline__ float round_f16(float f) { return (float)(_Float16)f; }
__device__ __forceinline__ float round_fmt(float f, uint32_t fmt) {
  return fmt == kFmtBF16 ? round_bf16(f) : (fmt == kFmtF16 ? round_f16(f) : f);
}
__device__ __forceinline__ float4 round_fmt4(float4 v, uint32_t fmt) {
  return make_float4(round_fmt(v.x, fmt), round_fmt(v.y, fmt), round_fmt(v.z, fmt), round_fmt(v.w, fmt));
}
// The tensor norm from its sum of squares: fp32 sqrt (torch.norm's result), then the format.
__device__ __forceinline__ float finish_norm(double sumsq, uint32_t fmt) { return round_fmt(sqrtf((float)sumsq), fmt); }

__device__ __forceinline__ f32x2_t fma2(f32x2_t a, f32x2_t b, f32x2_t c) { return __builtin_elementwise_fma(a, b, c); }

// Correctly rounded x / d from r = RN(1/d) on a pair (see div_markstein in omf_common.h).
__device__ __forceinline__ f32x2_t div2_markstein(f32x2_t x, f32x2_t d, f32x2_t r) {
  f32x2_t q = x * r;
  f32x2_t e = fma2(-q, d, x);
  q = fma2(e, r, q);
  e = fma2(-q, d, x);
  return fma2(e, r, q);
}

// 0 < |x| < 2^-96 (frexp exponent < -95; zero, inf and NaN report 0): Markstein's bound.
__device__ __forceinline__ bool div_tiny(float x) { return __builtin_amdgcn_frexp_expf(x) < -95; }

// Per-tensor divisor state: IEEE x / norm, fast (Markstein) when norm is in range.
struct Divisor {
  float d, r;
  bool fast;
  uint32_t fmt;  // value format of the quotient (v / norm is rounded to it)
  __device__ __forceinline__ explicit Divisor(float norm, uint32_t fmt_ = kFmtF32) : d(norm), r(1.0f / norm), fmt(fmt_) {
    const float a = fabsf(norm);
    fast = a >= 0x1p-100f && a <= 0x1p100f;
  }
  __device__ __forceinline__ float4 div4(float4 x) const {
    const float4 q = div4_f32(x);
    return fmt ? round_fmt4(q, fmt) : q;  // uniform branch
  }
  __device__ __forceinline__ float4 div4_f32(float4 x) const {
    if (!fast) return make_float4(x.x / d, x.y / d, x.z / d, x.w / d);
    const f32x2_t D = {d, d}, R = {r, r};
    const f32x2_t lo = div2_markstein((f32x2_t){x.x, x.y}, D, R);
    const f32x2_t hi = div2_markstein((f32x2_t){x.z, x.w}, D, R);
    float4 q = make_float4(lo.x, lo.y, hi.x, hi.y);
    // Quad pre-test (v_min3 with |.| modifiers): min |x| < 2^-96 catches every tiny input
    // (and zeros, which Markstein divides exactly anyway); only then the per-element test.
    const float mn = fminf(fminf(fabsf(x.x), fabsf(x.y)), fminf(fabsf(x.z), fabsf(x.w)));
    if (__any(mn < 0x1p-96f)) {  // wave-uniform branch: tiny inputs take the exact division
      if (div_tiny(x.x)) q.x = x.x / d;
      if (div_tiny(x.y)) q.y = x.y / d;
      if (div_tiny(x.z)) q.z = x.z / d;
      if (div_tiny(x.w)) q.w = x.w / d;
    }
    return q;
  }
};

// One QSGD level from vn = RN(x / norm) (exact semantics above).  a >= 2^63 is handled by
// the caller (qsgd_quad) so that this stays branch-free.
__device__ __forceinline__ int32_t qsgd_level_fast(float vn, float L, float u) {
  const float a = fabsf(__fmul_rn(vn, L));
  const float fl = floorf(a);
  const float p = __fsub_rn(a, fl);
  float m = (u < p) ? __fadd_rn(fl, 1.0f) : fl;  // exact: p > 0 implies fl < 2^23
  m = __builtin_elementwise_minimum(m, L);        // clamp; NaN stays NaN
  return (int32_t)copysignf(m, vn);               // v_cvt_i32_f32: NaN -> 0
}

// Scalar form (tests / reference comments): identical results.
__device__ __forceinline__ int32_t qsgd_level(float vn, float L, float u) {
  const float a = fabsf(__fmul_rn(vn, L));
  if (!(a < 9.2233720e18f)) return 0;  // NaN / >= 2^63: INT64_MIN, clamped to 0
  return qsgd_level_fast(vn, L, u);
}

// Four levels of x (already scaled by alpha) with uniforms u.  `zero`: norm == 0 (all-zero
// payload; the Python layer sends the tensor dense, qsgd.py:47-48).  CHECK_BIG = false only
// where the norm is the encoder's own (|x| <= norm, so |vn| * L cannot reach 2^63).
template <bool CHECK_BIG = true>
__device__ __forceinline__ void qsgd_quad(float4 x, float4 u, const Divisor& dv, float L, bool zero,
                                          int32_t (&q)[4]) {
  if (zero) {
    q[0] = q[1] = q[2] = q[3] = 0;
    return;
  }
  const float4 vn = dv.div4(x);
  q[0] = qsgd_level_fast(vn.x, L, u.x);
  q[1] = qsgd_level_fast(vn.y, L, u.y);
  q[2] = qsgd_level_fast(vn.z, L, u.z);
  q[3] = qsgd_level_fast(vn.w, L, u.w);
  if (dv.fmt == kFmtF16) {  // fp16 |vn| * L >= 65520 is inf in the reference: level 0
    if (!(fabsf(__fmul_rn(vn.x, L)) < 65520.0f)) q[0] = 0;
    if (!(fabsf(__fmul_rn(vn.y, L)) < 65520.0f)) q[1] = 0;
    if (!(fabsf(__fmul_rn(vn.z, L)) < 65520.0f)) q[2] = 0;
    if (!(fabsf(__fmul_rn(vn.w, L)) < 65520.0f)) q[3] = 0;
  }
  if (!CHECK_BIG) return;
  // |vn| * L >= 2^63 (only with a caller-supplied norm far below |x|): the reference's
  // int64 conversion overflows to INT64_MIN and clamps to 0.  One test per quad.
  const float big = fmaxf(fmaxf(fabsf(vn.x), fabsf(vn.y)), fmaxf(fabsf(vn.z), fabsf(vn.w)));
  if (__any(!(__fmul_rn(big, L) < 9.2233720e18f) && big == big)) {
    if (!(fabsf(__fmul_rn(vn.x, L)) < 9.2233720e18f)) q[0] = 0;
    if (!(fabsf(__fmul_rn(vn.y, L)) < 9.2233720e18f)) q[1] = 0;
    if (!(fabsf(__fmul_rn(vn.z, L)) < 9.2233720e18f)) q[2] = 0;
    if (!(fabsf(__fmul_rn(vn.w, L)) < 9.2233720e18f)) q[3] = 0;
  }
}

__device__ __forceinline__ uint32_t pack_i8x4(const int32_t (&q)[4]) {
  return (uint32_t)(uint8_t)q[0] | ((uint32_t)(uint8_t)q[1] << 8) | ((uint32_t)(uint8_t)q[2] << 16) |
         ((uint32_t)(uint8_t)q[3] << 24);
}

}  // namespace omf
