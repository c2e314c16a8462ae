// omf_qsgd_pack.hip — opt-in bit-packed QSGD wire format, MI355X (gfx950).
//
// NOT reference-compatible: a new compression_type ("QSGDBitPackedCompression") that a
// sender uses only when asked to.  The levels q in [-L, L] of the reference wire (int8 or
// int32 per element, global_grpc_compression.py:111-123) become the codes q + L in
// b = ceil(log2(2L + 1)) bits (s = 4: 6 bits instead of 8; s = 8: 10 instead of 32),
// LSB-first little-endian: element i of a tensor occupies bits [i*b, (i+1)*b) of the
// tensor's stream.  In a plan's packed arena, tensor t's stream starts at 32-bit word
// offset_t * b / 32 (arena offsets are multiples of 64 elements, so this is exact), so 32
// consecutive elements are exactly b words and one thread packs or unpacks them alone.
// Decoding the codes gives the same floats as decoding the levels (qsgd_decode_flat's
// arithmetic: fl32(fl32(norm * q) / L)).
#include <algorithm>
#include <cstdint>

#include "../../include/omf_codec.h"
#include "omf_common.h"

using namespace omf;

namespace {

struct Item {  // the plan's flat items (omf_qsgd.hip): 16 Ki-element sub-chunks
  int64_t begin, end;
  int32_t tensor, kind, chunk, pad;
};

// B: compile-time code width (2..10, s = 0..8), or 0 = the runtime width b.
template <int WIDTH, int B>
__global__ __launch_bounds__(kThreads) void qsgd_pack(const void* __restrict__ q, const Item* __restrict__ items,
                                                      int32_t L, int32_t b_rt, uint32_t* __restrict__ out) {
  const int b = B ? B : b_rt;
  const Item it = items[blockIdx.x];
  for (int64_t e0 = it.begin + 32 * (int64_t)threadIdx.x; e0 < it.end; e0 += 32 * (int64_t)kThreads) {
    const int nv = (int)min((int64_t)32, it.end - e0);
    int32_t lv[32];
    if (WIDTH == 1) {
      const int8_t* q8 = static_cast<const int8_t*>(q) + e0;
      if (nv == 32) {
        const uint4 w0 = *reinterpret_cast<const uint4*>(q8), w1 = *reinterpret_cast<const uint4*>(q8 + 16);
        const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int i = 0; i < 32; ++i) lv[i] = (int32_t)(int8_t)(w[i >> 2] >> (8 * (i & 3)));
      } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) lv[i] = i < nv ? (int32_t)q8[i] : -L;
      }
    } else {
      const int32_t* q32 = static_cast<const int32_t*>(q) + e0;
      if (nv == 32) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          const int4 w = *reinterpret_cast<const int4*>(q32 + 4 * v);
          lv[4 * v] = w.x; lv[4 * v + 1] = w.y; lv[4 * v + 2] = w.z; lv[4 * v + 3] = w.w;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) lv[i] = i < nv ? q32[i] : -L;
      }
    }
    uint32_t* o = out + (e0 >> 5) * (int64_t)b;
    uint64_t acc = 0;
    int nb = 0, w = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      acc |= (uint64_t)(uint32_t)(lv[i] + L) << nb;  // padding (i >= nv) packs code 0
      nb += b;
      if (nb >= 32) {
        o[w++] = (uint32_t)acc;
        acc >>= 32;
        nb -= 32;
      }
    }
  }
}

// Decode: each thread unpacks its 32 elements (b words), then the workgroup transposes
// through LDS (33-word rows: conflict-free both ways) so the fp32 stores are lane-contiguous
// 16-byte non-temporal stores, like qsgd_decode_flat's.
template <int B, bool ACC, bool POW2>
__global__ __launch_bounds__(kThreads) void qsgd_decode_packed(const uint32_t* __restrict__ packed,
                                                               const Item* __restrict__ items,
                                                               const float* __restrict__ norm, float* __restrict__ y,
                                                               int32_t L, int32_t b_rt, float levels, float inv_levels) {
  constexpr int G = 32 * kThreads;  // elements per pass
  __shared__ float tile[kThreads * 33];
  const int b = B ? B : b_rt;
  const Item it = items[blockIdx.x];
  const float nrm = norm[it.tensor];
  const uint64_t mask = (1ull << b) - 1ull;
  for (int64_t base = it.begin; base < it.end; base += G) {
    const int64_t e0 = base + 32 * (int64_t)threadIdx.x;
    if (e0 < it.end) {
      const uint32_t* p = packed + (e0 >> 5) * (int64_t)b;
      uint32_t wd[B ? B : 32];
      if (B) {
#pragma unroll
        for (int i = 0; i < (B ? B : 1); ++i) wd[i] = p[i];  // every word up front
      } else {
        for (int i = 0; i < b; ++i) wd[i] = p[i];
      }
      uint64_t acc = 0;
      int nb = 0, w = 0;
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        if (nb < b) {
          acc |= (uint64_t)wd[w++] << nb;
          nb += 32;
        }
        const int32_t qi = (int32_t)(acc & mask) - L;
        acc >>= b;
        nb -= b;
        const float nq = __fmul_rn(nrm, (float)qi);  // qsgd_decode_flat's arithmetic
        tile[threadIdx.x * 33 + i] = POW2 ? __fmul_rn(nq, inv_levels) : nq / levels;
      }
    }
    __syncthreads();
    const int64_t lim = min((int64_t)G, it.end - base);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int e = 4 * (v * kThreads + (int)threadIdx.x);  // element of this pass
      if (e >= lim) continue;
      float f[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) f[c] = tile[((e + c) >> 5) * 33 + ((e + c) & 31)];
      float* yo = y + base + e;
      if (e + 4 <= lim) {
        float4 o = make_float4(f[0], f[1], f[2], f[3]);
        if (ACC) {
          const float4 prev = *reinterpret_cast<const float4*>(yo);
          o.x = __fadd_rn(prev.x, o.x); o.y = __fadd_rn(prev.y, o.y);
          o.z = __fadd_rn(prev.z, o.z); o.w = __fadd_rn(prev.w, o.w);
        }
        store_nt(yo, o);
      } else {
        for (int c = 0; c < 4 && e + c < lim; ++c) yo[c] = ACC ? __fadd_rn(yo[c], f[c]) : f[c];
      }
    }
    __syncthreads();  // the tile is rewritten by the next pass
  }
}

template <int WIDTH, int B>
void launch_pack(dim3 g, hipStream_t st, const void* q, const Item* items, int32_t L, int32_t b, uint32_t* out) {
  hipLaunchKernelGGL((qsgd_pack<WIDTH, B>), g, dim3(kThreads), 0, st, q, items, L, b, out);
}

template <int WIDTH>
void dispatch_pack(int b, dim3 g, hipStream_t st, const void* q, const Item* items, int32_t L, uint32_t* out) {
  switch (b) {
    case 2: launch_pack<WIDTH, 2>(g, st, q, items, L, b, out); break;
    case 3: launch_pack<WIDTH, 3>(g, st, q, items, L, b, out); break;
    case 4: launch_pack<WIDTH, 4>(g, st, q, items, L, b, out); break;
    case 5: launch_pack<WIDTH, 5>(g, st, q, items, L, b, out); break;
    case 6: launch_pack<WIDTH, 6>(g, st, q, items, L, b, out); break;
    case 7: launch_pack<WIDTH, 7>(g, st, q, items, L, b, out); break;
    case 8: launch_pack<WIDTH, 8>(g, st, q, items, L, b, out); break;
    case 9: launch_pack<WIDTH, 9>(g, st, q, items, L, b, out); break;
    case 10: launch_pack<WIDTH, 10>(g, st, q, items, L, b, out); break;
    default: launch_pack<WIDTH, 0>(g, st, q, items, L, b, out); break;
  }
}

template <bool ACC, bool POW2>
void dispatch_decode(int b, dim3 g, hipStream_t st, const uint32_t* packed, const Item* items, const float* norm,
                     float* y, int32_t L, float levels, float inv) {
#define OMF_DP(BB) \
  hipLaunchKernelGGL((qsgd_decode_packed<BB, ACC, POW2>), g, dim3(kThreads), 0, st, packed, items, norm, y, L, b, levels, inv)
  switch (b) {
    case 2: OMF_DP(2); break;
    case 3: OMF_DP(3); break;
    case 4: OMF_DP(4); break;
    case 5: OMF_DP(5); break;
    case 6: OMF_DP(6); break;
    case 7: OMF_DP(7); break;
    case 8: OMF_DP(8); break;
    case 9: OMF_DP(9); break;
    case 10: OMF_DP(10); break;
    default: OMF_DP(0); break;
  }
#undef OMF_DP
}

}  // namespace

namespace omf_plan_access {
const void* flat_items(const omf_plan* p, int64_t* n);
int device(const omf_plan* p);
}  // namespace omf_plan_access

extern "C" {

int32_t omf_qsgd_packed_bits(int32_t levels) {
  if (levels <= 0) return -1;
  const uint64_t codes = 2ull * (uint64_t)levels + 1ull;
  int32_t b = 0;
  while ((1ull << b) < codes) ++b;
  return b;
}

int omf_qsgd_pack(omf_plan* plan, const void* q, int32_t width, int32_t levels, uint32_t* packed, void* stream) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  if (width != 8 && width != 32) return fail(OMF_EINVAL, "width must be 8 or 32");
  const int32_t b = omf_qsgd_packed_bits(levels);
  if (b < 0 || b > 32) return fail(OMF_EINVAL, "levels must be in [1, 2^31 - 1)");
  if (width == 8 && levels > 127) return fail(OMF_EINVAL, "an int8 payload holds levels <= 127");
  if (!q || !packed) return fail(OMF_EINVAL, "q and packed must be non-NULL");
  if (((uintptr_t)q & 15) || ((uintptr_t)packed & 3)) return fail(OMF_EINVAL, "q must be 16-byte, packed 4-byte aligned");
  DeviceGuard g(omf_plan_access::device(plan));
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  int64_t n_items = 0;
  const Item* items = static_cast<const Item*>(omf_plan_access::flat_items(plan, &n_items));
  if (n_items == 0) return OMF_OK;
  const dim3 grid((unsigned)n_items);
  hipStream_t st = (hipStream_t)stream;
  if (width == 8) dispatch_pack<1>(b, grid, st, q, items, levels, packed);
  else dispatch_pack<4>(b, grid, st, q, items, levels, packed);
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

int omf_qsgd_decode_packed(omf_plan* plan, const uint32_t* packed, int32_t levels, const float* norm, float* y,
                           int32_t accumulate, void* stream) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  const int32_t b = omf_qsgd_packed_bits(levels);
  if (b < 0 || b > 32) return fail(OMF_EINVAL, "levels must be in [1, 2^31 - 1)");
  if (!packed || !norm || !y) return fail(OMF_EINVAL, "packed, norm and y must be non-NULL");
  if (((uintptr_t)y & 15) || ((uintptr_t)packed & 3)) return fail(OMF_EINVAL, "y must be 16-byte, packed 4-byte aligned");
  DeviceGuard g(omf_plan_access::device(plan));
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  int64_t n_items = 0;
  const Item* items = static_cast<const Item*>(omf_plan_access::flat_items(plan, &n_items));
  if (n_items == 0) return OMF_OK;
  const dim3 grid((unsigned)n_items);
  hipStream_t st = (hipStream_t)stream;
  const bool pow2 = (levels & (levels - 1)) == 0;
  const float lv = (float)levels, inv = pow2 ? 1.0f / (float)levels : 0.0f;
  if (accumulate) {
    if (pow2) dispatch_decode<true, true>(b, grid, st, packed, items, norm, y, levels, lv, inv);
    else dispatch_decode<true, false>(b, grid, st, packed, items, norm, y, levels, lv, inv);
  } else {
    if (pow2) dispatch_decode<false, true>(b, grid, st, packed, items, norm, y, levels, lv, inv);
    else dispatch_decode<false, false>(b, grid, st, packed, items, norm, y, levels, lv, inv);
  }
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

}  // extern "C"
