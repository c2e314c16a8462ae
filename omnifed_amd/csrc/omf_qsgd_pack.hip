// omf_qsgd_pack.hip — opt-in bit-packed QSGD wire format, MI355X (gfx950).
//
// NOT reference-compatible: a new compression_type ("QSGDBitPackedCompression") that a
// sender uses only when asked to.  The levels q in [-L, L] of the reference wire (int8 or
// int32 per element, global_grpc_compression.py:111-123) become the codes q + L in
// b = ceil(log2(2L + 1)) bits (s = 4: 6 bits instead of 8; s = 8: 10 instead of 32),
// LSB-first little-endian: element i of a tensor occupies bits [i*b, (i+1)*b) of the
// tensor's stream.  In a plan's packed arena, tensor t's stream starts at 32-bit word
// offset_t * b / 32 (the offsets must be multiples of 32 elements, else OMF_EINVAL;
// arena_layout's are multiples of 64), so 32 consecutive elements are exactly b words, lie in
// one tensor, and one thread packs or unpacks them alone.
// Decoding the codes gives the same floats as decoding the levels (qsgd_decode_flat's
// arithmetic: fl32(fl32(norm * q) / L)).
#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/omf_codec.h"
#include "omf_common.h"

using namespace omf;

namespace {

constexpr int64_t kTableBlk = 4096;  // elements per decoder-table block (omf_qsgd.hip kDecBlk)
constexpr int kGroupBlk = 32 * kThreads;  // elements per workgroup of the pack and the decode
static_assert(kGroupBlk == 2 * kTableBlk, "two table blocks per workgroup");

// A thread's 32-element group: the whole workgroup inside one tensor (both table blocks marked
// inside the same tensor), or the group's own tensor found from the block's first one (offsets
// are multiples of 32: a group never spans two tensors).  Returns the elements of the group in
// its tensor (0 = padding, or past the arena) and that tensor.
__device__ __forceinline__ int group_tensor(const uint32_t* __restrict__ binfo, int64_t nbinfo,
                                            const int64_t* __restrict__ begins, const int64_t* __restrict__ sizes,
                                            int32_t nt, int64_t e0, bool* whole, int32_t* tensor) {
  const int64_t k0 = 2 * (int64_t)blockIdx.x;
  const uint32_t i0 = binfo[k0];
  const uint32_t i1 = k0 + 1 < nbinfo ? binfo[k0 + 1] : 0u;
  int32_t t = (int32_t)(i0 & 0x7fffffffu);  // the last tensor starting at or before the block
  *whole = (i0 >> 31) && i1 == i0;
  if (*whole) {
    *tensor = t;
    return 32;
  }
  while (t + 1 < nt && e0 >= begins[t + 1]) ++t;
  *tensor = t;
  const int64_t lim = min((int64_t)32, begins[t] + sizes[t] - e0);
  return lim > 0 ? (int)lim : 0;
}

// Pack over the arena, one workgroup per 8 Ki-element block: each thread packs its 32-element
// group into b words.  The payload loads are issued before the block's table entry arrives,
// clamped to the last whole group of the arena (a thread whose group is whole in its tensor
// reads exactly its own elements); a group a tensor ends inside reloads its elements one by
// one and packs code 0 after them; padding groups are not written.
// B: compile-time code width (2..10, s = 0..8), or 0 = the runtime width b.
template <int WIDTH, int B>
__global__ __launch_bounds__(kThreads) void qsgd_pack(const void* __restrict__ q, const uint32_t* __restrict__ binfo,
                                                      int64_t nbinfo, const int64_t* __restrict__ begins,
                                                      const int64_t* __restrict__ sizes, int32_t nt, int64_t arena_end,
                                                      int32_t L, int32_t b_rt, uint32_t* __restrict__ out) {
  const int b = B ? B : b_rt;
  const int64_t e0 = (int64_t)blockIdx.x * kGroupBlk + 32 * (int64_t)threadIdx.x;
  const int64_t qmax = ((arena_end >> 5) - 1) << 5;  // the last whole group (< 0: none)
  const int64_t ec = max((int64_t)0, min(e0, qmax));
  int32_t lv[32];
  if (qmax >= 0) {  // uniform
    if (WIDTH == 1) {
      const int8_t* q8 = static_cast<const int8_t*>(q) + ec;
      const i32x4_t w0 = *reinterpret_cast<const i32x4_t*>(q8);
      const i32x4_t w1 = *reinterpret_cast<const i32x4_t*>(q8 + 16);
      const uint32_t w[8] = {(uint32_t)w0[0], (uint32_t)w0[1], (uint32_t)w0[2], (uint32_t)w0[3],
                             (uint32_t)w1[0], (uint32_t)w1[1], (uint32_t)w1[2], (uint32_t)w1[3]};
#pragma unroll
      for (int i = 0; i < 32; ++i) lv[i] = (int32_t)(int8_t)(w[i >> 2] >> (8 * (i & 3)));
    } else {
      const int32_t* q32 = static_cast<const int32_t*>(q) + ec;
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const i32x4_t w = *reinterpret_cast<const i32x4_t*>(q32 + 4 * v);
        lv[4 * v] = w[0]; lv[4 * v + 1] = w[1]; lv[4 * v + 2] = w[2]; lv[4 * v + 3] = w[3];
      }
    }
  }
  bool whole;
  int32_t t;
  const int nv = group_tensor(binfo, nbinfo, begins, sizes, nt, e0, &whole, &t);
  if (nv == 0) return;
  if (nv < 32) {  // the tensor ends inside this group (its elements only; codes 0 after them)
#pragma unroll
    for (int i = 0; i < 32; ++i)
      lv[i] = i < nv ? (WIDTH == 1 ? (int32_t)(static_cast<const int8_t*>(q)[e0 + i])
                                   : static_cast<const int32_t*>(q)[e0 + i])
                     : -L;
  }
  uint32_t* o = out + (e0 >> 5) * (int64_t)b;
  uint32_t wd[B ? B : 32];
  uint64_t acc = 0;
  int nb = 0, w = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    acc |= (uint64_t)(uint32_t)(lv[i] + L) << nb;
    nb += b;
    if (nb >= 32) {
      if (B) wd[w++] = (uint32_t)acc;  // static index once unrolled
      else o[w++] = (uint32_t)acc;     // runtime width: straight to memory
      acc >>= 32;
      nb -= 32;
    }
  }
  if (B && B % 2 == 0) {  // b words at a multiple of 8 bytes: 8-byte stores
#pragma unroll
    for (int i = 0; i < (B ? B : 2); i += 2)
      *reinterpret_cast<uint2*>(o + i) = make_uint2(wd[i], wd[i + 1]);
  } else if (B) {
#pragma unroll
    for (int i = 0; i < (B ? B : 1); ++i) o[i] = wd[i];
  }
}

// Decode over the arena, one workgroup per 8 Ki-element block (two blocks of the plan's 4 Ki
// decoder table, omf_qsgd.hip qsgd_decode_arena): every lane's b packed words go out first, their
// addresses depending on blockIdx only, with the block's tensor and norm as scalar loads in
// flight (the item-indexed version waited for its item and norm, then walked its item pass by
// pass: 0.38 ms on Llama-400M).  Each thread unpacks its 32 elements into LDS; the workgroup
// transposes them (33-word rows: conflict-free both ways) so the fp32 stores are lane-contiguous
// 16-byte non-temporal stores.  A block not inside one tensor finds each 32-element group's
// tensor (packed_arena requires offsets that are multiples of 32: a group never spans two) and
// writes only its elements;
// padding keeps what y held.
template <int B, bool ACC, bool POW2>
__global__ __launch_bounds__(kThreads) void qsgd_decode_packed(const uint32_t* __restrict__ packed,
                                                               const uint32_t* __restrict__ binfo, int64_t nbinfo,
                                                               const float* __restrict__ norm,
                                                               const int64_t* __restrict__ begins,
                                                               const int64_t* __restrict__ sizes, int32_t nt,
                                                               int64_t arena_end, float* __restrict__ y, int32_t L,
                                                               int32_t b_rt, float levels, float inv_levels) {
  constexpr int G = kGroupBlk;
  __shared__ float tile[kThreads * 33];
  __shared__ int32_t s_lim[kThreads];
  const int b = B ? B : b_rt;
  const int64_t base = (int64_t)blockIdx.x * G;
  const int64_t e0 = base + 32 * (int64_t)threadIdx.x;
  // unconditional loads, clamped to the packed arena's last group
  const uint32_t* p = packed + min(e0 >> 5, (arena_end - 1) >> 5) * (int64_t)b;
  uint32_t wd[B ? B : 32];
  if (B) {
#pragma unroll
    for (int i = 0; i < (B ? B : 1); ++i) wd[i] = __builtin_nontemporal_load(p + i);
  } else {
    for (int i = 0; i < b; ++i) wd[i] = p[i];
  }
  bool whole;
  int32_t t;
  const int lim = group_tensor(binfo, nbinfo, begins, sizes, nt, e0, &whole, &t);
  if (!whole) s_lim[threadIdx.x] = lim;
  const float nrm = lim > 0 ? norm[t] : 0.0f;
  const uint64_t mask = (1ull << b) - 1ull;
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
    const float nq = __fmul_rn(nrm, (float)qi);  // qsgd_decode_arena's arithmetic
    tile[threadIdx.x * 33 + i] = POW2 ? __fmul_rn(nq, inv_levels) : nq / levels;
  }
  __syncthreads();
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    const int e = 4 * (v * kThreads + (int)threadIdx.x);  // element of this block
    float f[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) f[c] = tile[((e + c) >> 5) * 33 + ((e + c) & 31)];
    float* yo = y + base + e;
    const int l = whole ? 4 : s_lim[e >> 5] - (e & 31);  // elements of the quad to write
    if (l >= 4) {
      float4 o = make_float4(f[0], f[1], f[2], f[3]);
      if (ACC) {
        const f32x4_t pv = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(yo));
        o.x = __fadd_rn(pv[0], o.x); o.y = __fadd_rn(pv[1], o.y);
        o.z = __fadd_rn(pv[2], o.z); o.w = __fadd_rn(pv[3], o.w);
      }
      store_nt(yo, o);
    } else {
      for (int c = 0; c < l; ++c) yo[c] = ACC ? __fadd_rn(yo[c], f[c]) : f[c];
    }
  }
}

// The plan's arena as the pack and the decode walk it.
struct ArenaArgs {
  const uint32_t* binfo;
  int64_t nbinfo;
  const int64_t* begins;
  const int64_t* sizes;
  int32_t nt;
  int64_t arena_end;
};

template <int WIDTH, int B>
void launch_pack(dim3 g, hipStream_t st, const void* q, const ArenaArgs& a, int32_t L, int32_t b, uint32_t* out) {
  hipLaunchKernelGGL((qsgd_pack<WIDTH, B>), g, dim3(kThreads), 0, st, q, a.binfo, a.nbinfo, a.begins, a.sizes, a.nt,
                     a.arena_end, L, b, out);
}

template <int WIDTH>
void dispatch_pack(int b, dim3 g, hipStream_t st, const void* q, const ArenaArgs& a, int32_t L, uint32_t* out) {
  switch (b) {
    case 2: launch_pack<WIDTH, 2>(g, st, q, a, L, b, out); break;
    case 3: launch_pack<WIDTH, 3>(g, st, q, a, L, b, out); break;
    case 4: launch_pack<WIDTH, 4>(g, st, q, a, L, b, out); break;
    case 5: launch_pack<WIDTH, 5>(g, st, q, a, L, b, out); break;
    case 6: launch_pack<WIDTH, 6>(g, st, q, a, L, b, out); break;
    case 7: launch_pack<WIDTH, 7>(g, st, q, a, L, b, out); break;
    case 8: launch_pack<WIDTH, 8>(g, st, q, a, L, b, out); break;
    case 9: launch_pack<WIDTH, 9>(g, st, q, a, L, b, out); break;
    case 10: launch_pack<WIDTH, 10>(g, st, q, a, L, b, out); break;
    default: launch_pack<WIDTH, 0>(g, st, q, a, L, b, out); break;
  }
}

template <bool ACC, bool POW2>
void dispatch_decode(int b, dim3 g, hipStream_t st, const uint32_t* packed, const ArenaArgs& a, const float* norm,
                     float* y, int32_t L, float levels, float inv) {
#define OMF_DP(BB)                                                                                               \
  hipLaunchKernelGGL((qsgd_decode_packed<BB, ACC, POW2>), g, dim3(kThreads), 0, st, packed, a.binfo, a.nbinfo, norm, \
                     a.begins, a.sizes, a.nt, a.arena_end, y, L, b, levels, inv)
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
int device(const omf_plan* p);
int32_t ntensors(const omf_plan* p);
int64_t arena_end(const omf_plan* p);
const int64_t* d_sizes(const omf_plan* p);
const int64_t* d_begins(const omf_plan* p);
const std::vector<int64_t>& offsets(const omf_plan* p);
const uint32_t* dec_blocks(const omf_plan* p, int64_t* n, int64_t* block_elems);
}  // namespace omf_plan_access

namespace {

// The plan's arena for the packed wire, or an error: every tensor offset a multiple of 32
// elements (a tensor's stream then starts on a word, and a 32-element group lies in one tensor).
int packed_arena(const omf_plan* plan, ArenaArgs* a, dim3* grid) {
  for (const int64_t o : omf_plan_access::offsets(plan))
    if (o & 31) return fail(OMF_EINVAL, "the packed wire needs tensor offsets that are multiples of 32 elements");
  int64_t tblk = 0;
  a->binfo = omf_plan_access::dec_blocks(plan, &a->nbinfo, &tblk);
  if (tblk != kTableBlk) return fail(OMF_EINVAL, "packed wire: decoder table block size mismatch (library build)");
  a->begins = omf_plan_access::d_begins(plan);
  a->sizes = omf_plan_access::d_sizes(plan);
  a->nt = omf_plan_access::ntensors(plan);
  a->arena_end = omf_plan_access::arena_end(plan);
  *grid = dim3((unsigned)((a->arena_end + kGroupBlk - 1) / kGroupBlk));
  return OMF_OK;
}

}  // namespace

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
  // even widths store 8-byte word pairs: the packed arena must be 8-byte aligned
  if (((uintptr_t)q & 15) || ((uintptr_t)packed & 7)) return fail(OMF_EINVAL, "q must be 16-byte, packed 8-byte aligned");
  ArenaArgs a;
  dim3 grid;
  if (const int rc = packed_arena(plan, &a, &grid)) return rc;
  DeviceGuard g(omf_plan_access::device(plan));
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;
  if (width == 8) dispatch_pack<1>(b, grid, st, q, a, levels, packed);
  else dispatch_pack<4>(b, grid, st, q, a, levels, packed);
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
  ArenaArgs a;
  dim3 grid;
  if (const int rc = packed_arena(plan, &a, &grid)) return rc;
  DeviceGuard g(omf_plan_access::device(plan));
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;
  const bool pow2 = (levels & (levels - 1)) == 0;
  const float lv = (float)levels, inv = pow2 ? 1.0f / (float)levels : 0.0f;
#define OMF_DD(A, P) dispatch_decode<A, P>(b, grid, st, packed, a, norm, y, levels, lv, inv)
  if (accumulate) {
    if (pow2) OMF_DD(true, true); else OMF_DD(true, false);
  } else {
    if (pow2) OMF_DD(false, true); else OMF_DD(false, false);
  }
#undef OMF_DD
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

}  // extern "C"
