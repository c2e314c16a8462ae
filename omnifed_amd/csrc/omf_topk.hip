// omf_topk.hip — Top-K sparsification with error feedback, MI355X (gfx950).
//
// Semantics: src/omnifed/hybrid/compression/topk.py:10-47 + core.py:19-37 (reference):
//   t' = residual + x ; k = max(1, int(n * ratio)) ; the k largest |t'| ;
//   residual := t' - desparse(values, indices)  (= t' with the selected slots set to t'-t').
//
// Passes (all tensors of a plan per launch):
//   1. topk_prep_hist   read x (+residual), write t' into the residual buffer, and a
//                       1024-bin histogram of the top 10 bits of |t'| (exponent + 2
//                       mantissa bits) per tensor (LDS histogram, non-zero bins flushed).
//   2. topk_select_bin  per tensor: the bin b1 holding the k-th largest magnitude.
//   3. topk_collect     re-read t'; every element whose bin >= b1 is a candidate
//                       (about 1-2.5 % of a gradient at k = 1 %), appended with one
//                       wave-aggregated atomic per wave as a 64-bit key
//                       (|t'| bits << 32 | ~index): descending key order = descending
//                       magnitude, ties by ascending index.
//   4. segmented descending radix sort of the candidates (rocPRIM).
//   5. topk_gather      first k keys of every tensor -> values / int64 indices; zero
//                       the selected residual slots.
// Decode is a scatter (mode 0 zero-fill, 1 overlay, 2 scatter-add).
#include <cstring>

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <vector>

#include "../../include/omf_codec.h"
#include "omf_common.h"

using namespace omf;

namespace {

constexpr int kBins = 1024;
constexpr int kShift = 21;  // key (31 bits) >> 21 -> 10-bit bin
constexpr int kV = 16;
constexpr int64_t kSub = (int64_t)kV * kThreads * 4;

// Mirrors the QSGD plan's item / tensor tables (omf_qsgd.hip); only the fields used here.
struct Item {
  int64_t begin, end;
  int32_t tensor, kind, chunk, pad;
};


__device__ __forceinline__ uint32_t mag_key(float v) { return __float_as_uint(v) & 0x7fffffffu; }

template <int MODE>  // 0: t' = x ; 1: t' = r + x, r := t' ; 2: t' = x, r := t'
__global__ __launch_bounds__(kThreads) void topk_prep_hist(const float* __restrict__ x, float* __restrict__ r,
                                                           const Item* __restrict__ items, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kBins];
  for (int b = threadIdx.x; b < kBins; b += kThreads) h[b] = 0;
  __syncthreads();
  const Item it = items[blockIdx.x];
  for (int64_t b = it.begin; b < it.end; b += kSub) {
    const int64_t end = min(b + kSub, it.end);
#pragma unroll 4
    for (int k = 0; k < kV; ++k) {
      const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
      if (e >= end) continue;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      const bool full = e + 4 <= end;
      const int nv = full ? 4 : (int)(end - e);
      if (full) {
        float4 t = *reinterpret_cast<const float4*>(x + e);
        if (MODE == 1) {
          const float4 rr = *reinterpret_cast<const float4*>(r + e);
          t.x = __fadd_rn(rr.x, t.x); t.y = __fadd_rn(rr.y, t.y);
          t.z = __fadd_rn(rr.z, t.z); t.w = __fadd_rn(rr.w, t.w);
        }
        if (MODE != 0) *reinterpret_cast<float4*>(r + e) = t;
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
      } else {
        for (int c = 0; c < nv; ++c) {
          float t = x[e + c];
          if (MODE == 1) t = __fadd_rn(r[e + c], t);
          if (MODE != 0) r[e + c] = t;
          v[c] = t;
        }
      }
      for (int c = 0; c < nv; ++c) atomicAdd(&h[mag_key(v[c]) >> kShift], 1u);
    }
  }
  __syncthreads();
  uint32_t* ht = hist + (size_t)it.tensor * kBins;
  for (int b = threadIdx.x; b < kBins; b += kThreads)
    if (h[b]) atomicAdd(&ht[b], h[b]);
}

// One block per tensor: b1 = max bin with suffix count >= k.
__global__ __launch_bounds__(kThreads) void topk_select_bin(const uint32_t* __restrict__ hist,
                                                            const int64_t* __restrict__ kk, uint32_t* __restrict__ bin) {
  __shared__ uint32_t s_part[kThreads];
  const int t = blockIdx.x;
  const uint32_t* ht = hist + (size_t)t * kBins;
  // thread i owns bins [4i, 4i+4); suffix sums over threads from the top.
  uint32_t c[4], loc = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) { c[j] = ht[4 * threadIdx.x + j]; loc += c[j]; }
  s_part[threadIdx.x] = loc;
  __syncthreads();
  // inclusive suffix scan (Hillis-Steele) over s_part
  for (int o = 1; o < kThreads; o <<= 1) {
    const uint32_t add = (threadIdx.x + o < kThreads) ? s_part[threadIdx.x + o] : 0u;
    __syncthreads();
    s_part[threadIdx.x] += add;
    __syncthreads();
  }
  const uint64_t k = (uint64_t)kk[t];
  uint64_t above = (threadIdx.x + 1 < kThreads) ? s_part[threadIdx.x + 1] : 0u;  // count in bins > 4i+3
  for (int j = 3; j >= 0; --j) {
    if (above < k && above + c[j] >= k) bin[t] = 4 * threadIdx.x + j;  // exactly one (thread, j) matches
    above += c[j];
  }
}

__global__ void topk_offsets(const int64_t* __restrict__ tsize,
                             int32_t nt, double ratio, int64_t* __restrict__ kk, int64_t* __restrict__ koff,
                             const int64_t* __restrict__ tbegin, const uint32_t* __restrict__ cnt,
                             uint32_t* __restrict__ seg_b, uint32_t* __restrict__ seg_e, int phase) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (phase == 0) {
    int64_t acc = 0;
    for (int t = 0; t < nt; ++t) {
      int64_t k = (int64_t)((double)tsize[t] * ratio);
      if (k < 1) k = 1;
      kk[t] = k;
      koff[t] = acc;
      acc += k;
    }
    koff[nt] = acc;
  } else {
    for (int t = 0; t < nt; ++t) {
      seg_b[t] = (uint32_t)tbegin[t];
      seg_e[t] = (uint32_t)(tbegin[t] + cnt[t]);
    }
  }
}

__global__ __launch_bounds__(kThreads) void topk_collect(const float* __restrict__ tp, const Item* __restrict__ items,
                                                         const int64_t* __restrict__ tbegin,
                                                         const uint32_t* __restrict__ bin, uint32_t* __restrict__ cnt,
                                                         uint64_t* __restrict__ cand) {
  const Item it = items[blockIdx.x];
  const uint32_t b1 = bin[it.tensor];
  const int64_t base = tbegin[it.tensor];
  const int lane = threadIdx.x & 63;
  for (int64_t b = it.begin; b < it.end; b += kSub) {
    const int64_t end = min(b + kSub, it.end);
#pragma unroll 4
    for (int k = 0; k < kV; ++k) {
      const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      int nv = 0;
      if (e + 4 <= end) {
        const float4 t = *reinterpret_cast<const float4*>(tp + e);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        nv = 4;
      } else if (e < end) {
        nv = (int)(end - e);
        for (int c = 0; c < nv; ++c) v[c] = tp[e + c];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t key = mag_key(v[c]);
        const bool sel = (c < nv) && ((key >> kShift) >= b1);
        const uint64_t m = __ballot(sel);
        if (m == 0) continue;  // wave-uniform
        const int leader = __ffsll((long long)m) - 1;
        uint32_t pos0 = 0;
        if (lane == leader) pos0 = atomicAdd(&cnt[it.tensor], (uint32_t)__popcll(m));
        pos0 = __shfl(pos0, leader, 64);
        if (sel) {
          const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
          const uint32_t idx = (uint32_t)(e + c - base);
          cand[base + pos0 + rank] = ((uint64_t)key << 32) | (uint64_t)(~idx);
        }
      }
    }
  }
}

__global__ __launch_bounds__(kThreads) void topk_gather(const float* __restrict__ tp, float* __restrict__ r,
                                                        const uint64_t* __restrict__ sorted,
                                                        const int64_t* __restrict__ tbegin,
                                                        const int64_t* __restrict__ kk, const int64_t* __restrict__ koff,
                                                        float* __restrict__ values, int64_t* __restrict__ indices) {
  const int t = blockIdx.y;
  const int64_t k = kk[t], base = tbegin[t], o = koff[t];
  for (int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x; j < k; j += (int64_t)gridDim.x * kThreads) {
    const uint32_t idx = ~(uint32_t)sorted[base + j];
    const float v = tp[base + idx];
    values[o + j] = v;
    indices[o + j] = (int64_t)idx;
    if (r) r[base + idx] = __fsub_rn(v, v);
  }
}

__global__ __launch_bounds__(kThreads) void topk_scatter(const float* __restrict__ values,
                                                         const int64_t* __restrict__ indices, int64_t k,
                                                         float* __restrict__ y, int64_t n, int add) {
  for (int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x; j < k; j += (int64_t)gridDim.x * kThreads) {
    const int64_t i = indices[j];
    if (i < 0 || i >= n) continue;
    y[i] = add ? __fadd_rn(y[i], values[j]) : values[j];
  }
}

}  // namespace

// ---------------------------------------------------------------- host side
// Plan internals (defined in omf_qsgd.hip): accessed through these helpers.
namespace omf_plan_access {
const void* flat_items(const omf_plan* p, int64_t* n);
int32_t ntensors(const omf_plan* p);
int device(const omf_plan* p);
int64_t arena_end(const omf_plan* p);
const int64_t* d_sizes(const omf_plan* p);
const int64_t* d_begins(const omf_plan* p);
const std::vector<int64_t>& sizes(const omf_plan* p);
}  // namespace omf_plan_access

namespace {

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t sort_tmp_bytes(int64_t size, int32_t nt) {
  size_t bytes = 0;
  uint64_t* dummy = nullptr;
  uint32_t* off = nullptr;
  (void)rocprim::segmented_radix_sort_keys_desc(nullptr, bytes, dummy, dummy, (unsigned int)size, (unsigned int)nt, off,
                                                off, 0, 64, (hipStream_t)0, false);
  return bytes;
}

struct WsLayout {
  size_t hist, bin, cnt, koff, kk, seg_b, seg_e, cand, sorted, tmp, total, tmp_bytes;
};

WsLayout layout(const omf_plan* p) {
  const int32_t nt = omf_plan_access::ntensors(p);
  const int64_t ae = omf_plan_access::arena_end(p);
  WsLayout L;
  size_t o = 0;
  L.hist = o; o = align256(o + 4 * (size_t)nt * kBins);
  L.bin = o; o = align256(o + 4 * (size_t)nt);
  L.cnt = o; o = align256(o + 4 * (size_t)nt);
  L.koff = o; o = align256(o + 8 * (size_t)(nt + 1));
  L.kk = o; o = align256(o + 8 * (size_t)nt);
  L.seg_b = o; o = align256(o + 4 * (size_t)nt);
  L.seg_e = o; o = align256(o + 4 * (size_t)nt);
  L.cand = o; o = align256(o + 8 * (size_t)ae);
  L.sorted = o; o = align256(o + 8 * (size_t)ae);
  L.tmp_bytes = sort_tmp_bytes(ae, nt);
  L.tmp = o; o = align256(o + L.tmp_bytes);
  L.total = o;
  return L;
}

}  // namespace

extern "C" {

int64_t omf_topk_k(int64_t numel, double ratio) {
  int64_t k = (int64_t)((double)numel * ratio);
  return k < 1 ? 1 : k;
}

size_t omf_topk_workspace_bytes(const omf_plan* plan, double ratio) {
  (void)ratio;
  if (!plan) return 0;
  return layout(plan).total;
}

int omf_topk_encode(omf_plan* plan, const float* x, float* residual, int32_t residual_mode, double ratio,
                    float* values, int64_t* indices, void* ws, size_t ws_bytes, void* stream) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  if (!x || !values || !indices || !ws) return fail(OMF_EINVAL, "x, values, indices and ws must be non-NULL");
  if (residual_mode < 0 || residual_mode > 2 || (residual_mode != 0 && !residual))
    return fail(OMF_EINVAL, "residual_mode must be 0 (none), 1 (compensate+update) or 2 (init) with a residual buffer");
  if (!(ratio == ratio)) return fail(OMF_EINVAL, "ratio is NaN");
  const std::vector<int64_t>& sizes = omf_plan_access::sizes(plan);
  int64_t kmax = 0;
  for (int64_t n : sizes) {
    const int64_t k = omf_topk_k(n, ratio);
    if (k > n) return fail(OMF_EINVAL, "selected index k out of range (k > numel): compress_ratio too large");
    if (n > 0x7fffffffLL) return fail(OMF_EINVAL, "tensor too large for 32-bit candidate indices");
    kmax = std::max(kmax, k);
  }
  if (omf_plan_access::arena_end(plan) > 0xffffffffLL) return fail(OMF_EINVAL, "arena too large for the sort");
  if (((uintptr_t)x & 15) || (residual && ((uintptr_t)residual & 15)))
    return fail(OMF_EINVAL, "x and residual must be 16-byte aligned");
  const WsLayout L = layout(plan);
  if (ws_bytes < L.total) return fail(OMF_EINVAL, "workspace too small (see omf_topk_workspace_bytes)");
  DeviceGuard g(omf_plan_access::device(plan));
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint32_t* hist = reinterpret_cast<uint32_t*>(w + L.hist);
  uint32_t* bin = reinterpret_cast<uint32_t*>(w + L.bin);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(w + L.cnt);
  int64_t* koff = reinterpret_cast<int64_t*>(w + L.koff);
  int64_t* kk = reinterpret_cast<int64_t*>(w + L.kk);
  uint32_t* seg_b = reinterpret_cast<uint32_t*>(w + L.seg_b);
  uint32_t* seg_e = reinterpret_cast<uint32_t*>(w + L.seg_e);
  uint64_t* cand = reinterpret_cast<uint64_t*>(w + L.cand);
  uint64_t* sorted = reinterpret_cast<uint64_t*>(w + L.sorted);
  const int32_t nt = omf_plan_access::ntensors(plan);
  int64_t n_items = 0;
  const Item* items = static_cast<const Item*>(omf_plan_access::flat_items(plan, &n_items));
  const int64_t* d_sizes = omf_plan_access::d_sizes(plan);
  const int64_t* d_begins = omf_plan_access::d_begins(plan);

  // hist + cnt are contiguous from the workspace start up to L.bin/L.koff: zero them.
  OMF_HIP(hipMemsetAsync(w, 0, L.koff, st));
  hipLaunchKernelGGL(topk_offsets, dim3(1), dim3(64), 0, st, d_sizes, nt, ratio, kk, koff, d_begins, cnt,
                     seg_b, seg_e, 0);
  const float* tp = (residual_mode == 0) ? x : residual;
  const dim3 grid((unsigned)n_items), blk(kThreads);
  if (residual_mode == 0) hipLaunchKernelGGL((topk_prep_hist<0>), grid, blk, 0, st, x, residual, items, hist);
  else if (residual_mode == 1) hipLaunchKernelGGL((topk_prep_hist<1>), grid, blk, 0, st, x, residual, items, hist);
  else hipLaunchKernelGGL((topk_prep_hist<2>), grid, blk, 0, st, x, residual, items, hist);
  hipLaunchKernelGGL(topk_select_bin, dim3((unsigned)nt), blk, 0, st, hist, kk, bin);
  hipLaunchKernelGGL(topk_collect, grid, blk, 0, st, tp, items, d_begins, bin, cnt, cand);
  hipLaunchKernelGGL(topk_offsets, dim3(1), dim3(64), 0, st, d_sizes, nt, ratio, kk, koff, d_begins, cnt,
                     seg_b, seg_e, 1);
  OMF_HIP(hipGetLastError());
  size_t tmp_bytes = L.tmp_bytes;
  OMF_HIP(rocprim::segmented_radix_sort_keys_desc(w + L.tmp, tmp_bytes, cand, sorted,
                                                  (unsigned int)omf_plan_access::arena_end(plan), (unsigned int)nt,
                                                  seg_b, seg_e, 0, 64, st, false));
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((kmax + kThreads - 1) / kThreads, 1024));
  hipLaunchKernelGGL(topk_gather, dim3(gx, (unsigned)nt), blk, 0, st, tp, residual_mode ? residual : nullptr, sorted,
                     d_begins, kk, koff, values, indices);
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

int omf_topk_decode(const float* values, const int64_t* indices, int64_t k, float* y, int64_t n, int32_t mode,
                    void* stream) {
  if (k < 0 || n < 0 || mode < 0 || mode > 2) return fail(OMF_EINVAL, "omf_topk_decode: bad arguments");
  if (n > 0 && !y) return fail(OMF_EINVAL, "omf_topk_decode: y is NULL");
  if (k > 0 && (!values || !indices)) return fail(OMF_EINVAL, "omf_topk_decode: values/indices NULL");
  hipStream_t st = (hipStream_t)stream;
  if (mode == 0 && n > 0) OMF_HIP(hipMemsetAsync(y, 0, (size_t)n * 4, st));
  if (k == 0) return OMF_OK;
  const unsigned g = (unsigned)std::min<int64_t>((k + kThreads - 1) / kThreads, 4096);
  hipLaunchKernelGGL(topk_scatter, dim3(g), dim3(kThreads), 0, st, values, indices, k, y, n, mode == 2 ? 1 : 0);
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

}  // extern "C"
