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
//   4. one device-wide radix sort of all candidates (rocPRIM onesweep) on the composite
//                       key (tensor << 56 | (2^31-1 - |t'|bits) << 25 | index), i.e.
//                       tensor ascending, magnitude descending, index ascending; when a
//                       plan exceeds 256 tensors or 2^25 elements per tensor, a segmented
//                       descending sort of (|t'|bits << 32 | ~index) per tensor instead.
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

// Candidates of one item: every |t'| whose bin is >= b1.  Counts are aggregated per
// sub-chunk (block scan in LDS) so each sub-chunk costs ONE global atomic on its tensor's
// counter; keys go to the tensor's own region cand[tbegin + pos] (capacity n_t).
template <bool GLOBAL>
__global__ __launch_bounds__(kThreads) void topk_collect(const float* __restrict__ tp, const Item* __restrict__ items,
                                                         const int64_t* __restrict__ tbegin,
                                                         const uint32_t* __restrict__ bin, uint32_t* __restrict__ cnt,
                                                         uint32_t* __restrict__ item_cnt, uint64_t* __restrict__ cand) {
  __shared__ uint32_t s_wsum[kWaves];
  __shared__ uint32_t s_base;
  const Item it = items[blockIdx.x];
  const uint32_t b1 = bin[it.tensor];
  const int64_t base = tbegin[it.tensor];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int CV = 8;                           // rows per pass (register budget)
  constexpr int64_t CS = (int64_t)CV * kThreads * 4;  // 8192 elements
  uint32_t item_total = 0;                         // GLOBAL: running offset in the item's region
  for (int64_t b = it.begin; b < it.end; b += CS) {
    const int64_t end = min(b + CS, it.end);
    const uint32_t lim = (uint32_t)(end - b);  // elements of this pass
    const uint32_t off0 = 4u * threadIdx.x;    // this lane's first element
    float4 v[CV];
    uint32_t selm = 0;  // bit 4k+c: element (row k, component c) is a candidate
#pragma unroll
    for (int k = 0; k < CV; ++k) {
      const uint32_t o = off0 + 1024u * k;
      if (o + 4 <= lim) {
        v[k] = *reinterpret_cast<const float4*>(tp + b + o);
      } else {
        v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (o < lim) v[k].x = tp[b + o];
        if (o + 1 < lim) v[k].y = tp[b + o + 1];
        if (o + 2 < lim) v[k].z = tp[b + o + 2];
      }
      const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (o + c < lim && (mag_key(vv[c]) >> kShift) >= b1) selm |= 1u << (4 * k + c);
    }
    const uint32_t nsel = (uint32_t)__popc(selm);
    // wave totals -> block scan in LDS
    uint32_t wtot = nsel;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wtot += __shfl_xor(wtot, o, 64);
    if (lane == 0) s_wsum[wave] = wtot;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
#pragma unroll
    for (int w2 = 0; w2 < kWaves; ++w2) {
      if (w2 < wave) wpre += s_wsum[w2];
      tot += s_wsum[w2];
    }
    // GLOBAL: the item's candidates go to its own element range (capacity = item size),
    // counted per item and packed after an exclusive scan — no contended atomics.
    if (!GLOBAL && threadIdx.x == 0) s_base = tot ? atomicAdd(&cnt[it.tensor], tot) : 0u;
    __syncthreads();
    // coalesced writes: per (row, component) the selected lanes of a wave store consecutively
    uint64_t* dst = GLOBAL ? cand + it.begin + item_total + wpre : cand + base + s_base + wpre;
    const uint32_t idx0 = (uint32_t)(b - base) + off0;
    const uint64_t tag = (uint64_t)it.tensor << 56;
    const uint64_t lt = (1ull << lane) - 1ull;
    if (wtot) {
#pragma unroll
      for (int k = 0; k < CV; ++k) {
        const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const bool sel = (selm >> (4 * k + c)) & 1u;
          const uint64_t m = __ballot(sel);
          if (sel) {
            const uint32_t idx = idx0 + 1024u * k + c;
            const uint32_t key = mag_key(vv[c]);
            dst[__popcll(m & lt)] = GLOBAL ? (tag | ((uint64_t)(0x7fffffffu - key) << 25) | (uint64_t)idx)
                                           : (((uint64_t)key << 32) | (uint64_t)(~idx));
          }
          dst += __popcll(m);
        }
      }
    }
    item_total += tot;
    __syncthreads();  // s_wsum / s_base reuse
  }
  if (GLOBAL && threadIdx.x == 0) item_cnt[blockIdx.x] = item_total;
}

// Pack every item's candidates (stored at the item's element range) at its scanned offset.
__global__ __launch_bounds__(kThreads) void topk_compact(const uint64_t* __restrict__ cand,
                                                         const Item* __restrict__ items,
                                                         const uint32_t* __restrict__ item_cnt,
                                                         const uint32_t* __restrict__ item_off,
                                                         uint64_t* __restrict__ packed) {
  const Item it = items[blockIdx.x];
  const uint32_t n = item_cnt[blockIdx.x], dst = item_off[blockIdx.x];
  for (uint32_t j = threadIdx.x; j < n; j += kThreads) packed[dst + j] = cand[it.begin + j];
}

// Per-tensor start and count of the packed candidates, from the item scan.
__global__ void topk_tensor_ranges(const Item* __restrict__ items, int64_t n_items,
                                   const uint32_t* __restrict__ item_cnt, const uint32_t* __restrict__ item_off,
                                   int64_t* __restrict__ cstart, uint32_t* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += (int64_t)gridDim.x * blockDim.x) {
    const Item it = items[i];
    if (it.chunk == 0) cstart[it.tensor] = item_off[i];
    atomicAdd(&cnt[it.tensor], item_cnt[i]);
  }
}

template <bool GLOBAL>
__global__ __launch_bounds__(kThreads) void topk_gather(const float* __restrict__ tp, float* __restrict__ r,
                                                        const uint64_t* __restrict__ sorted,
                                                        const int64_t* __restrict__ tbegin,
                                                        const int64_t* __restrict__ cstart,
                                                        const int64_t* __restrict__ kk, const int64_t* __restrict__ koff,
                                                        float* __restrict__ values, int64_t* __restrict__ indices) {
  const int t = blockIdx.y;
  const int64_t k = kk[t], base = tbegin[t], o = koff[t];
  const int64_t s0 = GLOBAL ? cstart[t] : base;
  for (int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x; j < k; j += (int64_t)gridDim.x * kThreads) {
    const uint64_t key = sorted[s0 + j];
    const uint32_t idx = GLOBAL ? (uint32_t)(key & 0x1FFFFFFull) : ~(uint32_t)key;
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

bool global_path(const omf_plan* p) {
  if (omf_plan_access::ntensors(p) > 256) return false;
  for (int64_t n : omf_plan_access::sizes(p))
    if (n > (int64_t)1 << 25) return false;
  return true;
}

size_t sort_tmp_bytes(const omf_plan* p) {
  const int64_t size = omf_plan_access::arena_end(p);
  const int32_t nt = omf_plan_access::ntensors(p);
  size_t bytes = 0;
  uint64_t* dummy = nullptr;
  if (global_path(p)) {
    (void)rocprim::radix_sort_keys(nullptr, bytes, dummy, dummy, (size_t)size, 0, 64, (hipStream_t)0, false);
    int64_t n_items = 0;
    (void)omf_plan_access::flat_items(p, &n_items);
    size_t sb = 0;
    uint32_t* u = nullptr;
    (void)rocprim::exclusive_scan(nullptr, sb, u, u, 0u, (size_t)n_items, rocprim::plus<uint32_t>(), (hipStream_t)0,
                                  false);
    bytes = std::max(bytes, sb);
  } else {
    uint32_t* off = nullptr;
    (void)rocprim::segmented_radix_sort_keys_desc(nullptr, bytes, dummy, dummy, (unsigned int)size, (unsigned int)nt,
                                                  off, off, 0, 64, (hipStream_t)0, false);
  }
  return bytes;
}

struct WsLayout {
  size_t hist, bin, cnt, cnt_all, koff, kk, seg_b, seg_e, cstart, item_cnt, item_off, cand, sorted, tmp, total,
      tmp_bytes;
};

WsLayout layout(const omf_plan* p) {
  const int32_t nt = omf_plan_access::ntensors(p);
  const int64_t ae = omf_plan_access::arena_end(p);
  WsLayout L;
  size_t o = 0;
  L.hist = o; o = align256(o + 4 * (size_t)nt * kBins);
  L.bin = o; o = align256(o + 4 * (size_t)nt);
  L.cnt = o; o = align256(o + 4 * (size_t)nt);
  L.cnt_all = o; o = align256(o + 4);
  L.koff = o; o = align256(o + 8 * (size_t)(nt + 1));
  L.kk = o; o = align256(o + 8 * (size_t)nt);
  L.seg_b = o; o = align256(o + 4 * (size_t)nt);
  L.seg_e = o; o = align256(o + 4 * (size_t)nt);
  L.cstart = o; o = align256(o + 8 * (size_t)nt);
  int64_t n_items = 0;
  (void)omf_plan_access::flat_items(p, &n_items);
  L.item_cnt = o; o = align256(o + 4 * (size_t)n_items);
  L.item_off = o; o = align256(o + 4 * (size_t)n_items);
  L.cand = o; o = align256(o + 8 * (size_t)ae);
  L.sorted = o; o = align256(o + 8 * (size_t)ae);
  L.tmp_bytes = sort_tmp_bytes(p);
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
  int64_t* cstart = reinterpret_cast<int64_t*>(w + L.cstart);
  uint32_t* item_cnt = reinterpret_cast<uint32_t*>(w + L.item_cnt);
  uint32_t* item_off = reinterpret_cast<uint32_t*>(w + L.item_off);
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

  // hist, bin, cnt and cnt_all precede L.koff: zero them.
  OMF_HIP(hipMemsetAsync(w, 0, L.koff, st));
  hipLaunchKernelGGL(topk_offsets, dim3(1), dim3(64), 0, st, d_sizes, nt, ratio, kk, koff, d_begins, cnt,
                     seg_b, seg_e, 0);
  const float* tp = (residual_mode == 0) ? x : residual;
  const dim3 grid((unsigned)n_items), blk(kThreads);
  if (residual_mode == 0) hipLaunchKernelGGL((topk_prep_hist<0>), grid, blk, 0, st, x, residual, items, hist);
  else if (residual_mode == 1) hipLaunchKernelGGL((topk_prep_hist<1>), grid, blk, 0, st, x, residual, items, hist);
  else hipLaunchKernelGGL((topk_prep_hist<2>), grid, blk, 0, st, x, residual, items, hist);
  hipLaunchKernelGGL(topk_select_bin, dim3((unsigned)nt), blk, 0, st, hist, kk, bin);
  const bool glob = global_path(plan);
  size_t tmp_bytes = L.tmp_bytes;
  if (glob) {
    hipLaunchKernelGGL((topk_collect<true>), grid, blk, 0, st, tp, items, d_begins, bin, cnt, item_cnt, cand);
    size_t sb = L.tmp_bytes;
    OMF_HIP(rocprim::exclusive_scan(w + L.tmp, sb, item_cnt, item_off, 0u, (size_t)n_items,
                                    rocprim::plus<uint32_t>(), st, false));
    hipLaunchKernelGGL(topk_tensor_ranges, dim3(64), blk, 0, st, items, n_items, item_cnt, item_off, cstart, cnt);
    OMF_HIP(hipGetLastError());
    uint32_t last[2];  // the sort needs the candidate count on the host
    OMF_HIP(hipMemcpyAsync(&last[0], item_off + n_items - 1, 4, hipMemcpyDeviceToHost, st));
    OMF_HIP(hipMemcpyAsync(&last[1], item_cnt + n_items - 1, 4, hipMemcpyDeviceToHost, st));
    OMF_HIP(hipStreamSynchronize(st));
    const uint64_t total = (uint64_t)last[0] + last[1];
    hipLaunchKernelGGL(topk_compact, grid, blk, 0, st, cand, items, item_cnt, item_off, sorted);
    // sort the packed keys back into `cand` (the per-item regions are no longer needed)
    OMF_HIP(rocprim::radix_sort_keys(w + L.tmp, tmp_bytes, sorted, cand, (size_t)total, 0, 64, st, false));
  } else {
    hipLaunchKernelGGL((topk_collect<false>), grid, blk, 0, st, tp, items, d_begins, bin, cnt, item_cnt, cand);
    hipLaunchKernelGGL(topk_offsets, dim3(1), dim3(64), 0, st, d_sizes, nt, ratio, kk, koff, d_begins, cnt,
                       seg_b, seg_e, 1);
    OMF_HIP(hipGetLastError());
    OMF_HIP(rocprim::segmented_radix_sort_keys_desc(w + L.tmp, tmp_bytes, cand, sorted,
                                                    (unsigned int)omf_plan_access::arena_end(plan), (unsigned int)nt,
                                                    seg_b, seg_e, 0, 64, st, false));
  }
  const uint64_t* sorted_keys = glob ? cand : sorted;
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((kmax + kThreads - 1) / kThreads, 1024));
  if (glob)
    hipLaunchKernelGGL((topk_gather<true>), dim3(gx, (unsigned)nt), blk, 0, st, tp, residual_mode ? residual : nullptr,
                       sorted_keys, d_begins, cstart, kk, koff, values, indices);
  else
    hipLaunchKernelGGL((topk_gather<false>), dim3(gx, (unsigned)nt), blk, 0, st, tp,
                       residual_mode ? residual : nullptr, sorted_keys, d_begins, cstart, kk, koff, values, indices);
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
