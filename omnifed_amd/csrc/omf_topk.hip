// omf_topk.hip — Top-K sparsification with error feedback, MI355X (gfx950).
//
// Semantics: src/omnifed/hybrid/compression/topk.py:10-47 + core.py:19-37 (reference):
//   t' = residual + alpha * x ; k = max(1, int(n * ratio)) ; the k largest |t'| ;
//   residual := t' - desparse(values, indices)  (= t' with the selected slots set to t'-t').
// alpha is the client weighting param * batch_samples (global_grpc.py:101-123), fused in;
// alpha = 1 leaves x's bits unchanged.
//
// Passes (all tensors of a plan per launch; <= 256 tensors of <= 2^25 elements):
//   1. topk_sample_threshold, one block per tensor: one aligned 16-element run of t' per
//                       max(256, n/4096) elements (hashed position; a random 64-byte sector
//                       costs the same as one element) into an LDS 8192-bin histogram of the top 13 bits of
//                       |t'| (exponent + 5 mantissa bits); the bin whose suffix holds
//                       k*S/n + 6 sqrt(k*S/n) + 32 of the S samples is the threshold — below
//                       the k-th magnitude with ~6 sigma of margin (tensors too small to
//                       sample keep every element).
//   3. topk_fused       ONE streaming pass: read x (+ residual), write t' into the residual,
//                       and append every |t'| at or above the threshold (~1.1-1.8 k) as a
//                       64-bit key (index << 39 | tensor << 31 | (2^31-1 - |t'|bits)) into the
//                       item's own region (one block scan per 8 Ki elements, no contended
//                       atomics).
//   4. topk_check       candidates per tensor from the item scan; a tensor whose sample put
//                       the threshold too high (fewer than k) is redone exactly from t': its
//                       1024-bin histogram, the bin of the k-th magnitude, a re-collection.
//   5. one device-wide radix sort of the candidates (rocPRIM onesweep): tensor ascending,
//      magnitude descending, index ascending (= torch's partial-sort order when k*64 <= n).
//   6. topk_gather      first k keys of every tensor -> values / int64 indices; zero the
//                       selected residual slots.
// Larger plans take the exact path (histogram of every t', collection, a segmented
// descending sort of (|t'|bits << 32 | ~index) per tensor).
// Decode is a scatter (mode 0 zero-fill, 1 overlay, 2 scatter-add).
#include <cmath>
#include <cstdlib>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <vector>

#include "../../include/omf_codec.h"
#include "omf_common.h"

using namespace omf;

namespace {

constexpr int kBins = 1024;
constexpr int kShift = 21;  // key (31 bits) >> 21 -> 10-bit bin (exact path)
constexpr int kSBits = 13;  // sample histogram: exponent + 5 mantissa bits
constexpr int kSBins = 1 << kSBits;
constexpr int kSShift = 31 - kSBits;
constexpr int kSRun = 16;       // a sample is a 64-byte run of 16 consecutive elements,
constexpr int kSStride = 256;   // one run per >= 256 elements,
constexpr int kSMaxRuns = 4096; // at most 4096 runs (64 Ki samples) per tensor
constexpr int kV = 16;
constexpr int64_t kSub = (int64_t)kV * kThreads * 4;
// Composite candidate key: index << 39 | tensor << 31 | (2^31 - 1 - |t'|bits).  Candidates are
// emitted in index order within each tensor, so a stable radix sort of the low 39 bits alone
// gives (tensor ascending, |t'| descending, index ascending): 5 digit passes instead of 8.
constexpr int kSortBits = 39;

// Mirrors the QSGD plan's item / tensor tables (omf_qsgd.hip); only the fields used here.
struct Item {
  int64_t begin, end;
  int32_t tensor, kind, chunk, pad;
};

__device__ __forceinline__ uint32_t mag_key(float v) { return __float_as_uint(v) & 0x7fffffffu; }

__device__ __forceinline__ uint32_t hash32(uint32_t h) {  // murmur3 finaliser
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  return h ^ (h >> 16);
}

// t' of one element: MODE 0/2: alpha * x ; MODE 1: r + alpha * x (the reference's order).
template <int MODE>
__device__ __forceinline__ float tprime(float x, float r, float alpha) {
  const float t = __fmul_rn(x, alpha);
  return MODE == 1 ? __fadd_rn(r, t) : t;
}

// Per tensor: k, the output offset, and the tensor's flat-item range (items are 16 Ki
// sub-chunks in tensor order: omf_qsgd.hip upload_plan).  One block; nt may exceed it.
__global__ __launch_bounds__(kThreads) void topk_setup(const int64_t* __restrict__ tsize, int32_t nt, double ratio,
                                                       int64_t* __restrict__ kk, int64_t* __restrict__ koff,
                                                       uint32_t* __restrict__ tfirst, uint32_t* __restrict__ tlast) {
  __shared__ int64_t s_k[kThreads], s_i[kThreads];
  int64_t carry_k = 0, carry_i = 0;
  for (int32_t t0 = 0; t0 < nt; t0 += kThreads) {
    const int32_t t = t0 + (int32_t)threadIdx.x;
    int64_t k = 0, ni = 0;
    if (t < nt) {
      k = (int64_t)((double)tsize[t] * ratio);
      if (k < 1) k = 1;
      ni = (tsize[t] + kSub - 1) / kSub;
    }
    s_k[threadIdx.x] = k;
    s_i[threadIdx.x] = ni;
    __syncthreads();
    for (int o = 1; o < kThreads; o <<= 1) {  // inclusive scans
      const int64_t ak = threadIdx.x >= (unsigned)o ? s_k[threadIdx.x - o] : 0;
      const int64_t ai = threadIdx.x >= (unsigned)o ? s_i[threadIdx.x - o] : 0;
      __syncthreads();
      s_k[threadIdx.x] += ak;
      s_i[threadIdx.x] += ai;
      __syncthreads();
    }
    if (t < nt) {
      kk[t] = k;
      koff[t] = carry_k + s_k[threadIdx.x] - k;
      tfirst[t] = (uint32_t)(carry_i + s_i[threadIdx.x] - ni);
      tlast[t] = (uint32_t)(carry_i + s_i[threadIdx.x] - 1);
      if (t == nt - 1) koff[nt] = carry_k + s_k[threadIdx.x];
    }
    carry_k += s_k[kThreads - 1];
    carry_i += s_i[kThreads - 1];
    __syncthreads();
  }
}

// Passes 1+2, one 1024-thread block per tensor: R = ceil(n / stride) runs, stride =
// max(256, n / 4096); run j covers 16 aligned elements at j*stride + 16 * (hash(.) % (span/16))
// (a whole 64-byte sector: random sectors, not elements, are what the sample costs), so
// S <= 16 R samples go into an LDS histogram of the top 13 bits of |t'|; then the bin whose
// suffix holds k*S/n + 6 sqrt(k*S/n) + 32 samples (0 = every element, for tensors too small
// to sample).  Four lanes read one run (float4 each).
__device__ __forceinline__ int64_t sample_stride(int64_t n) {
  return max((int64_t)kSStride, (n + kSMaxRuns - 1) / kSMaxRuns);
}
template <int MODE>
__global__ __launch_bounds__(1024) void topk_sample_threshold(const float* __restrict__ x, const float* __restrict__ r,
                                                              float alpha, const int64_t* __restrict__ tbegin,
                                                              const int64_t* __restrict__ tsize,
                                                              const int64_t* __restrict__ kk,
                                                              uint32_t* __restrict__ tbin,
                                                              uint32_t* __restrict__ hist) {
  constexpr int PER = kSBins / 1024;
  constexpr int U = 4;  // runs in flight per lane group
  __shared__ uint32_t h[kSBins];
  __shared__ uint32_t part[1024];
  const int t = blockIdx.x;
  for (int b = threadIdx.x; b < kSBins; b += 1024) h[b] = 0;
  for (int b = threadIdx.x; b < kBins; b += 1024) hist[(size_t)t * kBins + b] = 0;  // this call's redo histogram
  __syncthreads();
  const int64_t base = tbegin[t], n = tsize[t];
  const int64_t stride = sample_stride(n), nr = (n + stride - 1) / stride;
  const uint32_t salt = (uint32_t)t * 0x9E3779B9u;
  const int q = threadIdx.x & 3;  // float4 of the run
  for (int64_t j0 = threadIdx.x >> 2; j0 < nr; j0 += (int64_t)U * 256) {
    float4 xv[U], rv[U];
    int64_t rel[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // every load of the batch issued unconditionally (no branch
      // around a load: hipcc would wait for each one in turn); past-the-end runs clamped
      const int64_t j = min(j0 + (int64_t)u * 256, nr - 1);
      const int64_t lo = j * stride;
      const int64_t span = min(stride, n - lo);
      const int64_t runs = max((int64_t)1, span / kSRun);
      rel[u] = lo + kSRun * (int64_t)(hash32((uint32_t)lo ^ salt) % (uint32_t)runs) + 4 * q;
      const int64_t e = base + min(rel[u], (n - 1) & ~(int64_t)3);  // 16-byte aligned, inside the arena
      xv[u] = *reinterpret_cast<const float4*>(x + e);
      rv[u] = MODE == 1 ? *reinterpret_cast<const float4*>(r + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (j0 + (int64_t)u * 256 >= nr) continue;
      const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
      const float rs[4] = {rv[u].x, rv[u].y, rv[u].z, rv[u].w};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (rel[u] + c < n) atomicAdd(&h[mag_key(tprime<MODE>(xs[c], rs[c], alpha)) >> kSShift], 1u);
    }
  }
  __syncthreads();
  uint32_t c[PER], loc = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    c[j] = h[PER * threadIdx.x + j];
    loc += c[j];
  }
  part[threadIdx.x] = loc;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive suffix scan
    const uint32_t add = threadIdx.x + o < 1024 ? part[threadIdx.x + o] : 0u;
    __syncthreads();
    part[threadIdx.x] += add;
    __syncthreads();
  }
  const uint32_t S = part[0];
  const double m = (double)kk[t] * (double)S / (double)max(n, (int64_t)1);
  const double want = m + 6.0 * sqrt(m) + 32.0;
  if (m < 16.0 || want >= (double)S) {  // too few samples to trust: keep every element
    if (threadIdx.x == 0) tbin[t] = 0;
    return;
  }
  const uint32_t target = (uint32_t)ceil(want);
  uint32_t above = threadIdx.x + 1 < 1024 ? part[threadIdx.x + 1] : 0u;  // samples in higher bins
  for (int j = PER - 1; j >= 0; --j) {
    if (above < target && above + c[j] >= target) tbin[t] = PER * threadIdx.x + j;  // exactly one match
    above += c[j];
  }
}

// Append the selected elements of one 8 Ki-element pass of an item to the item's region in
// ascending element order (element idx0 + 1024 k + c of thread t is the pass's element
// 1024 k + 4 t + c): the 8 per-row counts of every thread are block-scanned as 16-bit
// fields, so a stable sort on the key bits above the index keeps index order for equal
// magnitudes (torch's tie order) without sorting the index bits.
struct PassCollector {
  uint32_t* s_wsum;  // 4 x kWaves packed row counts
  __device__ __forceinline__ uint32_t append(const float4 (&v)[8], uint32_t selm, uint64_t* dst, uint32_t idx0,
                                             uint64_t tag) const {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t pk[4], mine[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // rows 2i, 2i+1: counts 0..4 in 16-bit fields
      pk[i] = (uint32_t)__popc((selm >> (8 * i)) & 0xFu) | ((uint32_t)__popc((selm >> (8 * i + 4)) & 0xFu) << 16);
      mine[i] = pk[i];
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // wave inclusive scan (fields never carry: <= 256)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t u = __shfl_up(pk[i], o, 64);
        if (lane >= o) pk[i] += u;
      }
    }
    if (lane == 63) {
#pragma unroll
      for (int i = 0; i < 4; ++i) s_wsum[4 * wave + i] = pk[i];
    }
    __syncthreads();
    uint32_t wpre[4] = {0, 0, 0, 0}, tot[4] = {0, 0, 0, 0};
#pragma unroll
    for (int w2 = 0; w2 < kWaves; ++w2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t ws = s_wsum[4 * w2 + i];
        if (w2 < wave) wpre[i] += ws;
        tot[i] += ws;  // fields <= 1024: no carry
      }
    }
    __syncthreads();  // s_wsum reuse by the next pass
    uint32_t rowbase = 0, total = 0;
    uint32_t base[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = k >> 1, sh = 16 * (k & 1);
      const uint32_t ex = ((pk[i] - mine[i]) >> sh) & 0xFFFFu;  // threads before me in my wave
      base[k] = rowbase + ((wpre[i] >> sh) & 0xFFFFu) + ex;
      rowbase += (tot[i] >> sh) & 0xFFFFu;
    }
    total = rowbase;
    if (selm) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        uint32_t r = base[k];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if ((selm >> (4 * k + c)) & 1u) {
            const uint32_t idx = idx0 + 1024u * k + c;
            dst[r++] = ((uint64_t)idx << 39) | tag | (uint64_t)(0x7fffffffu - mag_key(vv[c]));
          }
        }
      }
    }
    return total;
  }
};

// Pass 3: t' (written to the residual in the EF modes) and the candidates above the
// sampled threshold, per item.  MODE 0: t' = alpha x (not stored); 1: r := r + alpha x;
// 2: r := alpha x.
template <int MODE>
__global__ __launch_bounds__(kThreads, MODE == 0 ? 4 : 6) void topk_fused(const float* __restrict__ x, float* __restrict__ r, float alpha,
                                                       const Item* __restrict__ items,
                                                       const int64_t* __restrict__ tbegin,
                                                       const uint32_t* __restrict__ tbin,
                                                       uint32_t* __restrict__ item_cnt, uint64_t* __restrict__ cand) {
  __shared__ uint32_t s_wsum[4 * kWaves];
  const Item it = items[blockIdx.x];
  const uint32_t thr = tbin[it.tensor];
  const int64_t base = tbegin[it.tensor];
  constexpr int64_t CS = 8 * kThreads * 4;  // 8192 elements per pass
  const PassCollector col{s_wsum};
  const uint64_t tag = (uint64_t)it.tensor << 31;
  uint32_t item_total = 0;
  for (int64_t b = it.begin; b < it.end; b += CS) {
    const uint32_t lim = (uint32_t)(min(b + CS, it.end) - b);
    const uint32_t off0 = 4u * threadIdx.x;
    float4 v[8];
    uint32_t selm = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t o = off0 + 1024u * k;
      float vv[4] = {0.f, 0.f, 0.f, 0.f};
      if (o + 4 <= lim) {
        const float4 xv = *reinterpret_cast<const float4*>(x + b + o);
        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (MODE == 1) rv = *reinterpret_cast<const float4*>(r + b + o);
        vv[0] = tprime<MODE>(xv.x, rv.x, alpha);
        vv[1] = tprime<MODE>(xv.y, rv.y, alpha);
        vv[2] = tprime<MODE>(xv.z, rv.z, alpha);
        vv[3] = tprime<MODE>(xv.w, rv.w, alpha);
        if (MODE != 0) *reinterpret_cast<float4*>(r + b + o) = make_float4(vv[0], vv[1], vv[2], vv[3]);
      } else {
        for (uint32_t c = 0; c < 4 && o + c < lim; ++c) {
          vv[c] = tprime<MODE>(x[b + o + c], MODE == 1 ? r[b + o + c] : 0.0f, alpha);
          if (MODE != 0) r[b + o + c] = vv[c];
        }
      }
      v[k] = make_float4(vv[0], vv[1], vv[2], vv[3]);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (o + c < lim && (mag_key(vv[c]) >> kSShift) >= thr) selm |= 1u << (4 * k + c);
    }
    item_total += col.append(v, selm, cand + it.begin + item_total, (uint32_t)(b - base) + off0, tag);
  }
  if (threadIdx.x == 0) item_cnt[blockIdx.x] = item_total;
}

// One block: exclusive scan of the per-item candidate counts (items in tensor order), then
// per tensor its candidate count and start; flag the tensors whose threshold was too high.
// status[0] = all candidates, status[1] = any flagged.  (Replaces a library scan: no
// workspace clears, one launch.)
__global__ __launch_bounds__(1024) void topk_scan_check(int32_t nt, const int64_t* __restrict__ kk,
                                                        const uint32_t* __restrict__ tfirst,
                                                        const uint32_t* __restrict__ tlast,
                                                        const uint32_t* __restrict__ item_cnt,
                                                        uint32_t* __restrict__ item_off, int64_t n_items,
                                                        int64_t* __restrict__ cstart, uint32_t* __restrict__ cnt,
                                                        uint32_t* __restrict__ flag, uint32_t* __restrict__ status) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t s_any;
  const int t = threadIdx.x;
  const int64_t per = (n_items + 1023) / 1024;
  const int64_t b = min((int64_t)t * per, n_items), e = min(b + per, n_items);
  uint32_t loc = 0;
  for (int64_t i = b; i < e; ++i) loc += item_cnt[i];
  part[t] = loc;
  if (t == 0) s_any = 0;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan
    const uint32_t add = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  uint32_t run = part[t] - loc;
  for (int64_t i = b; i < e; ++i) {
    item_off[i] = run;
    run += item_cnt[i];
  }
  // exclusive prefix of item i from the thread prefixes (no read-back of item_off)
  auto prefix = [&](int64_t i) -> uint32_t {
    const int64_t owner = i / per;
    uint32_t v = owner > 0 ? part[owner - 1] : 0u;
    for (int64_t j = owner * per; j < i; ++j) v += item_cnt[j];
    return v;
  };
  for (int32_t q = t; q < nt; q += 1024) {
    const uint32_t f = tfirst[q], l = tlast[q];
    const uint32_t of = prefix(f);
    const uint32_t c = prefix(l) + item_cnt[l] - of;
    cstart[q] = of;
    cnt[q] = c;
    const uint32_t redo = (int64_t)c < kk[q] ? 1u : 0u;
    flag[q] = redo;
    if (redo) s_any = 1u;
  }
  __syncthreads();
  if (t == 0) {
    status[0] = part[1023];
    status[1] = s_any;
  }
}

// Exact path, pass 1 (and the per-tensor redo): t' and its 1024-bin histogram per tensor.
// MODE as topk_fused.  flag != null: only the flagged tensors (a redo reads t' as x with
// MODE 0 and alpha = the scale of t').
template <int MODE>
__global__ __launch_bounds__(kThreads) void topk_prep_hist(const float* __restrict__ x, float* __restrict__ r,
                                                           float alpha, const Item* __restrict__ items,
                                                           const uint32_t* __restrict__ flag,
                                                           uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kBins];
  const Item it = items[blockIdx.x];
  if (flag && !flag[it.tensor]) return;  // block-uniform
  for (int b = threadIdx.x; b < kBins; b += kThreads) h[b] = 0;
  __syncthreads();
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
        const float4 xv = *reinterpret_cast<const float4*>(x + e);
        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (MODE == 1) rv = *reinterpret_cast<const float4*>(r + e);
        v[0] = tprime<MODE>(xv.x, rv.x, alpha);
        v[1] = tprime<MODE>(xv.y, rv.y, alpha);
        v[2] = tprime<MODE>(xv.z, rv.z, alpha);
        v[3] = tprime<MODE>(xv.w, rv.w, alpha);
        if (MODE != 0) *reinterpret_cast<float4*>(r + e) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        for (int c = 0; c < nv; ++c) {
          v[c] = tprime<MODE>(x[e + c], MODE == 1 ? r[e + c] : 0.0f, alpha);
          if (MODE != 0) r[e + c] = v[c];
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

// One block per tensor: b1 = max bin with suffix count >= k (flag: only flagged tensors).
__global__ __launch_bounds__(kThreads) void topk_select_bin(const uint32_t* __restrict__ hist,
                                                            const int64_t* __restrict__ kk,
                                                            const uint32_t* __restrict__ flag,
                                                            uint32_t* __restrict__ bin) {
  __shared__ uint32_t s_part[kThreads];
  const int t = blockIdx.x;
  if (flag && !flag[t]) return;
  const uint32_t* ht = hist + (size_t)t * kBins;
  // thread i owns bins [4i, 4i+4); suffix sums over threads from the top.
  uint32_t c[4], loc = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) { c[j] = ht[4 * threadIdx.x + j]; loc += c[j]; }
  s_part[threadIdx.x] = loc;
  __syncthreads();
  for (int o = 1; o < kThreads; o <<= 1) {  // inclusive suffix scan (Hillis-Steele)
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

// Segment bounds of the exact path's per-tensor sort.
__global__ void topk_segments(int32_t nt, const int64_t* __restrict__ tbegin, const uint32_t* __restrict__ cnt,
                              uint32_t* __restrict__ seg_b, uint32_t* __restrict__ seg_e) {
  for (int32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
    seg_b[t] = (uint32_t)tbegin[t];
    seg_e[t] = (uint32_t)(tbegin[t] + cnt[t]);
  }
}

// Exact-path candidates of one item: every t' (= scale * tp) whose bin is >= b1.
// GLOBAL: composite keys into the item's own region, counted per item (redo: flagged
// tensors only).  Otherwise (|t'|bits << 32 | ~index) appended to the tensor's region
// through one atomic per block pass.
template <bool GLOBAL>
__global__ __launch_bounds__(kThreads) void topk_collect(const float* __restrict__ tp, float scale,
                                                         const Item* __restrict__ items,
                                                         const int64_t* __restrict__ tbegin,
                                                         const uint32_t* __restrict__ bin,
                                                         const uint32_t* __restrict__ flag, uint32_t* __restrict__ cnt,
                                                         uint32_t* __restrict__ item_cnt, uint64_t* __restrict__ cand) {
  __shared__ uint32_t s_wsum[4 * kWaves];
  __shared__ uint32_t s_base;
  const Item it = items[blockIdx.x];
  if (flag && !flag[it.tensor]) return;  // block-uniform
  const uint32_t b1 = bin[it.tensor];
  const int64_t base = tbegin[it.tensor];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int CV = 8;
  constexpr int64_t CS = (int64_t)CV * kThreads * 4;
  const PassCollector col{s_wsum};
  const uint64_t tag = (uint64_t)it.tensor << 31;
  uint32_t item_total = 0;
  for (int64_t b = it.begin; b < it.end; b += CS) {
    const uint32_t lim = (uint32_t)(min(b + CS, it.end) - b);
    const uint32_t off0 = 4u * threadIdx.x;
    float4 v[CV];
    uint32_t selm = 0;
#pragma unroll
    for (int k = 0; k < CV; ++k) {
      const uint32_t o = off0 + 1024u * k;
      float vv[4] = {0.f, 0.f, 0.f, 0.f};
      if (o + 4 <= lim) {
        const float4 t4 = *reinterpret_cast<const float4*>(tp + b + o);
        vv[0] = t4.x; vv[1] = t4.y; vv[2] = t4.z; vv[3] = t4.w;
      } else {
        for (uint32_t c = 0; c < 4 && o + c < lim; ++c) vv[c] = tp[b + o + c];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) vv[c] = __fmul_rn(vv[c], scale);
      v[k] = make_float4(vv[0], vv[1], vv[2], vv[3]);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (o + c < lim && (mag_key(vv[c]) >> kShift) >= b1) selm |= 1u << (4 * k + c);
    }
    if (GLOBAL) {
      item_total += col.append(v, selm, cand + it.begin + item_total, (uint32_t)(b - base) + off0, tag);
      continue;
    }
    const uint32_t nsel = (uint32_t)__popc(selm);
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
    if (threadIdx.x == 0) s_base = tot ? atomicAdd(&cnt[it.tensor], tot) : 0u;
    __syncthreads();
    uint64_t* dst = cand + base + s_base + wpre;
    const uint32_t idx0 = (uint32_t)(b - base) + off0;
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
            dst[__popcll(m & lt)] = ((uint64_t)mag_key(vv[c]) << 32) | (uint64_t)(~idx);
          }
          dst += __popcll(m);
        }
      }
    }
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

template <bool GLOBAL>
__global__ __launch_bounds__(kThreads) void topk_gather(const float* __restrict__ tp, float scale,
                                                        float* __restrict__ r, const uint64_t* __restrict__ sorted,
                                                        const int64_t* __restrict__ tbegin,
                                                        const int64_t* __restrict__ tsize,
                                                        const int64_t* __restrict__ cstart,
                                                        const int64_t* __restrict__ kk, const int64_t* __restrict__ koff,
                                                        float* __restrict__ values, int64_t* __restrict__ indices) {
  const int t = blockIdx.y;
  const int64_t k = kk[t], base = tbegin[t], o = koff[t], n = tsize[t];
  const int64_t s0 = GLOBAL ? cstart[t] : base;
  for (int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x; j < k; j += (int64_t)gridDim.x * kThreads) {
    const uint64_t key = sorted[s0 + j];
    const uint32_t idx = GLOBAL ? (uint32_t)(key >> 39) : ~(uint32_t)key;
    if (idx >= n || (GLOBAL && (int)((key >> 31) & 0xFFu) != t)) {  // never expected: a key of another tensor
      values[o + j] = 0.0f;
      indices[o + j] = -1;
      continue;
    }
    const float v = __fmul_rn(tp[base + idx], scale);
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

// Whole-arena decode of one client's selection (values/indices packed per tensor at
// K_t = sum_{u<t} k_u, tensor-local indices): y[begin_t + idx] = v (mode 0/1) or += v (2).
// Indices are unique within a client, so the read-modify-write needs no atomics.
constexpr int kArenaMaxTensors = 4096;
__global__ __launch_bounds__(kThreads) void topk_scatter_arena(const float* __restrict__ values,
                                                               const int64_t* __restrict__ indices,
                                                               const int64_t* __restrict__ sizes,
                                                               const int64_t* __restrict__ begins, int nt,
                                                               double ratio, int64_t ktot, float* __restrict__ y,
                                                               int add) {
  __shared__ int64_t koff[kArenaMaxTensors + 1];
  if (threadIdx.x == 0) {  // k_t exactly as omf_topk_k, prefix-summed (nt is small)
    int64_t acc = 0;
    for (int t = 0; t < nt; ++t) {
      koff[t] = acc;
      const int64_t k = (int64_t)((double)sizes[t] * ratio);
      acc += k < 1 ? 1 : k;
    }
    koff[nt] = acc;
  }
  __syncthreads();
  for (int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x; j < ktot; j += (int64_t)gridDim.x * kThreads) {
    int lo = 0, hi = nt - 1;  // the tensor t with koff[t] <= j < koff[t + 1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (koff[mid] <= j) lo = mid;
      else hi = mid - 1;
    }
    const int64_t i = indices[j];
    if (i < 0 || i >= sizes[lo]) continue;  // padding (-1) or out of range: skipped
    float* p = y + begins[lo] + i;
    *p = add ? __fadd_rn(*p, values[j]) : values[j];
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
  } else {
    uint32_t* off = nullptr;
    (void)rocprim::segmented_radix_sort_keys_desc(nullptr, bytes, dummy, dummy, (unsigned int)size, (unsigned int)nt,
                                                  off, off, 0, 64, (hipStream_t)0, false);
  }
  return bytes;
}

// Workspace: everything up to `zero_end` is cleared once per call on the exact path; the
// sampled path clears its redo histograms in topk_sample_threshold and writes the rest.
struct WsLayout {
  size_t hist, bin, cnt, flag, status, zero_end, tbin, koff, kk, tfirst, tlast, seg_b, seg_e, cstart,
      item_cnt, item_off, cand, sorted, tmp, total, tmp_bytes;
};

WsLayout layout(const omf_plan* p) {
  const int32_t nt = omf_plan_access::ntensors(p);
  const int64_t ae = omf_plan_access::arena_end(p);
  WsLayout L;
  size_t o = 0;
  L.hist = o; o = align256(o + 4 * (size_t)nt * kBins);
  L.bin = o; o = align256(o + 4 * (size_t)nt);
  L.cnt = o; o = align256(o + 4 * (size_t)nt);
  L.flag = o; o = align256(o + 4 * (size_t)nt);
  L.status = o; o = align256(o + 16);
  L.zero_end = o;
  L.tbin = o; o = align256(o + 4 * (size_t)nt);
  L.koff = o; o = align256(o + 8 * (size_t)(nt + 1));
  L.kk = o; o = align256(o + 8 * (size_t)nt);
  L.tfirst = o; o = align256(o + 4 * (size_t)nt);
  L.tlast = o; o = align256(o + 4 * (size_t)nt);
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

int omf_topk_encode(omf_plan* plan, const float* x, float* residual, int32_t residual_mode, double ratio, float alpha,
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
  uint32_t* flag = reinterpret_cast<uint32_t*>(w + L.flag);
  uint32_t* status = reinterpret_cast<uint32_t*>(w + L.status);
  uint32_t* tbin = reinterpret_cast<uint32_t*>(w + L.tbin);
  int64_t* koff = reinterpret_cast<int64_t*>(w + L.koff);
  int64_t* kk = reinterpret_cast<int64_t*>(w + L.kk);
  uint32_t* tfirst = reinterpret_cast<uint32_t*>(w + L.tfirst);
  uint32_t* tlast = reinterpret_cast<uint32_t*>(w + L.tlast);
  uint32_t* seg_b = reinterpret_cast<uint32_t*>(w + L.seg_b);
  uint32_t* seg_e = reinterpret_cast<uint32_t*>(w + L.seg_e);
  int64_t* cstart = reinterpret_cast<int64_t*>(w + L.cstart);
  uint32_t* item_cnt = reinterpret_cast<uint32_t*>(w + L.item_cnt);
  uint32_t* item_off = reinterpret_cast<uint32_t*>(w + L.item_off);
  uint64_t* cand = reinterpret_cast<uint64_t*>(w + L.cand);
  uint64_t* sorted = reinterpret_cast<uint64_t*>(w + L.sorted);
  const int32_t nt = omf_plan_access::ntensors(plan);
  int64_t n_items = 0;
  const Item* items = static_cast<const Item*>(omf_plan_access::flat_items(plan, &n_items));
  const int64_t* d_sizes = omf_plan_access::d_sizes(plan);
  const int64_t* d_begins = omf_plan_access::d_begins(plan);
  // t' lives in the residual (EF modes) or is alpha * x (mode 0)
  const float* tp = residual_mode == 0 ? x : residual;
  const float scale = residual_mode == 0 ? alpha : 1.0f;
  float* rz = residual_mode ? residual : nullptr;  // selected slots to zero
  const dim3 grid((unsigned)n_items), blk(kThreads);

  const bool glob = global_path(plan);
  if (!glob) OMF_HIP(hipMemsetAsync(w, 0, L.zero_end, st));
  hipLaunchKernelGGL(topk_setup, dim3(1), blk, 0, st, d_sizes, nt, ratio, kk, koff, tfirst, tlast);
  size_t tmp_bytes = L.tmp_bytes;
  if (glob) {
    const dim3 sgrid((unsigned)nt), sblk(1024);
    if (residual_mode == 1) {
      hipLaunchKernelGGL((topk_sample_threshold<1>), sgrid, sblk, 0, st, x, residual, alpha, d_begins, d_sizes, kk,
                         tbin, hist);
      hipLaunchKernelGGL((topk_fused<1>), grid, blk, 0, st, x, residual, alpha, items, d_begins, tbin, item_cnt, cand);
    } else {
      hipLaunchKernelGGL((topk_sample_threshold<0>), sgrid, sblk, 0, st, x, residual, alpha, d_begins, d_sizes, kk,
                         tbin, hist);
      if (residual_mode == 2)
        hipLaunchKernelGGL((topk_fused<2>), grid, blk, 0, st, x, residual, alpha, items, d_begins, tbin, item_cnt,
                           cand);
      else
        hipLaunchKernelGGL((topk_fused<0>), grid, blk, 0, st, x, residual, alpha, items, d_begins, tbin, item_cnt,
                           cand);
    }
    uint32_t host_status[2] = {0, 0};
    auto scan_and_check = [&]() -> int {
      hipLaunchKernelGGL(topk_scan_check, dim3(1), dim3(1024), 0, st, nt, kk, tfirst, tlast, item_cnt, item_off,
                         n_items, cstart, cnt, flag, status);
      OMF_HIP(hipGetLastError());
      // the sort needs the candidate count on the host (and the redo decision)
      OMF_HIP(hipMemcpyAsync(host_status, status, 8, hipMemcpyDeviceToHost, st));
      OMF_HIP(hipStreamSynchronize(st));
      return OMF_OK;
    };
    if (int rc = scan_and_check()) return rc;
    if (host_status[1]) {  // a sample set the threshold too high for some tensor: redo it exactly
      hipLaunchKernelGGL((topk_prep_hist<0>), grid, blk, 0, st, tp, nullptr, scale, items, flag, hist);
      hipLaunchKernelGGL(topk_select_bin, dim3((unsigned)nt), blk, 0, st, hist, kk, flag, bin);
      hipLaunchKernelGGL((topk_collect<true>), grid, blk, 0, st, tp, scale, items, d_begins, bin, flag, cnt, item_cnt,
                         cand);
      if (int rc = scan_and_check()) return rc;
    }
    const uint64_t total = host_status[0];
    hipLaunchKernelGGL(topk_compact, grid, blk, 0, st, cand, items, item_cnt, item_off, sorted);
    // sort the packed keys back into `cand` (the per-item regions are no longer needed):
    // candidates are in index order within each tensor, so a stable sort of the tensor and
    // magnitude bits alone yields (tensor, |t'| descending, index ascending)
    OMF_HIP(rocprim::radix_sort_keys(w + L.tmp, tmp_bytes, sorted, cand, (size_t)total, 0, kSortBits, st, false));
  } else {
    if (residual_mode == 0)
      hipLaunchKernelGGL((topk_prep_hist<0>), grid, blk, 0, st, x, residual, alpha, items, nullptr, hist);
    else if (residual_mode == 1)
      hipLaunchKernelGGL((topk_prep_hist<1>), grid, blk, 0, st, x, residual, alpha, items, nullptr, hist);
    else
      hipLaunchKernelGGL((topk_prep_hist<2>), grid, blk, 0, st, x, residual, alpha, items, nullptr, hist);
    hipLaunchKernelGGL(topk_select_bin, dim3((unsigned)nt), blk, 0, st, hist, kk, nullptr, bin);
    hipLaunchKernelGGL((topk_collect<false>), grid, blk, 0, st, tp, scale, items, d_begins, bin, nullptr, cnt, item_cnt,
                       cand);
    hipLaunchKernelGGL(topk_segments, dim3(((unsigned)nt + kThreads - 1) / kThreads), blk, 0, st, nt, d_begins, cnt,
                       seg_b, seg_e);
    OMF_HIP(hipGetLastError());
    OMF_HIP(rocprim::segmented_radix_sort_keys_desc(w + L.tmp, tmp_bytes, cand, sorted,
                                                    (unsigned int)omf_plan_access::arena_end(plan), (unsigned int)nt,
                                                    seg_b, seg_e, 0, 64, st, false));
  }
  const uint64_t* sorted_keys = glob ? cand : sorted;
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((kmax + kThreads - 1) / kThreads, 1024));
  if (glob)
    hipLaunchKernelGGL((topk_gather<true>), dim3(gx, (unsigned)nt), blk, 0, st, tp, scale, rz, sorted_keys, d_begins,
                       d_sizes, cstart, kk, koff, values, indices);
  else
    hipLaunchKernelGGL((topk_gather<false>), dim3(gx, (unsigned)nt), blk, 0, st, tp, scale, rz, sorted_keys, d_begins,
                       d_sizes, cstart, kk, koff, values, indices);
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

int omf_topk_decode_arena(omf_plan* plan, double ratio, const float* values, const int64_t* indices, float* y,
                          int32_t mode, void* stream) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  if (mode < 0 || mode > 2) return fail(OMF_EINVAL, "omf_topk_decode_arena: mode must be 0, 1 or 2");
  if (!(ratio == ratio)) return fail(OMF_EINVAL, "ratio is NaN");
  if (!values || !indices || !y) return fail(OMF_EINVAL, "omf_topk_decode_arena: NULL buffer");
  const int32_t nt = omf_plan_access::ntensors(plan);
  if (nt > kArenaMaxTensors) return fail(OMF_EINVAL, "omf_topk_decode_arena: too many tensors (decode per tensor)");
  int64_t ktot = 0;
  for (int64_t n : omf_plan_access::sizes(plan)) {
    const int64_t k = omf_topk_k(n, ratio);
    if (k > n) return fail(OMF_EINVAL, "selected index k out of range (k > numel): compress_ratio too large");
    ktot += k;
  }
  DeviceGuard g(omf_plan_access::device(plan));
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;
  if (mode == 0) OMF_HIP(hipMemsetAsync(y, 0, 4 * (size_t)omf_plan_access::arena_end(plan), st));
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ktot + kThreads - 1) / kThreads, 4096));
  hipLaunchKernelGGL(topk_scatter_arena, dim3(gx), dim3(kThreads), 0, st, values, indices,
                     omf_plan_access::d_sizes(plan), omf_plan_access::d_begins(plan), (int)nt, ratio, ktot, y,
                     mode == 2 ? 1 : 0);
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
