// omf_topk_host.cpp — the reference's Top-K selection rule on the host (ties, order), no GPU.
//
// The reference selects with torch.topk(t.abs(), k, sorted=False) on the CPU
// (src/omnifed/hybrid/compression/topk.py:13; the compressor is always built with device="cpu":
// src/omnifed/hybrid/grpc_leader_comm.py:59, slurm_hybrid_runner.py:437).  torch's CPU kernel
// (ATen/native/TopKImpl.h, topk_impl_loop) fills (|t_i|, i) pairs in index order, then
//   k * 64 <= n:  std::partial_sort(q, q + k, q + n, comp)     (libstdc++: heap select + heap sort)
//   otherwise:    std::nth_element(q, q + k - 1, q + n, comp)  (introselect; no sort: sorted=False)
// with comp(a, b) = (isnan(a) && !isnan(b)) || a > b on the magnitudes alone.  The selection and
// its order are therefore fixed by those algorithms wherever magnitudes tie: which of several
// equal magnitudes at rank k are taken, and the order of equal magnitudes inside the selection
// (a 32 Mi-element Gaussian tensor's top 1 % holds ~19 000 equal pairs).
//
// Here:
//   - magnitudes become 31-bit keys (the bits of |t|, every NaN one key above +inf), so
//     comp(a, b) == key(a) > key(b) exactly (equal keys <=> neither is before the other);
//   - the heap regime is libstdc++'s algorithm restated on a k-entry heap: make the heap of the
//     first k pairs (std::make_heap), then for each later pair that compares before the top, the
//     top's replacement (__pop_heap(first, middle, i): the hole walks from the root to a leaf along
//     the child that is not "before" its sibling — the right one on a tie — and the new pair
//     bubbles up from there), then the heap sort (the same replacement with the last entry,
//     shrinking).  Pairs that never enter the heap are only compared, so the n-pair array is never
//     built; keys and indices live in two arrays, the walk reading keys only;
//   - the introselect regime calls std::nth_element on the n pairs with the same comparison.
// tests/test_topk_order_host.py pins both against torch.topk on tie-heavy inputs (CPU).
#include <immintrin.h>

#include <algorithm>
#ifdef OMF_EXP_TIE_TS
#include <chrono>
#include <cstdio>
#endif
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/omf_codec.h"

namespace omf {

int fail(int code, const std::string& msg);

namespace {

typedef uint64_t Entry;  // magnitude key << 32 | index

inline uint32_t mag_key_host(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u &= 0x7fffffffu;
  return u > 0x7f800000u ? 0x7fc00000u : u;  // every NaN: one key, above +inf
}

struct Before {  // torch's comparison: a goes before b
  bool operator()(Entry a, Entry b) const { return (a >> 32) > (b >> 32); }
};

// libstdc++'s __adjust_heap(h, 0, len, v) followed by its __push_heap — the replacement of the
// top of the heap [0, len) by (kv, iv) — on split key / index arrays (the walk reads keys only).
// The hole walks from the root to a leaf along the child that is not "before" its sibling (the
// right one on a tie), two levels per step where both exist: the children and the four
// grandchildren are loaded together and the two choices made without branches, so one memory
// round trip serves two levels; then the new pair bubbles up from the leaf.
inline void replace_top(uint32_t* __restrict K, uint32_t* __restrict I, int64_t len, uint32_t kv, uint32_t iv) {
  int64_t hole = 0;
  const int64_t inner = (len - 1) / 2;    // a hole below this has two children
  const int64_t inner2 = (inner - 1) / 2;  // ... and so do both of them
  while (hole < inner2) {
    __builtin_prefetch(&K[16 * hole + 15]);  // four levels down
    const int64_t c = 2 * hole + 1;
    const uint32_t kl = K[c], kr = K[c + 1];
    const uint32_t g0 = K[2 * c + 1], g1 = K[2 * c + 2], g2 = K[2 * c + 3], g3 = K[2 * c + 4];
    const bool left = kr > kl;
    const int64_t cc = left ? c : c + 1;
    const uint32_t a = left ? g0 : g2, b = left ? g1 : g3;
    const bool left2 = b > a;
    const int64_t c2 = 2 * cc + (left2 ? 1 : 2);
    K[hole] = left ? kl : kr;
    I[hole] = I[cc];
    K[cc] = left2 ? a : b;
    I[cc] = I[c2];
    hole = c2;
  }
  while (hole < inner) {
    const int64_t c = 2 * hole + 1;
    const int64_t cc = K[c + 1] > K[c] ? c : c + 1;
    K[hole] = K[cc];
    I[hole] = I[cc];
    hole = cc;
  }
  if ((len & 1) == 0 && hole == (len - 2) / 2) {  // the one node with a left child only
    const int64_t c = 2 * hole + 1;
    K[hole] = K[c];
    I[hole] = I[c];
    hole = c;
  }
  int64_t parent = (hole - 1) / 2;
  while (hole > 0 && K[parent] > kv) {
    K[hole] = K[parent];
    I[hole] = I[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  K[hole] = kv;
  I[hole] = iv;
}

// The heap select's pass over t[k, n): every element whose key beats the heap's top replaces the top,
// in index order.  The top only grows, so an element whose key does not beat the top as it was at the
// start of its group of 8 cannot beat it later: the AVX2 pass compares 8 keys at once against that top
// and visits, in order, only the lanes that beat it (each re-checked against the current top) — the
// same replacements in the same order as the scalar loop, about a third of the groups visited at k = 1 %.
inline void heap_pass_scalar(const float* t, int64_t k, int64_t n, uint32_t* kp, uint32_t* ip, int64_t len) {
  for (int64_t i = k; i < n; ++i) {
    const uint32_t key = mag_key_host(t[i]);
    if (key > kp[0]) replace_top(kp, ip, len, key, (uint32_t)i);  // before(pair i, top): it replaces the top
  }
}
__attribute__((target("avx2"))) void heap_pass_avx2(const float* t, int64_t k, int64_t n, uint32_t* kp, uint32_t* ip,
                                                    int64_t len) {
  const __m256i abs_mask = _mm256_set1_epi32(0x7fffffff), inf = _mm256_set1_epi32(0x7f800000),
                nan_key = _mm256_set1_epi32(0x7fc00000);
  int64_t i = k;
  for (; i < n && (i & 7); ++i) {  // to an 8-element boundary of t (aligned loads below when t is)
    const uint32_t key = mag_key_host(t[i]);
    if (key > kp[0]) replace_top(kp, ip, len, key, (uint32_t)i);
  }
  for (; i + 8 <= n; i += 8) {
    const __m256i u = _mm256_and_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(t + i)), abs_mask);
    const __m256i key = _mm256_blendv_epi8(u, nan_key, _mm256_cmpgt_epi32(u, inf));  // keys < 2^31: signed compare
    uint32_t m = (uint32_t)_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_cmpgt_epi32(key, _mm256_set1_epi32((int)kp[0]))));
    while (m) {
      const int j = __builtin_ctz(m);
      m &= m - 1;
      const uint32_t kv = mag_key_host(t[i + j]);
      if (kv > kp[0]) replace_top(kp, ip, len, kv, (uint32_t)(i + j));
    }
  }
  for (; i < n; ++i) {
    const uint32_t key = mag_key_host(t[i]);
    if (key > kp[0]) replace_top(kp, ip, len, key, (uint32_t)i);
  }
}

}  // namespace

// torch.topk(|t|, k, sorted=False).indices of t[0, n) on the CPU, into out[0, k).  1 <= k <= n < 2^32.
int torch_topk_select(const float* t, int64_t n, int64_t k, int64_t* out) {
  if (k < 1 || k > n || n > 0xffffffffLL) return fail(OMF_EINVAL, "omf_topk_select_host: need 1 <= k <= n < 2^32");
  const Before before;
  if (k * 64 <= n) {
    std::vector<Entry> h;
    std::vector<uint32_t> K, I;
    try {
      h.resize((size_t)k);
      K.resize((size_t)k + 64);
      I.resize((size_t)k + 64);
    } catch (const std::bad_alloc&) {
      return fail(OMF_ENOMEM, "omf_topk_select_host: heap allocation failed");
    }
    for (int64_t i = 0; i < k; ++i) h[i] = (Entry)mag_key_host(t[i]) << 32 | (uint32_t)i;
    std::make_heap(h.begin(), h.end(), before);
    for (int64_t i = 0; i < k; ++i) {
      K[i] = (uint32_t)(h[i] >> 32);
      I[i] = (uint32_t)h[i];
    }
    uint32_t* kp = K.data();
    uint32_t* ip = I.data();
#ifdef OMF_EXP_TIE_TS
    const auto T0 = std::chrono::steady_clock::now();
    const int64_t nrep = -1;  // (not counted since the AVX2 pass)
#endif
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2)
      heap_pass_avx2(t, k, n, kp, ip, k);
    else
      heap_pass_scalar(t, k, n, kp, ip, k);
#ifdef OMF_EXP_TIE_TS
    const auto T1 = std::chrono::steady_clock::now();
#endif
    for (int64_t last = k - 1; last > 0; --last) {  // the heap sort: __pop_heap(h, h + last, h + last)
      const uint32_t kv = kp[last], iv = ip[last];
      kp[last] = kp[0];
      ip[last] = ip[0];
      replace_top(kp, ip, last, kv, iv);
    }
#ifdef OMF_EXP_TIE_TS
    if (n >= (1 << 24))
      fprintf(stderr, "TIE_HEAP n=%lld k=%lld replacements=%lld select=%.1f sort=%.1f ms\n", (long long)n, (long long)k,
              (long long)nrep, std::chrono::duration<double, std::milli>(T1 - T0).count(),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T1).count());
#endif
    for (int64_t j = 0; j < k; ++j) out[j] = (int64_t)ip[j];
    return OMF_OK;
  }
  std::vector<Entry> q;
  try {
    q.resize((size_t)n);
  } catch (const std::bad_alloc&) {
    return fail(OMF_ENOMEM, "omf_topk_select_host: pair array allocation failed");
  }
  for (int64_t i = 0; i < n; ++i) q[i] = (Entry)mag_key_host(t[i]) << 32 | (uint32_t)i;
  std::nth_element(q.begin(), q.begin() + (k - 1), q.end(), before);
  for (int64_t j = 0; j < k; ++j) out[j] = (int64_t)(uint32_t)q[j];
  return OMF_OK;
}

}  // namespace omf

extern "C" int omf_topk_select_host(const float* t, int64_t n, int64_t k, int64_t* indices) {
  if (!t || !indices) return omf::fail(OMF_EINVAL, "omf_topk_select_host: t and indices must be non-NULL");
  return omf::torch_topk_select(t, n, k, indices);
}
