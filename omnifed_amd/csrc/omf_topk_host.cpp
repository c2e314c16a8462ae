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
//     first k pairs, then for each later pair that compares before the top, the top's
//     replacement (__pop_heap(first, middle, i): the hole walks from the root to a leaf along the
//     child that is not "before" its sibling — the right one on a tie — and the new pair bubbles
//     up from there), then the heap sort (the same replacement with the last entry, shrinking).
//     Pairs that never enter the heap are only compared, so the n-pair array is never built;
//   - the introselect regime calls std::nth_element on the n pairs with the same comparison.
// tests/test_topk_order_host.py pins both against torch.topk on tie-heavy inputs (CPU).
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
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

// libstdc++'s __adjust_heap(h, 0, len, v) followed by its __push_heap: the replacement of the
// top of the heap h[0, len) by v.  The walk prefetches the one 64-byte line that holds the hole's
// descendants three levels down (the heap's base is placed so that line is aligned).
inline void replace_top(Entry* h, int64_t len, Entry v) {
  const Before before;
  int64_t hole = 0, child = 0;
  const int64_t inner = (len - 1) / 2;
  while (child < inner) {
    __builtin_prefetch(&h[8 * (child + 1) - 1]);
    child = 2 * (child + 1);
    if (before(h[child], h[child - 1])) --child;
    h[hole] = h[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    h[hole] = h[child - 1];
    hole = child - 1;
  }
  int64_t parent = (hole - 1) / 2;
  while (hole > 0 && before(h[parent], v)) {
    h[hole] = h[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  h[hole] = v;
}

struct AlignedEntries {
  Entry* base = nullptr;
  Entry* data = nullptr;  // data[8m - 1] starts a 64-byte line
  explicit AlignedEntries(int64_t n) {
    base = static_cast<Entry*>(::operator new[](sizeof(Entry) * (size_t)(n + 8), std::align_val_t(64), std::nothrow));
    data = base ? base + 1 : nullptr;
  }
  ~AlignedEntries() {
    if (base) ::operator delete[](base, std::align_val_t(64));
  }
  AlignedEntries(const AlignedEntries&) = delete;
  AlignedEntries& operator=(const AlignedEntries&) = delete;
};

}  // namespace

// torch.topk(|t|, k, sorted=False).indices of t[0, n) on the CPU, into out[0, k).  1 <= k <= n < 2^32.
int torch_topk_select(const float* t, int64_t n, int64_t k, int64_t* out) {
  if (k < 1 || k > n || n > 0xffffffffLL) return fail(OMF_EINVAL, "omf_topk_select_host: need 1 <= k <= n < 2^32");
  const Before before;
  if (k * 64 <= n) {
    AlignedEntries heap(k);
    if (!heap.data) return fail(OMF_ENOMEM, "omf_topk_select_host: heap allocation failed");
    Entry* h = heap.data;
    for (int64_t i = 0; i < k; ++i) h[i] = (Entry)mag_key_host(t[i]) << 32 | (uint32_t)i;
    std::make_heap(h, h + k, before);
    uint32_t top = (uint32_t)(h[0] >> 32);
    for (int64_t i = k; i < n; ++i) {
      const uint32_t key = mag_key_host(t[i]);
      if (key > top) {  // before(pair i, top): it replaces the top
        replace_top(h, k, (Entry)key << 32 | (uint32_t)i);
        top = (uint32_t)(h[0] >> 32);
      }
    }
    for (int64_t last = k - 1; last > 0; --last) {  // the heap sort: __pop_heap(h, h + last, h + last)
      const Entry v = h[last];
      h[last] = h[0];
      replace_top(h, last, v);
    }
    for (int64_t j = 0; j < k; ++j) out[j] = (int64_t)(uint32_t)h[j];
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
