// omf_qsgd.hip — QSGD encode / decode for the hybrid global hop, MI355X (gfx950).
//
// Semantics: SURVEY.md §8a "Exact QSGD semantics", restating
//   src/omnifed/hybrid/compression/qsgd.py:36-96 (reference, Python/torch CPU).
//
// Kernel map:
//   qsgd_encode_ordered  one launch for every tensor of a client.  Work items
//                        (64 KiB of fp32 each) are taken in ticket order:
//                        NORM(t) chunks publish fp64 partial sums of squares,
//                        the last arriver folds them in fixed order into
//                        norm[t] and publishes a {tag, norm} granule; QUANT(t)
//                        chunks wait on that granule and re-read x (served by
//                        the 256 MiB Infinity Cache: NORM(t+1) is the only
//                        traffic in between); tensors of <= 16 Ki elements are
//                        one FUSED item (norm + quantise from registers).
//   qsgd_quant_flat      norm supplied by the caller: one pass, no hand-off.
//   qsgd_decode_flat     y = (norm * q) / L, optionally accumulated (PS).
//
// HBM-bound; no MFMA (no contraction).  Coalesced 16 B/lane fp32 loads and stores,
// 4 B/lane int8 payload stores (one 256 B line per wave instruction).
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/omf_codec.h"
#include "omf_common.h"

using namespace omf;

namespace {

constexpr int kV = 16;                          // float4 per thread per sub-chunk
constexpr int64_t kSub = (int64_t)kV * kThreads * 4;  // 16384 elements = 64 KiB fp32
constexpr uint64_t kTimeoutTicks = 200000000ull;      // 2 s of the 100 MHz realtime clock

enum : int32_t { kNorm = 0, kQuant = 1, kFused = 2 };

struct Item {
  int64_t begin, end;  // arena element range of this work item
  int32_t tensor, kind, chunk, pad;
};

struct TensorInfo {
  int64_t begin, n;
  int32_t nchunks, pbase;
};

struct EncArgs {
  const float* x;
  const float* u;
  const float* norm_in;
  void* q;
  float* norm_out;
  const Item* items;
  const TensorInfo* tinfo;
  uint64_t* partials;  // fp64 bit patterns
  uint32_t* ticket;
  uint32_t* err;
  uint32_t* counters;
  uint64_t* gran;
  float alpha;
  float levels;  // 2^s as float (exact)
  uint32_t seed_lo, seed_hi, offset;
};

struct DecArgs {
  const void* q;
  const float* norm;
  float* y;
  const Item* items;
  float levels;      // fl32(levels)
  float inv_levels;  // 2^-s when levels is a power of two (exact), else unused
};

// ---------------------------------------------------------------- element math

// One QSGD level, qsgd.py:50-63.  xs / norm is IEEE division (hipcc default:
// correctly rounded); the remaining steps are exact in fp32.  Out-of-range or NaN
// magnitudes follow the reference's x86 float->int64 conversion (INT64_MIN, then
// clamp to 0): the payload element is 0.
__device__ __forceinline__ int32_t qsgd_level(float xs, float norm, float L, float u) {
  const float vn = xs / norm;
  const float a = fabsf(vn);
  const float sc = __fmul_rn(a, L);
  int32_t mag = 0;
  if (sc < 9.2233720e18f) {  // false for NaN / inf / >= 2^63
    const float fl = floorf(sc);
    const float p = __fsub_rn(sc, fl);
    float m = fl + ((u < p) ? 1.0f : 0.0f);  // exact: p > 0 implies fl < 2^23
    m = fminf(m, L);
    mag = (int32_t)m;
  }
  const int32_t sg = (vn > 0.0f) - (vn < 0.0f);
  return sg * mag;
}

template <int V>
__device__ __forceinline__ void load_f4(const float* __restrict__ p, int64_t b, int64_t end, float4 (&v)[V]) {
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
    if (e + 4 <= end) {
      v[k] = *reinterpret_cast<const float4*>(p + e);
    } else {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < end) t.x = p[e];
      if (e + 1 < end) t.y = p[e + 1];
      if (e + 2 < end) t.z = p[e + 2];
      v[k] = t;
    }
  }
}

template <int V>
__device__ __forceinline__ void scale_f4(float4 (&v)[V], float alpha) {
  if (alpha == 1.0f) return;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    v[k].x = __fmul_rn(v[k].x, alpha);
    v[k].y = __fmul_rn(v[k].y, alpha);
    v[k].z = __fmul_rn(v[k].z, alpha);
    v[k].w = __fmul_rn(v[k].w, alpha);
  }
}

template <int V>
__device__ __forceinline__ float sumsq_f4(const float4 (&v)[V], float acc) {
#pragma unroll
  for (int k = 0; k < V; ++k) {
    acc = fmaf(v[k].x, v[k].x, acc);
    acc = fmaf(v[k].y, v[k].y, acc);
    acc = fmaf(v[k].z, v[k].z, acc);
    acc = fmaf(v[k].w, v[k].w, acc);
  }
  return acc;
}

// Quantise V float4 of one sub-chunk starting at b (tensor t begins at tbegin) and store.
template <int WIDTH, bool HAS_U, int V>
__device__ __forceinline__ void quant_store(const float4 (&v)[V], const EncArgs& a, int64_t b, int64_t end,
                                            int64_t tbegin, int32_t tensor, float norm) {
  float4 uu[V];
  if (HAS_U) {
    load_f4<V>(a.u, b, end, uu);
  } else {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
      const uint64_t j = (uint64_t)(e - tbegin) >> 2;
      const uint4 r = philox4x32_10(make_uint4((uint32_t)j, (uint32_t)(j >> 32), (uint32_t)tensor, a.offset),
                                    a.seed_lo, a.seed_hi);
      uu[k] = make_float4(u24(r.x), u24(r.y), u24(r.z), u24(r.w));
    }
  }
  const bool zero = !(norm != 0.0f);  // norm == 0: all-zero payload (reference: dense passthrough)
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
    if (e >= end) continue;
    int32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    if (!zero) {
      q0 = qsgd_level(v[k].x, norm, a.levels, uu[k].x);
      q1 = qsgd_level(v[k].y, norm, a.levels, uu[k].y);
      q2 = qsgd_level(v[k].z, norm, a.levels, uu[k].z);
      q3 = qsgd_level(v[k].w, norm, a.levels, uu[k].w);
    }
    if (WIDTH == 1) {
      int8_t* q8 = reinterpret_cast<int8_t*>(a.q);
      if (e + 4 <= end) {
        const uint32_t packed = (uint32_t)(uint8_t)q0 | ((uint32_t)(uint8_t)q1 << 8) |
                                ((uint32_t)(uint8_t)q2 << 16) | ((uint32_t)(uint8_t)q3 << 24);
        *reinterpret_cast<uint32_t*>(q8 + e) = packed;
      } else {
        q8[e] = (int8_t)q0;
        if (e + 1 < end) q8[e + 1] = (int8_t)q1;
        if (e + 2 < end) q8[e + 2] = (int8_t)q2;
      }
    } else {
      int32_t* q32 = reinterpret_cast<int32_t*>(a.q);
      if (e + 4 <= end) {
        *reinterpret_cast<int4*>(q32 + e) = make_int4(q0, q1, q2, q3);
      } else {
        q32[e] = q0;
        if (e + 1 < end) q32[e + 1] = q1;
        if (e + 2 < end) q32[e + 2] = q2;
      }
    }
  }
}

__device__ __forceinline__ float wait_norm(const EncArgs& a, int32_t t) {
  const uint64_t t0 = wall_clock64();
  for (;;) {
    const uint64_t g = ld_agent(&a.gran[t]);
    if ((g >> 32) == 1u) return __uint_as_float((uint32_t)g);
    if (wall_clock64() - t0 > kTimeoutTicks) {
      __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return __uint_as_float(0x7fc00000u);
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// ---------------------------------------------------------------- kernels

template <int WIDTH, bool HAS_U, bool NORM_ONLY>
__global__ __launch_bounds__(kThreads) void qsgd_encode_ordered(EncArgs a) {
  __shared__ double s_red[kWaves];
  __shared__ uint32_t s_ticket;
  __shared__ uint32_t s_last;
  __shared__ float s_norm;
  const int tid = threadIdx.x;
  if (tid == 0) s_ticket = add_agent(a.ticket, 1u);
  __syncthreads();
  const Item it = a.items[s_ticket];
  const TensorInfo ti = a.tinfo[it.tensor];

  if (it.kind == kQuant) {
    if (NORM_ONLY) return;
    if (tid == 0) s_norm = wait_norm(a, it.tensor);
    __syncthreads();
    const float norm = s_norm;
    for (int64_t b = it.begin; b < it.end; b += kSub) {
      const int64_t e = min(b + kSub, it.end);
      float4 v[kV];
      load_f4<kV>(a.x, b, e, v);
      scale_f4<kV>(v, a.alpha);
      quant_store<WIDTH, HAS_U, kV>(v, a, b, e, ti.begin, it.tensor, norm);
    }
    return;
  }

  if (it.kind == kNorm) {
    float acc = 0.0f;
    for (int64_t b = it.begin; b < it.end; b += kSub) {
      const int64_t e = min(b + kSub, it.end);
      float4 v[kV];
      load_f4<kV>(a.x, b, e, v);
      scale_f4<kV>(v, a.alpha);
      acc = sumsq_f4<kV>(v, acc);
    }
    const double s = block_sum_f64((double)acc, s_red);
    if (tid == 0) {
      st_agent(&a.partials[ti.pbase + it.chunk], (uint64_t)__double_as_longlong(s));
      drain_vmem();  // partial globally visible before the arrival count
      const uint32_t old = add_agent(&a.counters[it.tensor], 1u);
      s_last = (old == (uint32_t)(ti.nchunks - 1)) ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
    // Last arriver: fold the partials in a fixed order (deterministic norm).
    double p = 0.0;
    for (int j = tid; j < ti.nchunks; j += kThreads) p += __longlong_as_double((long long)ld_agent(&a.partials[ti.pbase + j]));
    const double tot = block_sum_f64(p, s_red);
    if (tid == 0) {
      const float norm = sqrtf((float)tot);
      a.norm_out[it.tensor] = norm;
      st_agent(&a.gran[it.tensor], (1ull << 32) | (uint64_t)__float_as_uint(norm));
    }
    return;
  }

  // kFused: whole tensor (<= kSub elements) in registers.
  float4 v[kV];
  load_f4<kV>(a.x, it.begin, it.end, v);
  scale_f4<kV>(v, a.alpha);
  const double s = block_sum_f64((double)sumsq_f4<kV>(v, 0.0f), s_red);
  const float norm = sqrtf((float)s);
  if (tid == 0) a.norm_out[it.tensor] = norm;
  if (!NORM_ONLY) quant_store<WIDTH, HAS_U, kV>(v, a, it.begin, it.end, ti.begin, it.tensor, norm);
}

template <int WIDTH, bool HAS_U>
__global__ __launch_bounds__(kThreads) void qsgd_quant_flat(EncArgs a) {
  const Item it = a.items[blockIdx.x];
  const TensorInfo ti = a.tinfo[it.tensor];
  const float norm = a.norm_in[it.tensor];
  if (it.chunk == 0 && threadIdx.x == 0) a.norm_out[it.tensor] = norm;
  for (int64_t b = it.begin; b < it.end; b += kSub) {
    const int64_t e = min(b + kSub, it.end);
    float4 v[kV];
    load_f4<kV>(a.x, b, e, v);
    scale_f4<kV>(v, a.alpha);
    quant_store<WIDTH, HAS_U, kV>(v, a, b, e, ti.begin, it.tensor, norm);
  }
}

template <int WIDTH, bool ACC, bool POW2>
__global__ __launch_bounds__(kThreads) void qsgd_decode_flat(DecArgs a) {
  const Item it = a.items[blockIdx.x];
  const float norm = a.norm[it.tensor];
  for (int64_t b = it.begin; b < it.end; b += kSub) {
    const int64_t end = min(b + kSub, it.end);
    int32_t raw[kV][WIDTH == 1 ? 1 : 4];
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
      if (WIDTH == 1) {
        const int8_t* q8 = reinterpret_cast<const int8_t*>(a.q);
        if (e + 4 <= end) {
          raw[k][0] = *reinterpret_cast<const int32_t*>(q8 + e);
        } else {
          uint32_t t = 0;
          if (e < end) t |= (uint32_t)(uint8_t)q8[e];
          if (e + 1 < end) t |= (uint32_t)(uint8_t)q8[e + 1] << 8;
          if (e + 2 < end) t |= (uint32_t)(uint8_t)q8[e + 2] << 16;
          raw[k][0] = (int32_t)t;
        }
      } else {
        const int32_t* q32 = reinterpret_cast<const int32_t*>(a.q);
        if (e + 4 <= end) {
          const int4 t = *reinterpret_cast<const int4*>(q32 + e);
          raw[k][0] = t.x; raw[k][1] = t.y; raw[k][2] = t.z; raw[k][3] = t.w;
        } else {
          raw[k][0] = (e < end) ? q32[e] : 0;
          raw[k][1] = (e + 1 < end) ? q32[e + 1] : 0;
          raw[k][2] = (e + 2 < end) ? q32[e + 2] : 0;
          raw[k][3] = 0;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
      if (e >= end) continue;
      int32_t qi[4];
      if (WIDTH == 1) {
        qi[0] = (int32_t)(int8_t)(raw[k][0] & 0xff);
        qi[1] = (int32_t)(int8_t)((raw[k][0] >> 8) & 0xff);
        qi[2] = (int32_t)(int8_t)((raw[k][0] >> 16) & 0xff);
        qi[3] = (int32_t)(int8_t)((raw[k][0] >> 24) & 0xff);
      } else {
        qi[0] = raw[k][0]; qi[1] = raw[k][1]; qi[2] = raw[k][2]; qi[3] = raw[k][3];
      }
      // (norm * q) / 2^s == (norm * q) * 2^-s exactly (power-of-two scaling, both correctly rounded).
      float yv[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float nq = __fmul_rn(norm, (float)qi[c]);
        yv[c] = POW2 ? __fmul_rn(nq, a.inv_levels) : nq / a.levels;
      }
      float* y = a.y + e;
      if (e + 4 <= end) {
        float4 o = make_float4(yv[0], yv[1], yv[2], yv[3]);
        if (ACC) {
          const float4 prev = *reinterpret_cast<const float4*>(y);
          o.x = __fadd_rn(prev.x, o.x); o.y = __fadd_rn(prev.y, o.y);
          o.z = __fadd_rn(prev.z, o.z); o.w = __fadd_rn(prev.w, o.w);
        }
        *reinterpret_cast<float4*>(y) = o;
      } else {
#pragma unroll
        for (int c = 0; c < 3; ++c)
          if (e + c < end) y[c] = ACC ? __fadd_rn(y[c], yv[c]) : yv[c];
      }
    }
  }
}

__global__ __launch_bounds__(kThreads) void div_f32_kernel(float* __restrict__ y, int64_t n, float d) {
  const int64_t stride = (int64_t)gridDim.x * kThreads * 4;
  for (int64_t e = 4 * ((int64_t)blockIdx.x * kThreads + threadIdx.x); e < n; e += stride) {
    if (e + 4 <= n) {
      float4 v = *reinterpret_cast<float4*>(y + e);
      v.x = v.x / d; v.y = v.y / d; v.z = v.z / d; v.w = v.w / d;
      *reinterpret_cast<float4*>(y + e) = v;
    } else {
      for (int64_t i = e; i < n; ++i) y[i] = y[i] / d;
    }
  }
}

}  // namespace

// ====================================================================== host side

struct omf_plan {
  int device = 0;
  int32_t nt = 0;
  int64_t chunk = kSub;
  std::vector<int64_t> sizes, offsets;
  int64_t n_enc = 0, n_flat = 0, n_partials = 0;
  void* d_block = nullptr;  // one allocation: items, tensor info, partials, sync words
  Item* d_enc = nullptr;
  Item* d_flat = nullptr;
  TensorInfo* d_tinfo = nullptr;
  uint64_t* d_partials = nullptr;
  int64_t* d_sizes = nullptr;   // per-tensor element counts (Top-K)
  int64_t* d_begins = nullptr;  // per-tensor arena offsets (Top-K)
  int64_t arena_end = 0;
  uint8_t* d_sync = nullptr;  // [ticket u32, err u32, pad 8][counters u32 x nt, pad16][granules u64 x nt, pad16]
  size_t sync_bytes = 0, off_counters = 16, off_gran = 0;
};

// Plan internals shared with omf_topk.hip.
namespace omf_plan_access {
const void* flat_items(const omf_plan* p, int64_t* n) {
  *n = p->n_flat;
  return p->d_flat;
}
int32_t ntensors(const omf_plan* p) { return p->nt; }
int device(const omf_plan* p) { return p->device; }
int64_t arena_end(const omf_plan* p) { return p->arena_end; }
const int64_t* d_sizes(const omf_plan* p) { return p->d_sizes; }
const int64_t* d_begins(const omf_plan* p) { return p->d_begins; }
const std::vector<int64_t>& sizes(const omf_plan* p) { return p->sizes; }
}  // namespace omf_plan_access

static size_t round16(size_t b) { return (b + 15) & ~(size_t)15; }

static bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

extern "C" {

int omf_plan_create(const int64_t* sizes, const int64_t* offsets, int32_t ntensors, int64_t chunk_elems, int device,
                    omf_plan** out) {
  if (!out) return fail(OMF_EINVAL, "omf_plan_create: out is NULL");
  *out = nullptr;
  if (ntensors <= 0 || !sizes || !offsets) return fail(OMF_EINVAL, "omf_plan_create: need >= 1 tensor");
  if (chunk_elems == 0) chunk_elems = kSub;
  if (chunk_elems < kSub || chunk_elems % kSub != 0)
    return fail(OMF_EINVAL, "omf_plan_create: chunk_elems must be a positive multiple of 16384");
  auto* p = new (std::nothrow) omf_plan();
  if (!p) return fail(OMF_ENOMEM, "omf_plan_create: host allocation failed");
  p->device = device;
  p->nt = ntensors;
  p->chunk = chunk_elems;
  p->sizes.assign(sizes, sizes + ntensors);
  p->offsets.assign(offsets, offsets + ntensors);

  std::vector<TensorInfo> tinfo(ntensors);
  std::vector<Item> enc, flat;
  std::vector<std::vector<Item>> quant(ntensors);
  int64_t pbase = 0;
  for (int32_t t = 0; t < ntensors; ++t) {
    const int64_t n = sizes[t], b = offsets[t];
    if (n <= 0 || b < 0 || (b & 3)) {
      delete p;
      return fail(OMF_EINVAL, "omf_plan_create: tensor " + std::to_string(t) +
                                  ": size must be > 0 and offset a non-negative multiple of 4");
    }
    if (t > 0 && b < offsets[t - 1] + sizes[t - 1]) {
      delete p;
      return fail(OMF_EINVAL, "omf_plan_create: tensors must be ordered and non-overlapping");
    }
    TensorInfo ti{b, n, 0, (int32_t)pbase};
    if (n <= kSub) {
      ti.nchunks = 1;
      Item f{b, b + n, t, kFused, 0, 0};
      enc.push_back(f);
      flat.push_back(Item{b, b + n, t, kQuant, 0, 0});
    } else {
      const int64_t nc = (n + chunk_elems - 1) / chunk_elems;
      ti.nchunks = (int32_t)nc;
      pbase += nc;
      for (int64_t c = 0; c < nc; ++c) {
        const int64_t cb = b + c * chunk_elems, ce = std::min(b + n, cb + chunk_elems);
        enc.push_back(Item{cb, ce, t, kNorm, (int32_t)c, 0});
        quant[t].push_back(Item{cb, ce, t, kQuant, (int32_t)c, 0});
        flat.push_back(Item{cb, ce, t, kQuant, (int32_t)c, 0});
      }
    }
    tinfo[t] = ti;
    // QUANT(t-1) follows the producers of t: one tensor of slack for the norm hand-off.
    if (t >= 1) enc.insert(enc.end(), quant[t - 1].begin(), quant[t - 1].end());
  }
  enc.insert(enc.end(), quant[ntensors - 1].begin(), quant[ntensors - 1].end());
  p->n_enc = (int64_t)enc.size();
  p->n_flat = (int64_t)flat.size();
  p->n_partials = std::max<int64_t>(pbase, 1);
  if (p->n_enc > 0x7fffffffLL) {
    delete p;
    return fail(OMF_EINVAL, "omf_plan_create: too many work items");
  }

  p->off_counters = 16;
  p->off_gran = round16(p->off_counters + 4 * (size_t)ntensors);
  p->sync_bytes = round16(p->off_gran + 8 * (size_t)ntensors);
  // sync block first (its memset starts at the allocation start, multiple of 16 bytes)
  const size_t o_sync = 0;
  const size_t o_enc = round16(o_sync + p->sync_bytes);
  const size_t o_flat = round16(o_enc + sizeof(Item) * enc.size());
  const size_t o_tinfo = round16(o_flat + sizeof(Item) * flat.size());
  const size_t o_part = round16(o_tinfo + sizeof(TensorInfo) * tinfo.size());
  const size_t o_sizes = round16(o_part + 8 * (size_t)p->n_partials);
  const size_t o_begins = round16(o_sizes + 8 * (size_t)ntensors);
  const size_t total = round16(o_begins + 8 * (size_t)ntensors);
  p->arena_end = offsets[ntensors - 1] + sizes[ntensors - 1];

  DeviceGuard g(device);
  if (!g.ok) {
    delete p;
    return fail(OMF_EHIP, "omf_plan_create: hipSetDevice failed");
  }
  hipError_t e = hipMalloc(&p->d_block, total);
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "hipMalloc(plan)");
  }
  uint8_t* base = static_cast<uint8_t*>(p->d_block);
  p->d_sync = base + o_sync;
  p->d_enc = reinterpret_cast<Item*>(base + o_enc);
  p->d_flat = reinterpret_cast<Item*>(base + o_flat);
  p->d_tinfo = reinterpret_cast<TensorInfo*>(base + o_tinfo);
  p->d_partials = reinterpret_cast<uint64_t*>(base + o_part);
  p->d_sizes = reinterpret_cast<int64_t*>(base + o_sizes);
  p->d_begins = reinterpret_cast<int64_t*>(base + o_begins);
  e = hipMemcpy(p->d_enc, enc.data(), sizeof(Item) * enc.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_flat, flat.data(), sizeof(Item) * flat.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_tinfo, tinfo.data(), sizeof(TensorInfo) * tinfo.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_sizes, sizes, 8 * (size_t)ntensors, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_begins, offsets, 8 * (size_t)ntensors, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(p->d_sync, 0, p->sync_bytes);
  if (e != hipSuccess) {
    (void)hipFree(p->d_block);
    delete p;
    return hip_fail(e, "omf_plan_create: upload");
  }
  *out = p;
  return OMF_OK;
}

int omf_plan_destroy(omf_plan* plan) {
  if (!plan) return OMF_OK;
  DeviceGuard g(plan->device);
  if (plan->d_block) (void)hipFree(plan->d_block);
  delete plan;
  return OMF_OK;
}

int64_t omf_plan_encode_items(const omf_plan* plan) { return plan ? plan->n_enc : -1; }

int omf_plan_check(omf_plan* plan, void* stream) {
  if (!plan) return fail(OMF_EINVAL, "omf_plan_check: plan is NULL");
  DeviceGuard g(plan->device);
  OMF_HIP(hipStreamSynchronize((hipStream_t)stream));
  uint32_t err = 0;
  OMF_HIP(hipMemcpy(&err, plan->d_sync + 4, 4, hipMemcpyDeviceToHost));
  if (err) return fail(OMF_ETIMEOUT, "in-kernel norm hand-off timed out");
  return OMF_OK;
}

static int check_bits(int32_t s) {
  if (s < 0 || s > 30) return fail(OMF_EINVAL, "bit_width must be in [0, 30] (levels = 2^bit_width is an int32 on the wire)");
  return OMF_OK;
}

static int encode_impl(omf_plan* p, const float* x, float alpha, int32_t s, const float* u, uint64_t seed,
                       uint64_t offset, const float* norm_in, void* q, float* norm_out, bool norm_only, void* stream) {
  if (!p) return fail(OMF_EINVAL, "plan is NULL");
  if (int r = check_bits(s)) return r;
  const int width = (1 << s) <= 127 ? 1 : 4;
  if (!x || !norm_out || (!norm_only && !q)) return fail(OMF_EINVAL, "x, q and norm_out must be non-NULL");
  if (!aligned(x, 16) || (u && !aligned(u, 16)) || (q && !aligned(q, width == 1 ? 4 : 16)))
    return fail(OMF_EINVAL, "misaligned buffer (fp32/int32 need 16 B, int8 needs 4 B alignment)");
  DeviceGuard g(p->device);
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;
  EncArgs a;
  a.x = x; a.u = u; a.norm_in = norm_in; a.q = q; a.norm_out = norm_out;
  a.tinfo = p->d_tinfo;
  a.partials = p->d_partials;
  a.ticket = reinterpret_cast<uint32_t*>(p->d_sync);
  a.err = reinterpret_cast<uint32_t*>(p->d_sync + 4);
  a.counters = reinterpret_cast<uint32_t*>(p->d_sync + p->off_counters);
  a.gran = reinterpret_cast<uint64_t*>(p->d_sync + p->off_gran);
  a.alpha = alpha;
  a.levels = (float)(1u << s);
  a.seed_lo = (uint32_t)seed; a.seed_hi = (uint32_t)(seed >> 32); a.offset = (uint32_t)offset;
  const dim3 blk(kThreads);
  if (norm_in && !norm_only) {
    a.items = p->d_flat;
    const dim3 grid((unsigned)p->n_flat);
    if (width == 1) {
      if (u) hipLaunchKernelGGL((qsgd_quant_flat<1, true>), grid, blk, 0, st, a);
      else hipLaunchKernelGGL((qsgd_quant_flat<1, false>), grid, blk, 0, st, a);
    } else {
      if (u) hipLaunchKernelGGL((qsgd_quant_flat<4, true>), grid, blk, 0, st, a);
      else hipLaunchKernelGGL((qsgd_quant_flat<4, false>), grid, blk, 0, st, a);
    }
    OMF_HIP(hipGetLastError());
    return OMF_OK;
  }
  OMF_HIP(hipMemsetAsync(p->d_sync, 0, p->sync_bytes, st));
  a.items = p->d_enc;
  const dim3 grid((unsigned)p->n_enc);
  if (norm_only) {
    hipLaunchKernelGGL((qsgd_encode_ordered<1, false, true>), grid, blk, 0, st, a);
  } else if (width == 1) {
    if (u) hipLaunchKernelGGL((qsgd_encode_ordered<1, true, false>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((qsgd_encode_ordered<1, false, false>), grid, blk, 0, st, a);
  } else {
    if (u) hipLaunchKernelGGL((qsgd_encode_ordered<4, true, false>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((qsgd_encode_ordered<4, false, false>), grid, blk, 0, st, a);
  }
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

int omf_qsgd_encode(omf_plan* plan, const float* x, float alpha, int32_t bit_width, const float* u, uint64_t seed,
                    uint64_t offset, const float* norm_in, void* q_out, float* norm_out, void* stream) {
  return encode_impl(plan, x, alpha, bit_width, u, seed, offset, norm_in, q_out, norm_out, false, stream);
}

int omf_qsgd_norms(omf_plan* plan, const float* x, float alpha, float* norm_out, void* stream) {
  return encode_impl(plan, x, alpha, 0, nullptr, 0, 0, nullptr, nullptr, norm_out, true, stream);
}

int omf_qsgd_decode(omf_plan* p, const void* q, int32_t width, int32_t levels, const float* norm, float* y,
                    int32_t accumulate, void* stream) {
  if (!p) return fail(OMF_EINVAL, "plan is NULL");
  if (width != 8 && width != 32) return fail(OMF_EINVAL, "width must be 8 or 32");
  if (levels <= 0) return fail(OMF_EINVAL, "levels must be > 0");
  if (!q || !norm || !y) return fail(OMF_EINVAL, "q, norm and y_out must be non-NULL");
  if (!aligned(y, 16) || !aligned(q, width == 8 ? 4 : 16))
    return fail(OMF_EINVAL, "misaligned buffer (fp32/int32 need 16 B, int8 needs 4 B alignment)");
  DeviceGuard g(p->device);
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  DecArgs a;
  a.q = q; a.norm = norm; a.y = y; a.items = p->d_flat;
  a.levels = (float)levels;
  const bool pow2 = (levels & (levels - 1)) == 0;
  a.inv_levels = pow2 ? 1.0f / (float)levels : 0.0f;  // exact for a power of two
  const dim3 grid((unsigned)p->n_flat), blk(kThreads);
  hipStream_t st = (hipStream_t)stream;
#define OMF_DEC(W, A, P) hipLaunchKernelGGL((qsgd_decode_flat<W, A, P>), grid, blk, 0, st, a)
  if (width == 8) {
    if (accumulate) { if (pow2) OMF_DEC(1, true, true); else OMF_DEC(1, true, false); }
    else { if (pow2) OMF_DEC(1, false, true); else OMF_DEC(1, false, false); }
  } else {
    if (accumulate) { if (pow2) OMF_DEC(4, true, true); else OMF_DEC(4, true, false); }
    else { if (pow2) OMF_DEC(4, false, true); else OMF_DEC(4, false, false); }
  }
#undef OMF_DEC
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

int omf_div_f32(float* y, int64_t n, float divisor, void* stream) {
  if (n < 0 || (n > 0 && !y)) return fail(OMF_EINVAL, "omf_div_f32: bad arguments");
  if (n == 0) return OMF_OK;
  if (!aligned(y, 16)) return fail(OMF_EINVAL, "omf_div_f32: y must be 16-byte aligned");
  const int64_t blocks = std::min<int64_t>((n + 4 * kThreads - 1) / (4 * kThreads), 8192);
  hipLaunchKernelGGL(div_f32_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, y, n, divisor);
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

}  // extern "C"
