// omf_qsgd.hip — QSGD encode / decode for the hybrid global hop, MI355X (gfx950).
//
// Semantics: SURVEY.md §8a "Exact QSGD semantics", restating
//   src/omnifed/hybrid/compression/qsgd.py:36-96 (reference, Python/torch CPU).
//
// Kernel map:
//   qsgd_encode_ordered  one launch for every tensor of a client.  Work items are
//                        taken in ticket order (an atomic counter, so a workgroup
//                        only ever waits on items that are already running):
//                        RESIDENT(t)  16 Ki elements held in registers: publish the
//                                     fp64 partial sum of squares, wait for the
//                                     tensor norm, quantise from registers — x is
//                                     read once (tensors of <= cap/2 items);
//                        NORM(t)      chunk partial only (large tensors, pass 1);
//                        QUANT(t)     wait for the norm, re-read, quantise (pass 2).
//                        The last arriver of a tensor folds its partials in fixed
//                        order (deterministic norm) and publishes a {tag, norm}
//                        granule that the waiters poll.
//   qsgd_quant_sub       norm supplied by the caller: one pass, no hand-off.
//   qsgd_decode_flat     y = (norm * q) / L, optionally accumulated (PS).
//
// HBM-bound; no MFMA (no contraction).  Coalesced 16 B/lane fp32 loads, non-temporal
// 16 B/lane fp32 and 4 B/lane int8 payload stores.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/omf_codec.h"
#include "../../include/omf_codec_experimental.h"
#include "omf_common.h"
#include "omf_qsgd_dev.h"
#include "omf_ring.h"

using namespace omf;

namespace {

constexpr int kV = 16;                                // float4 per thread per sub-chunk
constexpr int64_t kSub = (int64_t)kV * kThreads * 4;  // 16384 elements = 64 KiB fp32
constexpr uint64_t kWaitTicks = 2000000ull;           // 20 ms of the 100 MHz realtime clock

enum : int32_t { kNorm = 0, kQuant = 1, kResident = 2 };

struct Item {
  int64_t begin, end;  // arena element range of this work item
  int32_t tensor, kind, chunk, pad;
};

struct TensorInfo {
  int64_t begin, n;
  int64_t chunk;          // elements per item of this tensor
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
  uint32_t fmt;  // value format (omf_qsgd_dev.h kFmt*)
  float levels;  // 2^s as float (exact)
  uint32_t seed_lo, seed_hi, offset;
  uint64_t wait_ticks;  // bounded norm wait (100 MHz ticks)
  uint32_t epoch;       // per-launch granule tag (never 0)
  uint32_t n_items;     // items of this launch (the last ticket resets the counter)
};

struct DecArgs {
  const void* q;
  const float* norm;
  float* y;
  const Item* items;
  float levels;      // fl32(levels)
  float inv_levels;  // 2^-s when levels is a power of two (exact), else unused
};

template <int V, bool FULL, bool NT = false>
__device__ __forceinline__ void load_f4(const float* __restrict__ p, int64_t b, int64_t end, float4 (&v)[V],
                                        int tid) {
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = b + 4 * ((int64_t)k * kThreads + tid);
    if (FULL || e + 4 <= end) {
      if (NT) {  // a last read (the second pass of a two-pass tensor)
        const f32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p + e));
        v[k] = make_float4(t[0], t[1], t[2], t[3]);
      } else {
        v[k] = *reinterpret_cast<const float4*>(p + e);
      }
    } else {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < end) t.x = p[e];
      if (e + 1 < end) t.y = p[e + 1];
      if (e + 2 < end) t.z = p[e + 2];
      v[k] = t;
    }
  }
}
template <int V, bool FULL, bool NT = false>
__device__ __forceinline__ void load_f4(const float* __restrict__ p, int64_t b, int64_t end, float4 (&v)[V]) {
  load_f4<V, FULL, NT>(p, b, end, v, (int)threadIdx.x);
}

// x * alpha (the client weighting), rounded to the value format for bf16/fp16 tensors
// (torch.mul on a reduced-precision tensor rounds its product; with alpha = 1 it is exact).
template <int V, class A>
__device__ __forceinline__ void scale_f4(float4 (&v)[V], const A& a) {
  const float alpha = a.alpha;
  if (alpha == 1.0f) return;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    v[k].x = __fmul_rn(v[k].x, alpha);
    v[k].y = __fmul_rn(v[k].y, alpha);
    v[k].z = __fmul_rn(v[k].z, alpha);
    v[k].w = __fmul_rn(v[k].w, alpha);
    if (a.fmt) v[k] = round_fmt4(v[k], a.fmt);
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

// Uniforms of rows k = 4g .. 4g+3 of this thread in a sub-chunk starting at b:
// 3 Philox calls per 16 elements (oracle/philox.py: group G, 96-bit slots).
__device__ __forceinline__ void philox_rows(const EncArgs& a, int64_t b, int64_t tbegin, int32_t tensor, int g,
                                            float4 (&uu)[4], int tid) {
  const uint64_t G = ((uint64_t)((b - tbegin) >> 12) + (uint64_t)g) * (uint64_t)kThreads + (uint32_t)tid;
  uint32_t w[12];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const uint64_t ctr = 3 * G + c;
    const uint4 r = philox4x32_10(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)tensor, a.offset),
                                  a.seed_lo, a.seed_hi);
    w[4 * c] = r.x; w[4 * c + 1] = r.y; w[4 * c + 2] = r.z; w[4 * c + 3] = r.w;
  }
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) uu[sl] = u24x4(w[3 * sl], w[3 * sl + 1], w[3 * sl + 2]);
}
__device__ __forceinline__ void philox_rows(const EncArgs& a, int64_t b, int64_t tbegin, int32_t tensor, int g,
                                            float4 (&uu)[4]) {
  philox_rows(a, b, tbegin, tensor, g, uu, (int)threadIdx.x);
}

// Quantise V float4 of one sub-chunk starting at b (tensor t begins at tbegin) and store.
// FULL: the sub-chunk is complete (no bounds checks).
template <int WIDTH, bool HAS_U, bool FULL, int V>
__device__ __forceinline__ void quant_store(const float4 (&v)[V], const EncArgs& a, int64_t b, int64_t end,
                                            int64_t tbegin, int32_t tensor, float norm) {
  static_assert(V % 4 == 0, "rows come in groups of 4 (RNG slots)");
  const bool zero = !(norm != 0.0f);  // norm == 0: all-zero payload (reference: dense passthrough)
  const Divisor dv(norm, a.fmt);
#pragma unroll
  for (int g = 0; g < V / 4; ++g) {
    float4 uu[4];
    if (HAS_U) {
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        const int64_t e = b + 4 * ((int64_t)(4 * g + sl) * kThreads + threadIdx.x);
        if (FULL || e + 4 <= end) {
          uu[sl] = *reinterpret_cast<const float4*>(a.u + e);
        } else {
          uu[sl] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (e < end) uu[sl].x = a.u[e];
          if (e + 1 < end) uu[sl].y = a.u[e + 1];
          if (e + 2 < end) uu[sl].z = a.u[e + 2];
        }
      }
    } else {
#ifdef OMF_EXP_NORNG  // experiment builds only: price the RNG
      for (int sl = 0; sl < 4; ++sl) uu[sl] = make_float4(0.5f, 0.25f, 0.75f, 0.125f);
#else
      philox_rows(a, b, tbegin, tensor, g, uu);
#endif
    }
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      const int k = 4 * g + sl;
      const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
      if (!FULL && e >= end) continue;
      int32_t qq[4];
      qsgd_quad(v[k], uu[sl], dv, a.levels, zero, qq);
      const int32_t q0 = qq[0], q1 = qq[1], q2 = qq[2], q3 = qq[3];
      if (WIDTH == 1) {
        int8_t* q8 = reinterpret_cast<int8_t*>(a.q);
        if (FULL || e + 4 <= end) {
          store_nt(reinterpret_cast<uint32_t*>(q8 + e), pack_i8x4(qq));
        } else {
          q8[e] = (int8_t)q0;
          if (e + 1 < end) q8[e + 1] = (int8_t)q1;
          if (e + 2 < end) q8[e + 2] = (int8_t)q2;
        }
      } else {
        int32_t* q32 = reinterpret_cast<int32_t*>(a.q);
        if (FULL || e + 4 <= end) {
          store_nt(q32 + e, make_int4(q0, q1, q2, q3));
        } else {
          q32[e] = q0;
          if (e + 1 < end) q32[e + 1] = q1;
          if (e + 2 < end) q32[e + 2] = q2;
        }
      }
    }
  }
}

// Load + scale + quantise + store one sub-chunk [b, e) of V rows (V * 1024 elements).
template <int WIDTH, bool HAS_U, int V = kV, bool NT = false>
__device__ __forceinline__ void quant_sub(const EncArgs& a, int64_t b, int64_t e, int64_t tbegin, int32_t tensor,
                                          float norm) {
  float4 v[V];
  if (e - b == (int64_t)V * 1024) {
    load_f4<V, true, NT>(a.x, b, e, v);
    scale_f4<V>(v, a);
    quant_store<WIDTH, HAS_U, true, V>(v, a, b, e, tbegin, tensor, norm);
  } else {
    load_f4<V, false, NT>(a.x, b, e, v);
    scale_f4<V>(v, a);
    quant_store<WIDTH, HAS_U, false, V>(v, a, b, e, tbegin, tensor, norm);
  }
}

// ---------------------------------------------------------------- norm hand-off

// Sum of squares of one item's range, exactly as a NORM item computes it: sub-chunks in
// order, each thread accumulating its own rows in fp32.
template <int V>
__device__ __forceinline__ float chunk_sumsq(const EncArgs& a, int64_t b, int64_t e) {
  constexpr int64_t S = (int64_t)V * 1024;
  float acc = 0.0f;
  for (int64_t sb = b; sb < e; sb += S) {
    const int64_t se = min(sb + S, e);
    float4 v[V];
    if (se - sb == S) load_f4<V, true>(a.x, sb, se, v);  // default policy: the QUANT re-read hits the Infinity Cache
    else load_f4<V, false>(a.x, sb, se, v);
    scale_f4<V>(v, a);
    acc = sumsq_f4<V>(v, acc);
  }
  return acc;
}

struct HandoffShared {
  double red[kWaves];
  uint32_t last, ok;
  float norm;
};

// Publish one item's partial; the last arriver of the tensor folds all partials in a fixed
// order (deterministic norm) and publishes the {tag = 1, norm} granule.  Protocol
// (cdna_hip_programming.md §6 G16): partial stored sc1 and drained before the
// agent-scope counter add; the last arriver reads the partials with sc1 loads.
__device__ __forceinline__ void publish_partial(const EncArgs& a, const TensorInfo& ti, int32_t t, int32_t idx,
                                                float acc, HandoffShared& sh) {
  const double s = block_sum_f64((double)acc, sh.red);
  if (threadIdx.x == 0) {
    st_agent(&a.partials[ti.pbase + idx], (uint64_t)__double_as_longlong(s));
    drain_vmem();
    const uint32_t old = add_agent(&a.counters[t], 1u);
    sh.last = (old == (uint32_t)(ti.nchunks - 1)) ? 1u : 0u;
    // Every partial of t has arrived: reset the counter for the next launch (stream order).
    if (sh.last) __hip_atomic_store(&a.counters[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (sh.last) {
    double p = 0.0;
    for (int j = threadIdx.x; j < ti.nchunks; j += kThreads)
      p += __longlong_as_double((long long)ld_agent(&a.partials[ti.pbase + j]));
    const double tot = block_sum_f64(p, sh.red);
    if (threadIdx.x == 0) {
      const float norm = finish_norm(tot, a.fmt);
      a.norm_out[t] = norm;
      st_agent(&a.gran[t], ((uint64_t)a.epoch << 32) | (uint64_t)__float_as_uint(norm));
    }
  }
}

// Poll the tensor's granule (one lane, relaxed sc1 loads, bounded).  On timeout (the
// tensor's items were not all co-resident) recompute every partial exactly as its owner
// does and fold them in the last arriver's order: identical bits, err bit 2 set.
template <int V>
__device__ __forceinline__ float norm_wait_or_recompute(const EncArgs& a, const TensorInfo& ti, int32_t t,
                                                        HandoffShared& sh) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = wall_clock64();
    uint32_t ok = 0;
    float nv = 0.0f;
    for (;;) {
      const uint64_t g = ld_agent(&a.gran[t]);
      if ((uint32_t)(g >> 32) == a.epoch) {
        nv = __uint_as_float((uint32_t)g);
        ok = 1;
        break;
      }
      if (wall_clock64() - t0 > a.wait_ticks) break;
      __builtin_amdgcn_s_sleep(1);
    }
    sh.norm = nv;
    sh.ok = ok;
  }
  __syncthreads();
  const float nv = sh.norm;
  const uint32_t ok = sh.ok;
  __syncthreads();
  if (ok) return nv;
  double p = 0.0;
  for (int j = 0; j < ti.nchunks; ++j) {
    const int64_t b = ti.begin + (int64_t)j * ti.chunk, e = min(b + ti.chunk, ti.begin + ti.n);
    const double sj = block_sum_f64((double)chunk_sumsq<V>(a, b, e), sh.red);
    if ((j % kThreads) == (int)threadIdx.x) p += sj;
  }
  const double tot = block_sum_f64(p, sh.red);
  if (threadIdx.x == 0) __hip_atomic_fetch_or(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return finish_norm(tot, a.fmt);
}

// ---------------------------------------------------------------- kernels

// EV: float4 rows per thread of one encode sub-chunk (EV * 1024 elements); RESIDENT items
// are one sub-chunk, NORM/QUANT items loop over the sub-chunks of their chunk.
template <int WIDTH, bool HAS_U, bool NORM_ONLY, int EV>
__global__ __launch_bounds__(kThreads) void qsgd_encode_ordered(EncArgs a) {
  constexpr int64_t ES = (int64_t)EV * 1024;
  __shared__ HandoffShared sh;
  __shared__ uint32_t s_ticket;
  if (threadIdx.x == 0) {
    const uint32_t tk = add_agent(a.ticket, 1u);
    // The last ticket of the launch: every workgroup has taken its ticket, reset for the next.
    if (tk == a.n_items - 1) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ticket = tk;
  }
  __syncthreads();
  const Item it = a.items[s_ticket];
  const TensorInfo ti = a.tinfo[it.tensor];

  if (it.kind == kResident) {  // one sub-chunk, x read once
    const bool full = (it.end - it.begin) == ES;
    float4 v[EV];
    if (full) load_f4<EV, true>(a.x, it.begin, it.end, v);
    else load_f4<EV, false>(a.x, it.begin, it.end, v);
    scale_f4<EV>(v, a);
    publish_partial(a, ti, it.tensor, it.chunk, sumsq_f4<EV>(v, 0.0f), sh);
    if (NORM_ONLY) return;
    const float norm = norm_wait_or_recompute<EV>(a, ti, it.tensor, sh);
    if (full) quant_store<WIDTH, HAS_U, true, EV>(v, a, it.begin, it.end, ti.begin, it.tensor, norm);
    else quant_store<WIDTH, HAS_U, false, EV>(v, a, it.begin, it.end, ti.begin, it.tensor, norm);
    return;
  }
  if (it.kind == kNorm) {
    publish_partial(a, ti, it.tensor, it.chunk, chunk_sumsq<EV>(a, it.begin, it.end), sh);
    return;
  }
  // kQuant: second pass of a large tensor.
  if (NORM_ONLY) return;
  const float norm = norm_wait_or_recompute<EV>(a, ti, it.tensor, sh);
  for (int64_t b = it.begin; b < it.end; b += ES)
    quant_sub<WIDTH, HAS_U, EV>(a, b, min(b + ES, it.end), ti.begin, it.tensor, norm);
}

template <int WIDTH, bool HAS_U, int V, bool NT>
__global__ __launch_bounds__(kThreads) void qsgd_quant_sub(EncArgs a) {
  // kSub / (V * 1024) blocks per 16 Ki item, V float4 per thread: 4 float4 (4 Ki-element
  // blocks) quantise 7 % faster than one 16 Ki block with 16 float4 per thread
  // (scripts/exp/ab_quant.py: 0.343 vs 0.368 ms on Llama-400M)
  constexpr int PER = (int)(kSub / ((int64_t)V * 1024));
  const Item it = a.items[blockIdx.x / PER];
  const int64_t b = it.begin + (int64_t)(blockIdx.x % PER) * V * 1024;
  if (b >= it.end) return;
  const TensorInfo ti = a.tinfo[it.tensor];
  const float norm = a.norm_in[it.tensor];
  if (it.chunk == 0 && blockIdx.x % PER == 0 && threadIdx.x == 0) a.norm_out[it.tensor] = norm;
  quant_sub<WIDTH, HAS_U, V, NT>(a, b, min(b + (int64_t)V * 1024, it.end), ti.begin, it.tensor, norm);
}

// ---------------------------------------------------------------- bracketed single-read encoder
//
// Strategy 3: x is read once without waiting for any norm.
//   qsgd_spec_bracket  one workgroup per tensor: a bracket [n_lo, n_hi] of its norm from a
//                      stratified sample (exact for small tensors) and the multipliers
//                      c_lo <= L / n_hi, c_hi >= L / n_lo (outward margins of 2^-20).
//   qsgd_spec_quant    one workgroup per 4 Ki-element block, no barrier: each wave's fp64
//                      partial sum of squares, and every element's level for ANY norm in the
//                      bracket: dl = fma(|x|, c_lo, -u), dh = fma(|x|, c_hi, -u); the level is
//                      ceil(dl) == ceil(dh) (clamped to L, sign of x) when they agree — the
//                      exact level is ceil(|RN(x/n)| L - u), monotone in n — else the quad is
//                      "undecided" and listed in the wave's slot (scripts/exp/spec_check.c
//                      checks the rule: 0 mismatches at brackets' end points and at decision
//                      points j + u; u == 0 with x != 0 is always undecided).
//   qsgd_spec_finish   its first workgroups fold the wave partials in segments (the last
//                      arriver folds the segments in order: the deterministic norm), check it
//                      lies in the bracket and publish {epoch, bad, norm}; the rest fix the
//                      listed quads exactly from their records (Markstein division, the shared
//                      element math), one thread per quad, polling their tensor's granule; a
//                      tensor whose norm fell outside its bracket, whose slots overflowed or
//                      whose sample was degenerate is requantised whole from x (the rare path).
// Payload bits equal every other strategy's for the same norm.
constexpr int kSpecV = 4;                                    // float4 rows per thread
constexpr int64_t kSpecBlk = (int64_t)kSpecV * kThreads * 4;  // 4096 elements per block
constexpr int kSpecSlot = 32;                                 // words per block: 4 waves x 7 quads (+ 4 spare)
constexpr int kSpecPerWave = 7;                               // listed quads per wave
// Wide levels (bit_width 5-8, fp32: the reference's default int32 wire at 8): the undecided fraction
// grows with L (a level step is norm / L wide), so a wave lists up to 32 quads (Llama-400M s = 8 with
// the sampled +-2.4 % brackets: ~10 per wave on its 1 Mi-element tensors, 2.1 M quads in all) and
// four fix threads share a wave slot.  Slots and records of this capacity are allocated at the
// plan's first wide encode.
constexpr int kSpecPerWaveWide = 32;
constexpr int kSpecMaxBitsWide = 8;
__host__ __device__ constexpr int spec_slot_words(int pw) { return pw == kSpecPerWave ? kSpecSlot : kWaves * pw; }
constexpr int64_t kSpecExact = 16384;                         // tensors read whole by the bracket
constexpr int kSpecRun = 64;                                  // elements per sampled run (256 B: DRAM-friendly)
constexpr int kSpecRuns = 512;                                // sampled runs per larger tensor (at most)
// wide levels: 4x the sampled elements (half the bracket width: the undecided quads, the fix pass's
// work, grow with L and with the bracket's width) in runs of 256 elements (1 KiB: four times fewer
// random DRAM accesses than 2 Ki runs of 64), kBrParts workgroups per tensor, 128 runs each
constexpr int kSpecRunWide = 256;
constexpr int kSpecRunsWide = 512;
#ifndef OMF_BR_PARTS  // experiment builds may override it (scripts/exp/s8_variants.sh)
#define OMF_BR_PARTS 2
#endif
constexpr int kBrParts = OMF_BR_PARTS;
constexpr int kSpecSeg = 4096;                                // wave partials per fold workgroup (16 loads per thread
                                                              // in flight: a 4 Mi-element tensor is one segment)
// Widest level count the bracket serves: the undecided fraction grows with L (a level step is
// norm / L wide), and at L = 32 a 1 Mi-element tensor's sampled bracket already leaves ~1.3
// undecided quads per wave; wider payloads take the two-pass encoder.
constexpr int kSpecMaxBits = 4;
constexpr int kSpecMinBits = 1;  // L >= 2 (spec_check.c's underflow argument)

struct SpecBracket {
  float c_lo, c_hi, n_lo, n_hi;
  uint32_t mode;  // 0 speculate, 1 deferred (degenerate sample: the fix pass requantises)
  uint32_t pad[3];
};

// Bracket work item: one per tensor, one workgroup each (qsgd_spec_bracket writes the
// tensor's bracket from that workgroup's sums alone; upload_plan builds exactly one).
struct SpecBrItem {
  int64_t begin, n;  // the tensor's arena range
  int64_t base;      // stratum length n / R (R = runs of the tensor); rem = n % R strata are one longer
  int32_t R, rem;
  int32_t tensor, Rw;  // Rw: the runs of kSpecRunWide sampled for wide levels (strata n / Rw)
};
// Fold work item: wave partials [p_begin, p_end) of tensor `tensor`, segment `seg` of `nsegs`.
struct SpecFoldItem {
  int64_t p_begin, p_end;
  int32_t tensor, seg, nsegs, sbase;
};

struct SpecArgs {
  EncArgs e;               // x, q, norm_out, items (flat 16 Ki items), alpha, levels, Philox key
  const int64_t* begins;   // per tensor
  const int64_t* sizes;
  const SpecBrItem* br_items;
  const SpecFoldItem* fold_items;
  SpecBracket* br;
  uint64_t* seg_part;      // per fold item: fp64 bits
  uint32_t* fold_cnt;      // per tensor arrival counters of the fold segments (reset by the last arriver)
  uint64_t* partials;      // fp64 bits, one per wave (kWaves per block)
  uint32_t* heads;         // per wave (dense, kWaves per block): (tensor << 8) | count of listed quads
  uint32_t* slots;         // spec_slot_words(PW) words per block: PW quad indices per wave
  float4* recs;            // per listed quad: its scaled x and its uniforms (2 float4), kWaves x PW per block
  uint32_t* flags;         // per tensor: a wave's slot overflowed (set by quant, cleared by fold)
  uint32_t* status;        // per tensor: 0 = listed quads only, 1 = requantise whole
  uint64_t* ngran;         // per tensor: {epoch << 1 | bad, norm} published by the fold
  uint64_t wait_ticks;     // bound of a fix thread's wait for its tensor's norm (100 MHz ticks)
  uint32_t dbg;            // test / experiment switches (omf_plan_set_debug spec bits 2-4), 0 in production
  float divisor;           // fused PS step: x := x / divisor (IEEE), written to xout; 0 = none
  float zsig;              // bracket half-width in standard deviations of the sample estimate (6)
  float* xout;
  uint32_t epoch;          // per-launch tag (never 0)
  uint32_t wide;           // wide levels: the bracket samples Rw runs (SpecBrItem), kBrParts workgroups per tensor
  double* br_part;         // wide / fused bracket: per (tensor, part) the partial {S1, S2}
  uint64_t* brgran;        // fused bracket: per tensor {epoch, c_lo} and {epoch, c_hi}
  uint32_t* br_cnt;        // wide: per tensor arrival counter (reset by the last arriver)
  int64_t nblocks;
  // Fused last-client decode-accumulate (omf_ps_accumulate_apply_encode; aq == NULL: none): before
  // the divide, x := fl32(x + fl32(fl32(anorm[t] * q) / alevels)) — the decoder's accumulate, bit
  // for bit (ainv = 2^-s for a power-of-two level count, else 0) — stored to aout when non-NULL.
  const void* aq;
  const float* anorm;
  float* aout;
  float alevels, ainv;
  int32_t awidth;          // 8 or 32: the last client's payload (LayerState.width)
};

// The last client's payload of one float4 row (AW = 1: int8, AW = 4: int32), loaded beside x.
template <int AW, bool FULL>
__device__ __forceinline__ int4 acc_load(const void* q, int64_t e, int64_t end) {
  if (AW == 1) {
    const int8_t* q8 = static_cast<const int8_t*>(q);
    if (FULL || e + 4 <= end)
      return make_int4(__builtin_nontemporal_load(reinterpret_cast<const int32_t*>(q8 + e)), 0, 0, 0);
    uint32_t w = 0;
    for (int c = 0; c < 3; ++c)
      if (e + c < end) w |= (uint32_t)(uint8_t)q8[e + c] << (8 * c);
    return make_int4((int32_t)w, 0, 0, 0);
  }
  const int32_t* q32 = static_cast<const int32_t*>(q);
  if (FULL || e + 4 <= end) {
    const i32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t*>(q32 + e));
    return make_int4(t[0], t[1], t[2], t[3]);
  }
  int4 r = make_int4(0, 0, 0, 0);
  if (e < end) r.x = q32[e];
  if (e + 1 < end) r.y = q32[e + 1];
  if (e + 2 < end) r.z = q32[e + 2];
  return r;
}

// v + decode(raw): the decoder's arithmetic (qsgd_decode_arena with accumulate).
template <int AW>
__device__ __forceinline__ float4 acc_add4(float4 v, int4 raw, float norm, float alevels, float ainv) {
  int32_t qi[4];
  if (AW == 1) {
    qi[0] = (int32_t)(int8_t)(raw.x & 0xff);
    qi[1] = (int32_t)(int8_t)((raw.x >> 8) & 0xff);
    qi[2] = (int32_t)(int8_t)((raw.x >> 16) & 0xff);
    qi[3] = (int32_t)(int8_t)((raw.x >> 24) & 0xff);
  } else {
    qi[0] = raw.x; qi[1] = raw.y; qi[2] = raw.z; qi[3] = raw.w;
  }
  float y[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float nq = __fmul_rn(norm, (float)qi[c]);
    y[c] = ainv != 0.0f ? __fmul_rn(nq, ainv) : nq / alevels;
  }
  return make_float4(__fadd_rn(v.x, y[0]), __fadd_rn(v.y, y[1]), __fadd_rn(v.z, y[2]), __fadd_rn(v.w, y[3]));
}

// The bracket's view of one float4 of x at arena element e: x (+ the fused last client's decode).
__device__ __forceinline__ float4 br_value(const SpecArgs& a, float4 v, int64_t e, int64_t end, int32_t t) {
  if (!a.aq) return v;
  const float nrm = a.anorm[t];
  if (a.awidth == 32) return acc_add4<4>(v, acc_load<4, false>(a.aq, e, end), nrm, a.alevels, a.ainv);
  return acc_add4<1>(v, acc_load<1, false>(a.aq, e, end), nrm, a.alevels, a.ainv);
}

__device__ __forceinline__ uint32_t spec_hash(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}

__device__ __forceinline__ float4 scale_alpha(float4 v, float alpha) {
  if (alpha != 1.0f) {
    v.x = __fmul_rn(v.x, alpha); v.y = __fmul_rn(v.y, alpha);
    v.z = __fmul_rn(v.z, alpha); v.w = __fmul_rn(v.w, alpha);
  }
  return v;
}

// x * alpha (rounded to the value format when alpha != 1: torch.mul on a bf16 / fp16 tensor),
// then / divisor for the fused PS step (divisor 0: none) — the pass's arithmetic.
__device__ __forceinline__ float4 spec_prologue(float4 v, float alpha, float divisor, uint32_t fmt) {
  v = scale_alpha(v, alpha);
  if (fmt && alpha != 1.0f) v = round_fmt4(v, fmt);
  if (divisor != 0.0f) {
    v.x = __fdiv_rn(v.x, divisor); v.y = __fdiv_rn(v.y, divisor);
    v.z = __fdiv_rn(v.z, divisor); v.w = __fdiv_rn(v.w, divisor);
  }
  return v;
}

__device__ __forceinline__ float sq4(float4 v, float s) {
  s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s);
  s = fmaf(v.z, v.z, s); return fmaf(v.w, v.w, s);
}

constexpr int kBrThreads = 1024;  // one bracket workgroup per tensor
constexpr int kBrWaves = kBrThreads / 64;

// Deterministic sum over a 1024-thread workgroup (wave butterflies, then the waves in order).
__device__ __forceinline__ double br_sum(double v, double* lds) {
  v = wave_sum_f64(v);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kBrWaves; ++w) s += lds[w];
  __syncthreads();
  return s;
}

// The bracket's sample of one tensor: runs of RUN elements at a hashed position inside each of R
// balanced strata (of >= 2 RUN elements); a run is RUN / 4 float4 loaded by consecutive lanes, 8
// passes per round (their loads in flight together); this workgroup takes the rounds part, part +
// parts, ...  Per run: s1 += its sum of squares, s2 += its square (in lane 0 of the run).
template <int RUN, bool AQ, int NT = kBrThreads, int PASSES = 8>
__device__ __forceinline__ void bracket_sample(const SpecArgs& a, const float* __restrict__ x, int32_t t, int64_t tb,
                                               int64_t n, int64_t R, int part, int parts, double& s1, double& s2) {
  constexpr int LPR = RUN / 4, RPP = NT / LPR, PER_ROUND = RPP * PASSES;
  const int64_t base = n / R, rem = n % R;
  const int j = threadIdx.x & (LPR - 1);
  const float alpha = a.e.alpha;
  for (int64_t rb = (int64_t)part * PER_ROUND; rb < R; rb += (int64_t)parts * PER_ROUND) {
    float4 v[PASSES];
    bool live[PASSES];
    auto run_pos = [&](int i) {  // element of this lane's float4 in pass i (recomputed: no VGPRs held)
      const int64_t r0 = rb + (int64_t)i * RPP + (threadIdx.x / LPR);
      const int64_t r = r0 < R ? r0 : 0;  // a dead lane re-reads run 0 (masked below)
      const int64_t lo = r * base + min(r, rem), len = base + (r < rem ? 1 : 0);
      return ((lo + (int64_t)(spec_hash((uint32_t)r, (uint32_t)t) % (uint32_t)(len - (RUN - 1)))) & ~(int64_t)3) + 4 * j;
    };
#pragma unroll
    for (int i = 0; i < PASSES; ++i) {
      live[i] = rb + (int64_t)i * RPP + (threadIdx.x / LPR) < R;
      v[i] = *reinterpret_cast<const float4*>(x + run_pos(i));
    }
    if (AQ) {  // the fused PS step's last client (after every x load is issued)
#pragma unroll
      for (int i = 0; i < PASSES; ++i) v[i] = br_value(a, v[i], tb + run_pos(i), tb + n, t);
    }
#pragma unroll
    for (int i = 0; i < PASSES; ++i) {
      float sr = live[i] ? sq4(spec_prologue(v[i], alpha, a.divisor, a.e.fmt), 0.0f) : 0.0f;
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) sr += __shfl_xor(sr, o, LPR);  // the run's sum in every lane
      if (live[i] && j == 0) {
        s1 += (double)sr;
        s2 += (double)sr * (double)sr;
      }
    }
  }
}

// WIDE: kBrParts workgroups per tensor, runs of kSpecRunWide (bit widths 5-8); AQ: the fused PS
// step's last client is added to the sample (narrow only).  One instance per case keeps each small
// enough for two 1024-thread workgroups per CU (one kernel for all three took 94 VGPRs).
__device__ SpecBracket bracket_from_sums(const SpecArgs& a, bool exact, int64_t n, int64_t R, int run, double S1,
                                         double S2);

template <bool WIDE, bool AQ>
__device__ __forceinline__ void spec_bracket_body(const SpecArgs& a, const SpecBrItem* __restrict__ items,
                                                  double* red, uint32_t& s_last) {
  // wide levels: kBrParts workgroups per tensor, part g sampling runs [g kSpecRuns, (g + 1) kSpecRuns)
  const int parts = WIDE ? kBrParts : 1;
  const int part = (int)(blockIdx.x % (unsigned)parts);
  const SpecBrItem bi = items[blockIdx.x / (unsigned)parts];  // one scalar load: the tensor's range and strata
  const int32_t t = bi.tensor;
  const int64_t tb = bi.begin, n = bi.n;
  const float* __restrict__ x = a.e.x + tb;
  const float alpha = a.e.alpha;
  double s1 = 0.0, s2 = 0.0;
  const bool exact = n <= kSpecExact;
  const int64_t R = WIDE ? (int64_t)bi.Rw : (int64_t)bi.R;
  // Loads are unconditional (a clamped address, the value masked after): a load under a
  // branch is waited for at the branch's end, which would serialise the round trips.
  if (exact) {  // 4 float4 per thread, all loads in flight
    constexpr int PER = (int)(kSpecExact / (4 * kBrThreads));
    float4 v[PER];
    const int64_t nq = n & ~(int64_t)3;  // whole quads
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int64_t e = 4 * ((int64_t)i * kBrThreads + threadIdx.x);
      v[i] = nq ? *reinterpret_cast<const float4*>(x + (e < nq ? e : 0)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int64_t e = 4 * ((int64_t)i * kBrThreads + threadIdx.x);
      if (e >= nq) {
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < n) {  // the tensor's partial last quad (one thread)
          v[i].x = x[e];
          if (e + 1 < n) v[i].y = x[e + 1];
          if (e + 2 < n) v[i].z = x[e + 2];
        }
      }
    }
    if (AQ) {  // the fused PS step's last client, added before the divide
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int64_t e = 4 * ((int64_t)i * kBrThreads + threadIdx.x);
        if (e < n) v[i] = br_value(a, v[i], tb + e, tb + n, t);
      }
    }
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < PER; ++i) acc = sq4(spec_prologue(v[i], alpha, a.divisor, a.e.fmt), acc);
    s1 = acc;
  } else {
    bracket_sample<WIDE ? kSpecRunWide : kSpecRun, AQ>(a, x, t, tb, n, R, part, parts, s1, s2);
  }
  if (exact && part != 0) return;  // an exact tensor is one workgroup's
  double S1 = br_sum(s1, red);
  double S2 = br_sum(s2, red);
  if (!exact && parts > 1) {  // the last part to arrive combines the partials in part order
    if (threadIdx.x == 0) {
      double* bp = a.br_part + 2 * ((int64_t)t * parts + part);
      st_agent(reinterpret_cast<uint64_t*>(bp), (uint64_t)__double_as_longlong(S1));
      st_agent(reinterpret_cast<uint64_t*>(bp + 1), (uint64_t)__double_as_longlong(S2));
      drain_vmem();
      const uint32_t last = add_agent(&a.br_cnt[t], 1u) == (uint32_t)(parts - 1) ? 1u : 0u;
      if (last) __hip_atomic_store(&a.br_cnt[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
    S1 = S2 = 0.0;
    for (int g = 0; g < parts; ++g) {
      const uint64_t* bp = reinterpret_cast<const uint64_t*>(a.br_part + 2 * ((int64_t)t * parts + g));
      S1 += __longlong_as_double((long long)ld_agent(bp));
      S2 += __longlong_as_double((long long)ld_agent(bp + 1));
    }
  }
  if (threadIdx.x != 0) return;
  a.br[t] = bracket_from_sums(a, exact, n, R, WIDE ? kSpecRunWide : kSpecRun, S1, S2);
}

// The bracket of a tensor from its sample's sums (exact: S1 is the whole tensor's sum of squares).
__device__ SpecBracket bracket_from_sums(const SpecArgs& a, bool exact, int64_t n, int64_t R, int run, double S1,
                                         double S2) {
  double ss, k;
  if (exact) {
    ss = S1;
    k = 0x1p-12;  // fp32 per-thread accumulation differs from the fold's grouping
  } else {
    const double Rd = (double)R, m = S1 / Rd;
    const double var = fmax(0.0, (S2 - Rd * m * m) / (Rd - 1.0));
    ss = S1 * ((double)n / ((double)run * Rd));
    k = (double)a.zsig * sqrt(var / Rd) / m + 0x1p-10;  // 6 sigma of the run-sum estimate + 0.1 %
  }
  // bf16 / fp16 values: the norm is rounded to the format (at most half an ulp: 2^-8 / 2^-11
  // relative, so (1 + 2^-8)^2 < 1 + 2^-7 + 2^-14 on its square), and so is x / n, whose
  // rounding the multipliers absorb by the same relative bound (spec_quad_fmt).
  const uint32_t fmt = a.e.fmt;
  const double kf = fmt == kFmtBF16 ? 0x1p-7 + 0x1p-14 : (fmt == kFmtF16 ? 0x1p-10 + 0x1p-20 : 0.0);
  const double mf = fmt == kFmtBF16 ? 0x1p-8 + 0x1p-16 : (fmt == kFmtF16 ? 0x1p-11 + 0x1p-22 : 0.0);
  k += kf;
  SpecBracket o{0.f, 0.f, 0.f, 0.f, 1u, {0u, 0u, 0u}};  // deferred: c = 0 decides every level as 0
  if (ss > 0.0 && ss < 1e300 && k < 0.5) {
    const float n_lo = nextafterf((float)sqrt(ss * (1.0 - k)), 0.0f);
    const float n_hi = nextafterf((float)sqrt(ss * (1.0 + k)), INFINITY);
    if (n_lo >= 0x1p-90f && n_hi < INFINITY) {  // c_hi finite for L <= 2^30
      const double L = (double)a.e.levels;
      o.n_lo = n_lo;
      o.n_hi = n_hi;
      o.c_lo = nextafterf((float)(L / (double)n_hi * (1.0 - 0x1p-20) * (1.0 - mf)), 0.0f);
      o.c_hi = nextafterf((float)(L / (double)n_lo * (1.0 + 0x1p-20) * (1.0 + mf)), INFINITY);
      o.mode = 0u;
    }
  }
  return o;
}

template <bool WIDE, bool AQ>
__global__ __launch_bounds__(kBrThreads) void qsgd_spec_bracket(SpecArgs a, const SpecBrItem* __restrict__ items) {
  __shared__ double red[kBrWaves];
  __shared__ uint32_t s_last;
  spec_bracket_body<WIDE, AQ>(a, items, red, s_last);
}
// wide levels: two 1024-thread workgroups per CU (<= 64 VGPRs), so the kBrParts workgroups per
// tensor run in one generation
__global__ __launch_bounds__(kBrThreads) __attribute__((amdgpu_waves_per_eu(8))) void qsgd_spec_bracket_wide(
    SpecArgs a, const SpecBrItem* __restrict__ items) {
  __shared__ double red[kBrWaves];
  __shared__ uint32_t s_last;
  spec_bracket_body<true, false>(a, items, red, s_last);
}

// Levels of a quad for every norm of the bracket; und: some element is undecided.  u == 0 is
// raised to 2^-26 in the lower product only (x / n may underflow to 0 where |x| c does not:
// such an element is left undecided); a decided level needs no clamp (ceil(dl) <= the exact
// level <= L); NaN gives kl != kh.  scripts/exp/spec_check.c checks this exact form.
__device__ __forceinline__ void spec_quad(float4 x, float4 u, float c_lo, float c_hi, int32_t (&q)[4], bool& und) {
  const float xs[4] = {x.x, x.y, x.z, x.w}, us[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float ax = fabsf(xs[c]);
    const float kl = ceilf(fmaf(ax, c_lo, -fmaxf(us[c], 0x1p-26f)));
    const float kh = ceilf(fmaf(ax, c_hi, -us[c]));
    und |= kl != kh;
    q[c] = (int32_t)copysignf(kh, xs[c]);
  }
}

// The same for bf16 / fp16 values (vn = x / n rounded to the format, a = |vn| L): the bracket's
// multipliers carry the format's relative rounding bound (qsgd_spec_bracket), and fp16's
// subnormal quotients (|vn| < 2^-14: an absolute step of 2^-24, i.e. at most 2^-25 L on a) take
// an absolute slack `dl` on both sides (u + dl is exact: u is a multiple of 2^-24 below 1).
// Every level between the two bounds' is then the level for some norm of the bracket, so
// kl == kh decides it; bf16 subnormals (|vn| < 2^-126) fall under the u == 0
// rule as in fp32.
__device__ __forceinline__ void spec_quad_fmt(float4 x, float4 u, float c_lo, float c_hi, float dl, int32_t (&q)[4],
                                              bool& und) {
  const float xs[4] = {x.x, x.y, x.z, x.w}, us[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float ax = fabsf(xs[c]);
    const float kl = ceilf(fmaf(ax, c_lo, -(fmaxf(us[c], 0x1p-26f) + dl)));
    const float kh = ceilf(fmaf(ax, c_hi, dl - us[c]));
    und |= kl != kh;
    q[c] = (int32_t)copysignf(kh, xs[c]);
  }
}

template <int WIDTH>
__device__ __forceinline__ void store_quad(const EncArgs& a, int64_t e, int64_t end, const int32_t (&qq)[4]) {
  if (WIDTH == 1) {
    int8_t* q8 = reinterpret_cast<int8_t*>(a.q);
    if (e + 4 <= end) {
      store_nt(reinterpret_cast<uint32_t*>(q8 + e), pack_i8x4(qq));
    } else {
      q8[e] = (int8_t)qq[0];
      if (e + 1 < end) q8[e + 1] = (int8_t)qq[1];
      if (e + 2 < end) q8[e + 2] = (int8_t)qq[2];
    }
  } else {
    int32_t* q32 = reinterpret_cast<int32_t*>(a.q);
    if (e + 4 <= end) {
      store_nt(q32 + e, make_int4(qq[0], qq[1], qq[2], qq[3]));
    } else {
      q32[e] = qq[0];
      if (e + 1 < end) q32[e + 1] = qq[1];
      if (e + 2 < end) q32[e + 2] = qq[2];
    }
  }
}

// One block's pass: loads issued first, the Philox draws (independent of x) computed while
// they are in flight, then the partial, the levels and the undecided list.  FULL: a whole
// 4 Ki block (straight-line code, no bounds checks).
template <int WIDTH, bool FULL, bool DIV, uint32_t FMT, int AW = 0, int PW = kSpecPerWave, class GetBr>
__device__ __forceinline__ void spec_block(const SpecArgs& a, int64_t blk, int64_t b, int64_t end, int32_t t,
                                           int64_t tb, GetBr get_br, uint32_t* slot, uint64_t* part, float anorm,
                                           int tid) {
  const EncArgs& e = a.e;
  const int lane = tid & 63, wave = tid >> 6;
  float4 v[kSpecV];
  load_f4<kSpecV, FULL, true>(e.x, b, end, v, tid);  // x is read once: nontemporal (the fix uses the records)
  int4 araw[AW ? kSpecV : 1];
  if (AW) {  // the fused PS step's last client: its payload loaded beside x
#pragma unroll
    for (int k = 0; k < kSpecV; ++k)
      araw[k] = acc_load<AW ? AW : 1, FULL>(a.aq, b + 4 * ((int64_t)k * kThreads + tid), end);
  }
  float4 uu[4];
  philox_rows(e, b, tb, t, 0, uu, tid);
  // Branch-free from the loads to the stores, so that the scheduler can place the Philox
  // arithmetic under the load latency: x * alpha unconditionally (x * 1 = x; fp32 only, the
  // product is not rounded further), and levels computed for a deferred tensor too (its
  // multipliers are 0: every level 0, none undecided; the fix pass requantises it).
  const float alpha = e.alpha;
  float acc = 0.0f;
#pragma unroll
  for (int k = 0; k < kSpecV; ++k) {
    v[k].x = __fmul_rn(v[k].x, alpha); v[k].y = __fmul_rn(v[k].y, alpha);
    v[k].z = __fmul_rn(v[k].z, alpha); v[k].w = __fmul_rn(v[k].w, alpha);
    if (FMT != kFmtF32 && alpha != 1.0f) v[k] = round_fmt4(v[k], FMT);  // torch.mul on the half tensor
    if (AW) {  // acc + decode(last client), stored when the caller keeps the accumulator
      v[k] = acc_add4<AW ? AW : 1>(v[k], araw[k], anorm, a.alevels, a.ainv);
      if (a.aout) {
        const int64_t el = b + 4 * ((int64_t)k * kThreads + tid);
        if (FULL || el + 4 <= end) {
          store_nt(a.aout + el, v[k]);
        } else if (el < end) {
          a.aout[el] = v[k].x;
          if (el + 1 < end) a.aout[el + 1] = v[k].y;
          if (el + 2 < end) a.aout[el + 2] = v[k].z;
        }
      }
    }
    if (DIV) {  // fused PS step: the average, stored once (nontemporal) and quantised from registers
      const float d = a.divisor;
      v[k].x = __fdiv_rn(v[k].x, d); v[k].y = __fdiv_rn(v[k].y, d);
      v[k].z = __fdiv_rn(v[k].z, d); v[k].w = __fdiv_rn(v[k].w, d);
      const int64_t el = b + 4 * ((int64_t)k * kThreads + tid);
      if (FULL || el + 4 <= end) {
        store_nt(a.xout + el, v[k]);
      } else if (el < end) {
        a.xout[el] = v[k].x;
        if (el + 1 < end) a.xout[el + 1] = v[k].y;
        if (el + 2 < end) a.xout[el + 2] = v[k].z;
      }
    }
    acc = sq4(v[k], acc);
  }
  const SpecBracket br = get_br();  // (the fused-bracket pass polls for it here, its loads in flight)
  uint32_t cnt = 0;  // wave-uniform
  {
    uint32_t* list = slot + PW * wave;
#pragma unroll
    for (int k = 0; k < kSpecV; ++k) {
      const int64_t el = b + 4 * ((int64_t)k * kThreads + tid);
      const bool live = FULL || el < end;
      int32_t qq[4];
      bool und = false;
      if (FMT == kFmtF32) spec_quad(v[k], uu[k], br.c_lo, br.c_hi, qq, und);
      else spec_quad_fmt(v[k], uu[k], br.c_lo, br.c_hi, FMT == kFmtF16 ? 0x1p-25f * e.levels : 0.0f, qq, und);
      if (live) store_quad<WIDTH>(e, el, FULL ? el + 4 : end, qq);
      const uint64_t m = __ballot(live && und);
      if (m) {  // rare: list this wave's undecided quads
        const uint32_t pos = cnt + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (live && und && pos < (uint32_t)PW) {  // the quad, its x and its draws: no re-read
          list[pos] = (uint32_t)(el >> 2);
          float4* rec = a.recs + 2 * ((blk * kWaves + wave) * PW + pos);
          rec[0] = v[k];
          rec[1] = uu[k];
        }
        cnt += (uint32_t)__popcll(m);
      }
    }
  }
  const double s = wave_sum_f64((double)acc);
  if (lane == 0) {
    *part = (uint64_t)__double_as_longlong(s);
    a.heads[blk * kWaves + wave] = ((uint32_t)t << 8) | min(cnt, (uint32_t)PW);
    if (cnt > (uint32_t)PW)
      __hip_atomic_fetch_or(&a.flags[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The per-tensor tables are __restrict__ const kernel arguments so that they are read with
// scalar loads (a vector load there is waited for before the x loads are issued).
// WPB: waves per workgroup.  A 4 Ki-element block's waves keep their element map (thread t of the
// block owns rows b + 4 (k 256 + t)), partials, heads and lists whatever the workgroup size; wide
// levels run one wave per workgroup (scripts/exp/dec_shapes.hip, the int32 pass's shape: 0.508
// against 0.534 ms for four waves).
template <int WIDTH, bool DIV, uint32_t FMT = kFmtF32, int AW = 0, int PW = kSpecPerWave, int WPB = kWaves>
__global__ __launch_bounds__(64 * WPB) void qsgd_spec_quant(SpecArgs a, const SpecBracket* __restrict__ brs,
                                                            const int64_t* __restrict__ begins,
                                                            const float* __restrict__ anorms) {
  static_assert(kWaves % WPB == 0, "a block's waves split evenly");
  constexpr int kPer = kWaves / WPB;  // workgroups per 4 Ki block
  const int64_t blk = blockIdx.x / kPer;
  const int tid = (int)(blockIdx.x % kPer) * 64 * WPB + (int)threadIdx.x;
  const Item it = a.e.items[blk >> 2];
  const SpecBracket br = brs[it.tensor];
  const int64_t tb = begins[it.tensor];
  const float anorm = AW ? anorms[it.tensor] : 0.0f;
  const int64_t b = it.begin + (blk & 3) * kSpecBlk;
  const int wave = tid >> 6;
  uint32_t* slot = a.slots + blk * spec_slot_words(PW);
  uint64_t* part = a.partials + blk * kWaves + wave;
  if (b >= it.end) {  // past the tensor's end: an empty block still reports (stale values otherwise)
    if ((tid & 63) == 0) {
      *part = 0ull;
      a.heads[blk * kWaves + wave] = (uint32_t)it.tensor << 8;
    }
    return;
  }
  const int64_t end = min(b + kSpecBlk, it.end);
  auto get_br = [&]() { return br; };
  if (end - b == kSpecBlk)
    spec_block<WIDTH, true, DIV, FMT, AW, PW>(a, blk, b, end, it.tensor, tb, get_br, slot, part, anorm, tid);
  else
    spec_block<WIDTH, false, DIV, FMT, AW, PW>(a, blk, b, end, it.tensor, tb, get_br, slot, part, anorm, tid);
}

// Fused bracket (OMF_SPEC_FB / omf_plan_set_fused_bracket): the bracket launch folded into the pass.
// Its first kFbParts x (bracket items) workgroups sample the tensors (256 threads each, an eighth of
// a tensor's runs; the last part to arrive combines the sums and publishes the multipliers as two
// {epoch, value} granules); the rest are the pass's blocks, which issue their loads and draws and
// then poll their tensor's granules.  The bracket workgroups have the lowest ids, so they are
// dispatched before any pass block and never wait; a pass block's poll is bounded anyway (20 ms and a
// minimum of polls): on expiry the tensor is flagged and requantised whole by the finish — exact.
constexpr int kFbParts = 8;  // 64 runs each: four float4 per thread (the pass's blocks' register budget)

__device__ __forceinline__ void spec_bracket_part(const SpecArgs& a, const SpecBrItem* __restrict__ items, int64_t wg) {
  __shared__ double red[kWaves];
  __shared__ uint32_t s_last;
  const int part = (int)(wg % kFbParts);
  const SpecBrItem bi = items[wg / kFbParts];
  const int32_t t = bi.tensor;
  const int64_t tb = bi.begin, n = bi.n, R = bi.R;
  const float* __restrict__ x = a.e.x + tb;
  const bool exact = n <= kSpecExact;
  if (exact && part != 0) return;
  double s1 = 0.0, s2 = 0.0;
  if (exact) {  // 16 Ki elements at most: up to four rounds of four float4 per thread
    for (int64_t r0 = 0; r0 < n; r0 += 16 * kThreads) {
      float4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t e = r0 + 4 * ((int64_t)i * kThreads + threadIdx.x);
        v[i] = e + 4 <= n ? *reinterpret_cast<const float4*>(x + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < n && e + 4 > n) {  // the tensor's partial last quad
          v[i].x = x[e];
          if (e + 1 < n) v[i].y = x[e + 1];
          if (e + 2 < n) v[i].z = x[e + 2];
        }
      }
      float acc = 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = sq4(spec_prologue(v[i], a.e.alpha, a.divisor, a.e.fmt), acc);
      s1 += (double)acc;
    }
  } else {
    bracket_sample<kSpecRun, false, kThreads, 4>(a, x, t, tb, n, R, part, kFbParts, s1, s2);
  }
  double S1 = block_sum_f64(s1, red), S2 = block_sum_f64(s2, red);
  if (!exact) {  // the last part to arrive combines the partials in part order
    if (threadIdx.x == 0) {
      double* bp = a.br_part + 2 * ((int64_t)t * kFbParts + part);
      st_agent(reinterpret_cast<uint64_t*>(bp), (uint64_t)__double_as_longlong(S1));
      st_agent(reinterpret_cast<uint64_t*>(bp + 1), (uint64_t)__double_as_longlong(S2));
      drain_vmem();
      const uint32_t last = add_agent(&a.br_cnt[t], 1u) == (uint32_t)(kFbParts - 1) ? 1u : 0u;
      if (last) __hip_atomic_store(&a.br_cnt[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    S1 = S2 = 0.0;
    for (int g = 0; g < kFbParts; ++g) {
      const uint64_t* bp = reinterpret_cast<const uint64_t*>(a.br_part + 2 * ((int64_t)t * kFbParts + g));
      S1 += __longlong_as_double((long long)ld_agent(bp));
      S2 += __longlong_as_double((long long)ld_agent(bp + 1));
    }
  }
  if (threadIdx.x != 0) return;
  const SpecBracket o = bracket_from_sums(a, exact, n, R, kSpecRun, S1, S2);
  a.br[t] = o;  // the finish launch reads it (a later launch)
  const uint64_t ep = (uint64_t)a.epoch << 32;
  st_agent(&a.brgran[2 * t], ep | __float_as_uint(o.c_lo));
  st_agent(&a.brgran[2 * t + 1], ep | __float_as_uint(o.c_hi));
}

template <int WIDTH, bool DIV>
__global__ __launch_bounds__(kThreads) void qsgd_spec_quant_fb(SpecArgs a, const SpecBrItem* __restrict__ bitems,
                                                               int64_t nbrw, const int64_t* __restrict__ begins) {
  if ((int64_t)blockIdx.x < nbrw) {
    spec_bracket_part(a, bitems, blockIdx.x);
    return;
  }
  const int64_t blk = (int64_t)blockIdx.x - nbrw;
  const Item it = a.e.items[blk >> 2];
  const int32_t t = it.tensor;
  const int64_t tb = begins[t];
  const int64_t b = it.begin + (blk & 3) * kSpecBlk;
  const int wave = threadIdx.x >> 6;
  uint32_t* slot = a.slots + blk * kSpecSlot;
  uint64_t* part = a.partials + blk * kWaves + wave;
  if (b >= it.end) {
    if ((threadIdx.x & 63) == 0) {
      *part = 0ull;
      a.heads[blk * kWaves + wave] = (uint32_t)t << 8;
    }
    return;
  }
  auto get_br = [&]() {
    uint64_t g0 = ld_agent(&a.brgran[2 * t]), g1 = ld_agent(&a.brgran[2 * t + 1]);
    if ((uint32_t)(g0 >> 32) != a.epoch || (uint32_t)(g1 >> 32) != a.epoch) {
      const uint64_t t0 = wall_clock64(), min_polls = a.wait_ticks >> 10;
      uint64_t polls = 0;
      for (int k = 0;; k = min(k + 1, 6)) {
        if (k < 2) __builtin_amdgcn_s_sleep(2);
        else __builtin_amdgcn_s_sleep(8);
        g0 = ld_agent(&a.brgran[2 * t]);
        g1 = ld_agent(&a.brgran[2 * t + 1]);
        if ((uint32_t)(g0 >> 32) == a.epoch && (uint32_t)(g1 >> 32) == a.epoch) break;
        if (++polls > min_polls && wall_clock64() - t0 > a.wait_ticks) {  // never expected: requantise whole
          __hip_atomic_fetch_or(&a.flags[t], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          g0 = g1 = 0;
          break;
        }
      }
    }
    SpecBracket o{__uint_as_float((uint32_t)g0), __uint_as_float((uint32_t)g1), 0.f, 0.f, 0u, {0u, 0u, 0u}};
    return o;
  };
  const int64_t end = min(b + kSpecBlk, it.end);
  if (end - b == kSpecBlk) spec_block<WIDTH, true, DIV, kFmtF32>(a, blk, b, end, t, tb, get_br, slot, part, 0.0f, (int)threadIdx.x);
  else spec_block<WIDTH, false, DIV, kFmtF32>(a, blk, b, end, t, tb, get_br, slot, part, 0.0f, (int)threadIdx.x);
}

// Wide levels (bit widths 5-8): the bracket folded into the one-wave pass the same way.  Its first
// kWfbParts x (bracket items) one-wave workgroups sample the tensors — part g of a tensor its runs
// g kPassesW .., every kWfbParts kPassesW-th round, kPassesW 1 KiB runs in flight per lane — and
// the last part of each tensor to arrive combines the 16 parts' sums in part order and publishes
// the multipliers; the pass's one-wave blocks poll them as qsgd_spec_quant_fb's do.  A bracket from
// other partial sums than the separate launch's may list other quads: the payload is exact either
// way (test_fused_bracket_equals_bracket_launch).
#ifndef OMF_WFB_PARTS  // experiment builds may override them
#define OMF_WFB_PARTS 16
#endif
#ifndef OMF_WFB_PASSES
#define OMF_WFB_PASSES 8
#endif
constexpr int kWfbParts = OMF_WFB_PARTS;
constexpr int kPassesW = OMF_WFB_PASSES;

__device__ __forceinline__ void spec_bracket_part_wide(const SpecArgs& a, const SpecBrItem* __restrict__ items,
                                                       int64_t wg) {
  const int part = (int)(wg % kWfbParts);
  const SpecBrItem bi = items[wg / kWfbParts];
  const int32_t t = bi.tensor;
  const int64_t tb = bi.begin, n = bi.n, R = bi.Rw;
  const float* __restrict__ x = a.e.x + tb;
  const bool exact = n <= kSpecExact;
  if (exact && part != 0) return;
  const int lane = threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (exact) {  // 16 Ki elements at most: rounds of four float4 per lane
    for (int64_t r0 = 0; r0 < n; r0 += 16 * 64) {
      float4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t e = r0 + 4 * ((int64_t)i * 64 + lane);
        v[i] = e + 4 <= n ? *reinterpret_cast<const float4*>(x + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < n && e + 4 > n) {  // the tensor's partial last quad
          v[i].x = x[e];
          if (e + 1 < n) v[i].y = x[e + 1];
          if (e + 2 < n) v[i].z = x[e + 2];
        }
      }
      float acc = 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = sq4(spec_prologue(v[i], a.e.alpha, a.divisor, a.e.fmt), acc);
      s1 += (double)acc;
    }
  } else {
    bracket_sample<kSpecRunWide, false, 64, kPassesW>(a, x, t, tb, n, R, part, kWfbParts, s1, s2);
  }
  double S1 = wave_sum_f64(s1), S2 = wave_sum_f64(s2);
  if (lane != 0) return;
  if (!exact) {  // the last part to arrive combines the partials in part order
    double* bp = a.br_part + 2 * ((int64_t)t * kWfbParts + part);
    st_agent(reinterpret_cast<uint64_t*>(bp), (uint64_t)__double_as_longlong(S1));
    st_agent(reinterpret_cast<uint64_t*>(bp + 1), (uint64_t)__double_as_longlong(S2));
    drain_vmem();
    if (add_agent(&a.br_cnt[t], 1u) != (uint32_t)(kWfbParts - 1)) return;
    __hip_atomic_store(&a.br_cnt[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S1 = S2 = 0.0;
    for (int g = 0; g < kWfbParts; ++g) {
      const uint64_t* q = reinterpret_cast<const uint64_t*>(a.br_part + 2 * ((int64_t)t * kWfbParts + g));
      S1 += __longlong_as_double((long long)ld_agent(q));
      S2 += __longlong_as_double((long long)ld_agent(q + 1));
    }
  }
  const SpecBracket o = bracket_from_sums(a, exact, n, R, kSpecRunWide, S1, S2);
  a.br[t] = o;  // the finish launch reads it (a later launch)
  const uint64_t ep = (uint64_t)a.epoch << 32;
  st_agent(&a.brgran[2 * t], ep | __float_as_uint(o.c_lo));
  st_agent(&a.brgran[2 * t + 1], ep | __float_as_uint(o.c_hi));
}

// The pass blocks' poll for their tensor's fused bracket (bounded: on expiry the tensor is flagged
// and requantised whole by the finish — exact; the sampling workgroups have the lowest ids, so they
// are dispatched before any pass block and never wait).
__device__ __forceinline__ SpecBracket fb_poll(const SpecArgs& a, int32_t t) {
  uint64_t g0 = ld_agent(&a.brgran[2 * t]), g1 = ld_agent(&a.brgran[2 * t + 1]);
  if ((uint32_t)(g0 >> 32) != a.epoch || (uint32_t)(g1 >> 32) != a.epoch) {
    const uint64_t t0 = wall_clock64(), min_polls = a.wait_ticks >> 10;
    uint64_t polls = 0;
    for (int k = 0;; k = min(k + 1, 6)) {
      if (k < 2) __builtin_amdgcn_s_sleep(2);
      else __builtin_amdgcn_s_sleep(8);
      g0 = ld_agent(&a.brgran[2 * t]);
      g1 = ld_agent(&a.brgran[2 * t + 1]);
      if ((uint32_t)(g0 >> 32) == a.epoch && (uint32_t)(g1 >> 32) == a.epoch) break;
      if (++polls > min_polls && wall_clock64() - t0 > a.wait_ticks) {  // never expected: requantise whole
        __hip_atomic_fetch_or(&a.flags[t], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g0 = g1 = 0;
        break;
      }
    }
  }
  return SpecBracket{__uint_as_float((uint32_t)g0), __uint_as_float((uint32_t)g1), 0.f, 0.f, 0u, {0u, 0u, 0u}};
}

template <int WIDTH, bool DIV>
__global__ __launch_bounds__(64) void qsgd_spec_quant_wfb(SpecArgs a, const SpecBrItem* __restrict__ bitems,
                                                          int64_t nbrw, const int64_t* __restrict__ begins) {
  if ((int64_t)blockIdx.x < nbrw) {
    spec_bracket_part_wide(a, bitems, blockIdx.x);
    return;
  }
  const int64_t wgi = (int64_t)blockIdx.x - nbrw;
  const int64_t blk = wgi / kWaves;
  const int tid = (int)(wgi % kWaves) * 64 + (int)threadIdx.x;
  const Item it = a.e.items[blk >> 2];
  const int32_t t = it.tensor;
  const int64_t tb = begins[t];
  const int64_t b = it.begin + (blk & 3) * kSpecBlk;
  const int wave = tid >> 6;
  uint32_t* slot = a.slots + blk * spec_slot_words(kSpecPerWaveWide);
  uint64_t* part = a.partials + blk * kWaves + wave;
  if (b >= it.end) {
    if (threadIdx.x == 0) {
      *part = 0ull;
      a.heads[blk * kWaves + wave] = (uint32_t)t << 8;
    }
    return;
  }
  auto get_br = [&]() { return fb_poll(a, t); };
  const int64_t end = min(b + kSpecBlk, it.end);
  if (end - b == kSpecBlk)
    spec_block<WIDTH, true, DIV, kFmtF32, 0, kSpecPerWaveWide>(a, blk, b, end, t, tb, get_br, slot, part, 0.0f, tid);
  else
    spec_block<WIDTH, false, DIV, kFmtF32, 0, kSpecPerWaveWide>(a, blk, b, end, t, tb, get_br, slot, part, 0.0f, tid);
}

// One fold segment (a workgroup of the finish launch); the last arriver of the tensor folds the
// segments in order, checks the bracket and publishes {epoch, bad, norm} in the tensor's granule.
__device__ void spec_fold(const SpecArgs& a, const SpecFoldItem& fi) {
  __shared__ double red[kWaves];
  __shared__ uint32_t s_last;
  const int32_t t = fi.tensor;
  // up to kSpecSeg partials: 16 loads in flight per thread, a fixed order
  constexpr int U = kSpecSeg / kThreads;
  double v[U];
#pragma unroll
  for (int i = 0; i < U; ++i) {
    const int64_t j = fi.p_begin + threadIdx.x + (int64_t)i * kThreads;
    const double d = __longlong_as_double((long long)a.partials[j < fi.p_end ? j : fi.p_begin]);  // unconditional load
    v[i] = j < fi.p_end ? d : 0.0;
  }
  double p = 0.0;
#pragma unroll
  for (int i = 0; i < U; ++i) p += v[i];
  double tot = block_sum_f64(p, red);
  if (fi.nsegs > 1) {
    if (threadIdx.x == 0) {
      st_agent(&a.seg_part[fi.sbase + fi.seg], (uint64_t)__double_as_longlong(tot));
      drain_vmem();
      const uint32_t last = add_agent(&a.fold_cnt[t], 1u) == (uint32_t)(fi.nsegs - 1) ? 1u : 0u;
      if (last) __hip_atomic_store(&a.fold_cnt[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    double q = 0.0;
    for (int j = threadIdx.x; j < fi.nsegs; j += kThreads)
      q += __longlong_as_double((long long)ld_agent(&a.seg_part[fi.sbase + j]));
    tot = block_sum_f64(q, red);
  }
  if (threadIdx.x != 0) return;
  const float norm = finish_norm(tot, a.e.fmt);
  a.e.norm_out[t] = norm;
  const SpecBracket br = a.br[t];
  const uint32_t fl = a.flags[t];
  const bool ok = br.mode == 0u && fl == 0u && norm >= br.n_lo && norm <= br.n_hi;
  a.status[t] = ok ? 0u : 1u;
  if (fl) a.flags[t] = 0u;
  st_agent(&a.ngran[t], ((uint64_t)((a.epoch << 1) | (ok ? 0u : 1u)) << 32) | __float_as_uint(norm));
}

// The tensor's norm and status as its fold published them in this launch (bounded; the fold
// workgroups are dispatched before every fix workgroup and never wait, so the bound is only a
// guard against a logic error).  false: timed out (err bit 4 set, reported as OMF_ETIMEOUT by
// omf_plan_check, which every product entry point calls).  The bound needs the wall-clock
// time AND a minimum number of polls, so a context switch of the queue (the clock runs on
// while the wave is saved) cannot fake an expiry.
__device__ __forceinline__ bool spec_norm_wait(const SpecArgs& a, int32_t t, float& norm, bool& bad) {
  uint64_t g = ld_agent(&a.ngran[t]);
  if ((uint32_t)(g >> 33) != a.epoch) {
    // exponential back-off: every polling wave reads one of 183-odd granules, and tight
    // polling of a few lines by tens of thousands of waves congests them
    const uint64_t t0 = wall_clock64();
    const uint64_t min_polls = a.wait_ticks >> 10;  // a back-off poll is <= ~200 ticks
    uint64_t polls = 0;
    for (int k = 0;; k = min(k + 1, 6)) {
      if (k < 2) __builtin_amdgcn_s_sleep(4);
      else if (k < 4) __builtin_amdgcn_s_sleep(16);
      else __builtin_amdgcn_s_sleep(64);
      g = ld_agent(&a.ngran[t]);
      if ((uint32_t)(g >> 33) == a.epoch) break;
      if (++polls > min_polls && wall_clock64() - t0 > a.wait_ticks) {
        __hip_atomic_fetch_or(a.e.err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
  norm = __uint_as_float((uint32_t)g);
  bad = ((g >> 32) & 1u) != 0u;
  return true;
}

// The finish launch: its first nfold workgroups fold the partials (spec_fold); the rest fix the
// listed quads, one thread per wave slot: (the slot header), then (the block's item) with the
// tensor's norm granule, then per listed quad its index, recorded x and draws, the exact level
// from the shared element math (Markstein division) and its store.  A block whose tensor the fold marked bad (norm outside the bracket, a slot
// overflow, a deferred tensor) is requantised whole from x by its workgroup (the rare path).
template <int WIDTH, int PW = kSpecPerWave, int FT = 1>
__global__ __launch_bounds__(kThreads) void qsgd_spec_finish(SpecArgs a, const SpecFoldItem* __restrict__ fold_items,
                                                             int32_t nfold, const Item* __restrict__ items,
                                                             const int64_t* __restrict__ begins,
                                                             const uint32_t* __restrict__ slots,
                                                             const float4* __restrict__ recs,
                                                             const uint32_t* __restrict__ heads) {
  if ((int32_t)blockIdx.x < nfold) {
    if (!(a.dbg & 16u)) spec_fold(a, fold_items[blockIdx.x]);  // test hook: no fold, the fix waits expire
    return;
  }
  // FT threads per wave slot (its listed quads in turn, strided: narrow levels list none or one, so
  // FT = 1 there — 8 threads per slot took 8x the workgroups: +8-10 us; wide levels list ~10 per
  // slot, FT = 4), kThreads / (kWaves FT) blocks per workgroup: the fix is a few dependent round
  // trips per thread, so its cost is the number of workgroup generations, not the quads.
  constexpr int BPW = kThreads / (kWaves * FT);  // blocks per workgroup
  __shared__ uint32_t s_rep[BPW];
  __shared__ float s_rep_norm[BPW];  // the granule's norm (norm_out is written in this launch)
  __shared__ uint32_t s_nrep;
  const EncArgs& e = a.e;
  const int64_t fb = (int64_t)blockIdx.x - nfold;
  if (threadIdx.x == 0) s_nrep = 0u;
  const int64_t ws = (fb * kThreads + threadIdx.x) / FT;  // global wave slot
  const uint32_t sub = (uint32_t)(threadIdx.x % FT);
  const int64_t blk = ws / kWaves;
  const int w = (int)(ws % kWaves);
  bool rep = false;
  float rep_norm = 0.0f;
  if (blk < a.nblocks) {
    const uint32_t head = heads[ws];
    const uint32_t cnt = head & 0xffu;
    const int32_t t = (int32_t)(head >> 8);
    const bool leader = w == 0 && sub == 0;  // one status check per block
    if ((cnt > 0u || leader) && !(a.dbg & 8u)) {
      // this thread's first PRE listed quads (index, recorded x and draws) are loaded before the
      // norm wait, so their round trip overlaps it (clamped to the last listed quad: no load
      // under a branch); the rest, if any (narrow lists only), in the loop after
      constexpr int PRE = FT > 1 ? PW / FT : 0;  // (narrow lists: usually empty, the loop below)
      uint32_t qv[PRE > 0 ? PRE : 1];
      float4 rx[PRE > 0 ? PRE : 1], ru[PRE > 0 ? PRE : 1];
      const uint32_t jl = cnt > 0u ? cnt - 1u : 0u;
#pragma unroll
      for (int k = 0; k < PRE; ++k) {
        const uint32_t j = min(sub + (uint32_t)(k * FT), jl);
        qv[k] = slots[blk * spec_slot_words(PW) + PW * w + j];
        rx[k] = recs[2 * (ws * PW + j)];
        ru[k] = recs[2 * (ws * PW + j) + 1];
      }
      const Item it = items[blk >> 2];
      float norm;
      bool bad;
      if (spec_norm_wait(a, t, norm, bad)) {
        const int64_t b = it.begin + (blk & 3) * kSpecBlk, end = min(b + kSpecBlk, it.end);
        const Divisor dv(norm, e.fmt);
#pragma unroll
        for (int k = 0; k < PRE; ++k) {
          if (sub + (uint32_t)(k * FT) >= cnt) break;
          int32_t qq[4];
          qsgd_quad<false>(rx[k], ru[k], dv, e.levels, false, qq);
          if (!(a.dbg & 4u)) store_quad<WIDTH>(e, 4 * (int64_t)qv[k], end, qq);
        }
        for (uint32_t j = sub + (uint32_t)(PRE * FT); j < cnt; j += FT) {
          const uint32_t q = slots[blk * spec_slot_words(PW) + PW * w + j];
          const float4* rec = recs + 2 * (ws * PW + j);
          int32_t qq[4];
          qsgd_quad<false>(rec[0], rec[1], dv, e.levels, false, qq);
          if (!(a.dbg & 4u)) store_quad<WIDTH>(e, 4 * (int64_t)q, end, qq);
        }
        rep = leader && bad;
        rep_norm = norm;
      }
    }
  }
  __syncthreads();  // s_nrep initialised
  if (rep) {
    const uint32_t i = atomicAdd(&s_nrep, 1u);
    s_rep[i] = (uint32_t)(blk - fb * BPW);
    s_rep_norm[i] = rep_norm;
  }
  if (!__syncthreads_or(rep)) return;
  const uint32_t nrep = s_nrep;
  EncArgs er = e;  // the fused PS step requantises from the average the pass wrote
  if (a.divisor != 0.0f) {
    er.x = a.xout;
    er.alpha = 1.0f;
  }
  for (uint32_t r = 0; r < nrep; ++r) {  // whole blocks of requantised tensors, all 256 threads
    const int64_t rb = fb * BPW + s_rep[r];
    const Item it = items[rb >> 2];
    const int64_t b = it.begin + (rb & 3) * kSpecBlk;
    if (b < it.end)
      quant_sub<WIDTH, false, kSpecV>(er, b, min(b + kSpecBlk, it.end), begins[it.tensor], it.tensor, s_rep_norm[r]);
  }
}

// ---------------------------------------------------------------- grid encoder (strategy 4)
// Small arenas (ResNet-18: 11 M elements in 2 976 blocks of 4 Ki): ONE launch of one 1024-thread
// workgroup per CU; each quarter (256 threads) holds kGridNB 4 Ki blocks of x in registers
// (the 16 wave partials of an item — 4 blocks x 4 waves — are summed in a fixed order in LDS and
// published as ONE fp64 item partial), every workgroup arrives at one grid-wide counter, and
// after it every tensor's norm is the same deterministic fold of its item partials in every
// workgroup (no second barrier; one round of loads per wave for tensors of <= 512 items) and the blocks are
// quantised from registers: x is read once, with no per-tensor hand-off chain (the ring's) and
// no sampled bracket (the bracketed encoder's four launches).  The hand-off is cdna_hip_
// programming.md §6 Guideline 16, table row 1: 8-byte sc1 partial stores, every wave's
// vmcnt(0), a workgroup barrier, one agent-scope add per workgroup; an sc1 poll of the counter,
// a workgroup barrier, sc1 loads; one workgroup per CU.  The counter wait is bounded (20 ms
// and a minimum number of polls); on expiry each workgroup recomputes the partials it needs
// from x in the producers' exact order (same bits) and sets err bit 2.
constexpr int kGridNB = 3;  // 4 Ki blocks per quarter-workgroup per launch

struct GridArgs {
  EncArgs e;                    // x, q, norm_out, alpha, fmt, levels, Philox key / offset, err, wait_ticks
  uint64_t* partials;           // fp64 bits, one per flat item (16 Ki elements)
  unsigned long long* bar;      // grid arrival counter (monotonic over launches)
  unsigned long long target;    // its value once every workgroup of this launch has arrived
  int64_t nblocks;              // 4 Ki blocks of the plan (4 per flat item)
  uint32_t dbg;                 // test hooks (omf_plan_set_debug spec bits): 32 arrive late, 64 no wait,
                                // 128 no fold, 256 no quantisation
};

typedef uint32_t g32x4_t __attribute__((ext_vector_type(4)));
// Range-checked buffer load of the float4 at byte offset voff of [base, base + bytes): dwords
// past the range read 0, so a tensor's partial last block needs no branch around its loads.
__device__ __forceinline__ float4 grid_ld4(const float* base, int64_t bytes, int voff) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)max(bytes, (int64_t)0), 0x00020000);
  const g32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// Rows k = 0..3 of 4 Ki block [b, end) at quarter-thread lt: x * alpha (value format applied).
__device__ __forceinline__ void grid_load_block(const EncArgs& e, int64_t b, int64_t end, int lt, float4 (&v)[4]) {
  const float* base = e.x + b;
  const int64_t bytes = 4 * (end - b);
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = grid_ld4(base, bytes, 16 * (k * kThreads + lt));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (e.alpha != 1.0f) {
      v[k] = make_float4(__fmul_rn(v[k].x, e.alpha), __fmul_rn(v[k].y, e.alpha), __fmul_rn(v[k].z, e.alpha),
                         __fmul_rn(v[k].w, e.alpha));
      if (e.fmt) v[k] = round_fmt4(v[k], e.fmt);
    }
  }
}

// The block's wave partial of quarter-thread lt's wave: the fp32 fma chain over its 16 values,
// then the fp64 wave butterfly (identical in the producer and in the recovery).
__device__ __forceinline__ double grid_partial(const float4 (&v)[4]) {
  float acc = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) acc = sq4(v[k], acc);
  return wave_sum_f64((double)acc);
}

// Item partial: its 16 wave partials (block q = 0..3 of the item, wave w = 0..3 of the block's
// quarter-workgroup) summed in fp64 in the order q-major, w-minor (producer and recovery alike).
// Tensor t's norm by ONE wave: lane l sums item partials l, l + 64, ... in order (fp64), then
// the butterfly — the same bits in every workgroup.  recover: the item partials are recomputed
// from x.
__device__ float grid_fold(const GridArgs& a, const Item* __restrict__ items, uint32_t p0, uint32_t pn, bool recover) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  if (!recover) {
    constexpr int U = 8;
    for (uint32_t j0 = 0; j0 < pn; j0 += 64 * U) {
      double d[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t j = j0 + 64 * u + lane;
        d[u] = j < pn ? __longlong_as_double((long long)ld_agent(&a.partials[p0 + j])) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j0 + 64 * u + lane < pn) s += d[u];
    }
  } else {  // each item partial as its workgroup made it
    for (uint32_t j = 0; j < pn; ++j) {
      const Item it = items[p0 + j];
      double ip = 0.0;
      for (int q = 0; q < 4; ++q) {
        const int64_t b = it.begin + (int64_t)q * kSpecBlk, end = min(b + kSpecBlk, it.end);
        for (int wq = 0; wq < 4; ++wq) {
          float4 v[4];
          grid_load_block(a.e, b, end, 64 * wq + lane, v);
          ip += grid_partial(v);
        }
      }
      if ((j & 63) == (uint32_t)lane) s += ip;
    }
  }
  return finish_norm(wave_sum_f64(s), a.e.fmt);
}

template <int WIDTH>
__global__ __launch_bounds__(1024) void qsgd_encode_grid(GridArgs a, const Item* __restrict__ items,
                                                         const int64_t* __restrict__ begins,
                                                         const uint32_t* __restrict__ pbeg,
                                                         const uint32_t* __restrict__ pcnt) {
  __shared__ float s_norm[kGridNB];
  __shared__ double s_part[kGridNB][16];
  __shared__ uint32_t s_ok;
  const EncArgs& e = a.e;
  const int lt = threadIdx.x & 255, qv = threadIdx.x >> 8, lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6, wq = wave & 3;
  const int64_t W = gridDim.x;
  float4 v[kGridNB][4];
  int64_t bb[kGridNB], be[kGridNB];
  int32_t tt[kGridNB];
  // phase 1: the blocks' x into registers, their wave partials published
#pragma unroll
  for (int i = 0; i < kGridNB; ++i) {
    const int64_t item = (int64_t)i * W + blockIdx.x;
    const bool live = 4 * item < a.nblocks;
    const Item it = items[live ? item : 0];
    bb[i] = it.begin + qv * kSpecBlk;
    be[i] = live ? min(bb[i] + kSpecBlk, it.end) : bb[i];  // empty range: loads read 0
    tt[i] = live ? it.tensor : -1;
    grid_load_block(e, bb[i], be[i], lt, v[i]);
  }
#pragma unroll
  for (int i = 0; i < kGridNB; ++i) {
    const double p = grid_partial(v[i]);
    if (lane == 0) s_part[i][4 * qv + wq] = p;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kGridNB; ++i)  // thread i: item i's partial, in a fixed order
    if ((int)threadIdx.x == i && tt[i] >= 0) {
      double ip = 0.0;
#pragma unroll
      for (int j = 0; j < 16; ++j) ip += s_part[i][j];
      st_agent(&a.partials[(int64_t)i * W + blockIdx.x], (uint64_t)__double_as_longlong(ip));
    }
  drain_vmem();
  __syncthreads();
  if (threadIdx.x == 0) {
    // (test hook dbg & 32: arrive only after the wait, so that every wait expires and the counter
    // still advances by the grid size per launch)
    if (!(a.dbg & 32u)) __hip_atomic_fetch_add(a.bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // bounded wait: wall clock AND a minimum number of polls (a queue context switch advances
    // the clock while the wave is saved)
    uint32_t ok = 1;
    if (!(a.dbg & 64u) && __hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.target) {
      const uint64_t t0 = wall_clock64(), min_polls = e.wait_ticks >> 10;
      uint64_t polls = 0;
      for (int k = 0;; k = min(k + 1, 4)) {
        if (k < 2) __builtin_amdgcn_s_sleep(2);
        else __builtin_amdgcn_s_sleep(16);
        if (__hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.target) break;
        if (++polls > min_polls && wall_clock64() - t0 > e.wait_ticks) {
          ok = 0;
          __hip_atomic_fetch_or(e.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    if (a.dbg & 32u) __hip_atomic_fetch_add(a.bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ok = ok;
  }
  __syncthreads();
  // phase 2: wave i folds the norm of iteration i's tensor (the quarters of one item share it)
  if (wave < kGridNB && tt[wave] >= 0) {
    const int32_t t = tt[wave];
    const uint32_t p0 = pbeg[t];
    const float norm = (a.dbg & 128u) ? 1.0f : grid_fold(a, items, p0, pcnt[t], s_ok == 0u);
    if (lane == 0) {
      s_norm[wave] = norm;
      if ((int64_t)wave * W + blockIdx.x == (int64_t)p0) e.norm_out[t] = norm;  // the tensor's first item
    }
  }
  __syncthreads();
  // phase 3: levels from registers
  if (a.dbg & 256u) return;
#pragma unroll
  for (int i = 0; i < kGridNB; ++i) {
    if (tt[i] < 0 || bb[i] >= be[i]) continue;
    const float norm = s_norm[i];
    const Divisor dv(norm, e.fmt);
    float4 uu[4];
    {
      const uint64_t G = (uint64_t)((bb[i] - begins[tt[i]]) >> 12) * (uint64_t)kThreads + (uint64_t)lt;
      uint32_t w[12];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const uint64_t ctr = 3 * G + c;
        const uint4 r = philox4x32_10(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)tt[i], e.offset),
                                      e.seed_lo, e.seed_hi);
        w[4 * c] = r.x; w[4 * c + 1] = r.y; w[4 * c + 2] = r.z; w[4 * c + 3] = r.w;
      }
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) uu[sl] = u24x4(w[3 * sl], w[3 * sl + 1], w[3 * sl + 2]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t el = bb[i] + 4 * ((int64_t)k * kThreads + lt);
      if (el >= be[i]) continue;
      int32_t qq[4];
      qsgd_quad<false>(v[i][k], uu[k], dv, e.levels, !(norm != 0.0f), qq);
      store_quad<WIDTH>(e, el, be[i], qq);
    }
  }
}

// Decode one sub-chunk [b, end): y = fl32(fl32(norm * q) / L) (optionally acc += y).
template <int WIDTH, bool ACC, bool POW2, bool FULL, int V = kV>
__device__ __forceinline__ void decode_sub(const DecArgs& a, int64_t b, int64_t end, float norm) {
  int32_t raw[V][WIDTH == 1 ? 1 : 4];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
    if (WIDTH == 1) {
      const int8_t* q8 = reinterpret_cast<const int8_t*>(a.q);
      if (FULL || e + 4 <= end) {  // streamed once: nontemporal
        raw[k][0] = __builtin_nontemporal_load(reinterpret_cast<const int32_t*>(q8 + e));
      } else {
        uint32_t t = 0;
        if (e < end) t |= (uint32_t)(uint8_t)q8[e];
        if (e + 1 < end) t |= (uint32_t)(uint8_t)q8[e + 1] << 8;
        if (e + 2 < end) t |= (uint32_t)(uint8_t)q8[e + 2] << 16;
        raw[k][0] = (int32_t)t;
      }
    } else {
      const int32_t* q32 = reinterpret_cast<const int32_t*>(a.q);
      if (FULL || e + 4 <= end) {
        const i32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t*>(q32 + e));
        raw[k][0] = t[0]; raw[k][1] = t[1]; raw[k][2] = t[2]; raw[k][3] = t[3];
      } else {
        raw[k][0] = (e < end) ? q32[e] : 0;
        raw[k][1] = (e + 1 < end) ? q32[e + 1] : 0;
        raw[k][2] = (e + 2 < end) ? q32[e + 2] : 0;
        raw[k][3] = 0;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = b + 4 * ((int64_t)k * kThreads + threadIdx.x);
    if (!FULL && e >= end) continue;
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
    if (FULL || e + 4 <= end) {
      float4 o = make_float4(yv[0], yv[1], yv[2], yv[3]);
      if (ACC) {
        const f32x4_t pv = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(y));
        const float4 prev = make_float4(pv[0], pv[1], pv[2], pv[3]);
        o.x = __fadd_rn(prev.x, o.x); o.y = __fadd_rn(prev.y, o.y);
        o.z = __fadd_rn(prev.z, o.z); o.w = __fadd_rn(prev.w, o.w);
      }
      store_nt(y, o);
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (e + c < end) y[c] = ACC ? __fadd_rn(y[c], yv[c]) : yv[c];
    }
  }
}

template <int WIDTH, bool ACC, bool POW2>
__global__ __launch_bounds__(kThreads) void qsgd_decode_flat(DecArgs a) {
  const Item it = a.items[blockIdx.x];
  const float norm = a.norm[it.tensor];
  for (int64_t b = it.begin; b < it.end; b += kSub) {
    const int64_t end = min(b + kSub, it.end);
    if (end - b == kSub) decode_sub<WIDTH, ACC, POW2, true>(a, b, end, norm);
    else decode_sub<WIDTH, ACC, POW2, false>(a, b, end, norm);
  }
}

// Decoder over arena-aligned blocks: the payload loads depend on blockIdx only, so they go out
// at once; the block's tensor (binfo, one entry per 4 Ki-element table block: tensor id, bit 31 =
// the table block lies inside it) and its norm are scalar loads in flight with them.  A block in
// a table block that crosses a tensor boundary or padding (at most nt + 1 of them) finds each
// quad's tensor and writes only its elements.  Round 5: the decode block is narrower than the
// table block — kDecQuads(W, ACC) quads per thread: 2 for an int8 payload, 1 for an int32 payload
// or an accumulate — measured on Llama-400M (scripts/exp/dec_shapes.hip, interleaved): int8
// 0.298-0.304 ms against 0.331 with 4 quads, int32 0.492 against 0.550, accumulate 0.556 / 0.748
// against 0.612 / 0.807 (fewer bytes per thread, more workgroups in flight per CU).
constexpr int64_t kDecBlk = (int64_t)4 * kThreads * 4;  // 4096 elements per binfo table block
template <int WIDTH, bool ACC>
constexpr int kDecQuads = (WIDTH == 1 && !ACC) ? 2 : 1;

template <int WIDTH, bool ACC, bool POW2>
__device__ __forceinline__ void dec_quad(const DecArgs& a, int32_t raw[4], float norm, float (&yv)[4]) {
  int32_t qi[4];
  if (WIDTH == 1) {
    qi[0] = (int32_t)(int8_t)(raw[0] & 0xff);
    qi[1] = (int32_t)(int8_t)((raw[0] >> 8) & 0xff);
    qi[2] = (int32_t)(int8_t)((raw[0] >> 16) & 0xff);
    qi[3] = (int32_t)(int8_t)((raw[0] >> 24) & 0xff);
  } else {
    qi[0] = raw[0]; qi[1] = raw[1]; qi[2] = raw[2]; qi[3] = raw[3];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float nq = __fmul_rn(norm, (float)qi[c]);
    yv[c] = POW2 ? __fmul_rn(nq, a.inv_levels) : nq / a.levels;
  }
}

template <int WIDTH, bool ACC, bool POW2>
__global__ __launch_bounds__(kThreads) void qsgd_decode_arena(DecArgs a, const uint32_t* __restrict__ binfo,
                                                              const float* __restrict__ norms,
                                                              const int64_t* __restrict__ begins,
                                                              const int64_t* __restrict__ sizes, int32_t nt,
                                                              int64_t qlast, uint32_t blk0) {
  constexpr int V = kDecQuads<WIDTH, ACC>;
  const uint32_t bid = blk0 + blockIdx.x;  // a range launch starts at block blk0
  const int64_t base = (int64_t)bid * (V * kThreads * 4);
  int32_t raw[V][WIDTH == 1 ? 1 : 4];
#pragma unroll
  for (int k = 0; k < V; ++k) {  // unconditional (clamped) loads
    const int64_t e = min(base + 4 * ((int64_t)k * kThreads + threadIdx.x), qlast);
    if (WIDTH == 1) {  // default policy: 0.298 against 0.304 ms non-temporal (dec_shapes.hip)
      raw[k][0] = *reinterpret_cast<const int32_t*>(reinterpret_cast<const int8_t*>(a.q) + e);
    } else {
      const i32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t*>(reinterpret_cast<const int32_t*>(a.q) + e));
      raw[k][0] = t[0]; raw[k][1] = t[1]; raw[k][2] = t[2]; raw[k][3] = t[3];
    }
  }
  const uint32_t info = binfo[base / kDecBlk];
  const int32_t t0 = (int32_t)(info & 0x7fffffffu);
  if (info >> 31) {  // the whole table block lies inside tensor t0
    const float norm = norms[t0];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int64_t e = base + 4 * ((int64_t)k * kThreads + threadIdx.x);
      float yv[4];
      dec_quad<WIDTH, ACC, POW2>(a, raw[k], norm, yv);
      float4 o = make_float4(yv[0], yv[1], yv[2], yv[3]);
      if (ACC) {
        const f32x4_t pv = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(a.y + e));
        o.x = __fadd_rn(pv[0], o.x); o.y = __fadd_rn(pv[1], o.y);
        o.z = __fadd_rn(pv[2], o.z); o.w = __fadd_rn(pv[3], o.w);
      }
      store_nt(a.y + e, o);
    }
    return;
  }
  // boundary block: each quad's tensor, element by element
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = base + 4 * ((int64_t)k * kThreads + threadIdx.x);
    int32_t t = t0;
    while (t + 1 < nt && e >= begins[t + 1]) ++t;
    const int64_t tb = begins[t], te = tb + sizes[t];
    if (e + 3 < tb || e >= te) continue;  // padding (offsets are multiples of 4: a quad never
                                          // starts before its tensor and ends inside it)
    int32_t rr[4] = {raw[k][0], WIDTH == 1 ? 0 : raw[k][1], WIDTH == 1 ? 0 : raw[k][2], WIDTH == 1 ? 0 : raw[k][3]};
    if (e + 4 > te) {  // the tensor's partial last quad: its bytes only (the payload may end here)
      if (WIDTH == 1) {
        const int8_t* q8 = reinterpret_cast<const int8_t*>(a.q);
        uint32_t w = 0;
        for (int c = 0; c < 3; ++c)
          if (e + c < te) w |= (uint32_t)(uint8_t)q8[e + c] << (8 * c);
        rr[0] = (int32_t)w;
      } else {
        const int32_t* q32 = reinterpret_cast<const int32_t*>(a.q);
        for (int c = 0; c < 3; ++c) rr[c] = e + c < te ? q32[e + c] : 0;
        rr[3] = 0;
      }
    }
    float yv[4];
    dec_quad<WIDTH, ACC, POW2>(a, rr, norms[t], yv);
    for (int c = 0; c < 4; ++c)
      if (e + c < te) a.y[e + c] = ACC ? __fadd_rn(a.y[e + c], yv[c]) : yv[c];
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
  int64_t arena_end = 0;
  int64_t cap = 0;               // tensors of <= cap items take the register-resident path
  int32_t strategy = 2;          // 0 register-resident + two-pass, 1 ticket-ordered two-pass, 2 single-read ring,
                                 // 3 bracketed single-read (default by size: omf_plan_create)
  int32_t last_encoder = -1;     // the encoder the latest encode launched (omf_plan_last_encoder)
  uint64_t wait_ticks = kWaitTicks;      // norm waits (ring: expiry recomputes; bracketed fix: expiry fails)
  uint64_t lds_wait_ticks = kWaitTicks;  // the ring's on-chip hand-off waits (expiry aborts the workgroup)
  uint32_t epoch = 0;            // last granule tag used (host-side launch counter)
  int32_t ev = 8;                // encode rows per thread (sub-chunk = ev * 1024 elements): 8 measured
                                 // faster than 16 for the two-pass encoder (0.596 vs 0.606 ms, Llama-400M)
  int64_t n_enc[2] = {0, 0};
  Item* d_enc[2] = {nullptr, nullptr};
  TensorInfo* d_tinfo[2] = {nullptr, nullptr};
  int64_t n_flat = 0, n_partials = 0;
  Item* d_flat = nullptr;
  uint64_t* d_partials = nullptr;
  int64_t* d_sizes = nullptr;   // per-tensor element counts (Top-K)
  int64_t* d_begins = nullptr;  // per-tensor arena offsets (Top-K)
  void* d_block = nullptr;      // one allocation for everything above
  uint8_t* d_sync = nullptr;    // [ticket u32, err u32, pad 8][counters u32 x nt, pad16][granules u64 x nt, pad16]
  size_t sync_bytes = 0, off_counters = 16, off_gran = 0;
  // single-read ("ring") encoder, strategy 2 (omf_qsgd_ring.hip)
  int32_t ring_cfg = 0;         // omf_qsgd_ring.hip kConfigs[0]: 64 KiB chunks, 8 loader + 8 quantiser waves
  int32_t ring_grid = 0;
  int32_t ring_big_mode = 1;     // 0: QUANT chunks of a large tensor ring_gap items after its NORM chunks; 1: NORM first, QUANT last
  int64_t ring_gap = -1;         // items (-1: one grid)
  int64_t ring_hold_override = 0;  // > 0: hold limit in chunks (tests)
  uint32_t ring_dbg = 0;           // test / experiment switches (omf_plan_set_debug), 0 in production
  uint32_t ring_epoch = 0;
  int64_t n_ring = 0, n_ring_gran = 0, ring_hold_max = 0, ring_two_pass = 0;
  omf::ring::Item* d_ring = nullptr;
  omf::ring::Tensor* d_ring_t = nullptr;
  uint64_t* d_ring_gran = nullptr;
  unsigned long long* d_ring_prof = nullptr;  // 16 phase counters (OMF_RING_DBG & 4)
  // bracketed single-read encoder, strategy 3: per-tensor brackets / flags / status, per
  // 4 Ki-element block partials and undecided-quad slots
  int64_t n_spec_blocks = 0, n_spec_br = 0, n_spec_fold = 0;
  SpecBrItem* d_spec_br_items = nullptr;
  SpecFoldItem* d_spec_fold_items = nullptr;
  uint64_t* d_spec_seg_part = nullptr;
  uint32_t* d_spec_cnt = nullptr;  // fold_cnt x nt
  uint32_t spec_epoch = 0;
  uint32_t spec_skip = 0;  // test / experiment switches (omf_plan_set_debug), 0 in production
  // The bracket's width in sigmas (OMF_SPEC_ZSIG overrides both): a tensor whose norm falls
  // outside is requantised whole by the finish (exact; a miss per tensor at z sigmas has
  // probability ~erfc(z / sqrt 2): 6e-5 at 4, 6e-7 at 5), and a narrower bracket lists fewer
  // undecided quads.  scripts/exp/zsig_ab.sh, Llama-400M, two interleaved rounds: s = 4 encode
  // 0.349-0.352 ms at 5 sigmas against 0.357-0.361 at 6 (4: 0.350); s = 8 0.546-0.547 ms at 4
  // against 0.556-0.559 at 5 (3.5: 0.542-0.545).
  float spec_zsig = 5.0f;
  float spec_zsig_wide = 4.0f;
  SpecBracket* d_spec_br = nullptr;
  uint64_t* d_spec_ngran = nullptr;  // per tensor {epoch << 1 | bad, norm} granules of the fold
  uint64_t* d_spec_part = nullptr;
  uint32_t* d_spec_slots = nullptr;
  uint32_t* d_spec_heads = nullptr;
  float4* d_spec_recs = nullptr;  // listed quads' x and draws (32 B each)
  uint32_t* d_spec_slots_w = nullptr;  // the wide-level capacity (kSpecPerWaveWide), made at the first
  float4* d_spec_recs_w = nullptr;     // wide encode (bit_width 5-8)
  double* d_spec_br_part = nullptr;    // wide: the bracket parts' partial sums and arrival counters
  uint32_t* d_spec_br_cnt = nullptr;
  // the fused-bracket pass (OMF_SPEC_FB=0 / omf_plan_set_fused_bracket turn it off): Llama-400M s = 4
  // step 0.6977-0.7021 ms against 0.7009-0.7067 with the bracket's own launch (three interleaved
  // pairs), the encode alone unchanged (0.348-0.360 both); profiles/r05_fused_bracket_ab.txt
  int32_t spec_fb = 1;
  double* d_spec_fb_part = nullptr;    // its parts' partial sums, arrival counters and granules
  uint32_t* d_spec_fb_cnt = nullptr;
  uint64_t* d_spec_brgran = nullptr;
  int32_t spec_last_pw = kSpecPerWave;  // the list capacity of the latest bracketed encode
  int32_t spec_wide = 1;  // wide levels (5-8 bits, fp32) through the bracket (1) or as before (0): OMF_SPEC_WIDE
  // arena-aligned decoder: per 4 Ki block, tensor id | (1 << 31 when inside it)
  int64_t n_dec_blocks = 0;
  uint32_t* d_dec_binfo = nullptr;
  uint32_t* d_spec_flags = nullptr;
  uint32_t* d_spec_status = nullptr;
  // grid encoder (strategy 4): one workgroup per CU, kGridNB 4 Ki blocks per quarter
  int32_t grid_wgs = 0;             // workgroups of a launch (CUs; 0 = unavailable)
  uint32_t* d_grid_pbeg = nullptr;  // per tensor: first flat item (one partial per item)
  uint32_t* d_grid_pcnt = nullptr;  // per tensor: flat items
  unsigned long long* d_grid_bar = nullptr;  // arrival counter (zeroed at upload)
  uint64_t grid_launches = 0;
  // Top-K tiled decode: per-ratio constant tables (omf_topk.hip), allocated on first use, with
  // one host word each (the table's size facts)
  struct TopkTable {
    uint64_t key;
    void* dev;
    uint64_t host;
    std::vector<int64_t> counts;  // tables keyed by explicit per-tensor counts: the exact counts
  };
  std::vector<TopkTable> topk_tables;
  omf::TopkKnobs topk_knobs;
  // Launches that use the sync block / granules are ordered across streams: a launch on a
  // stream other than the previous one first waits for the previous launch's event.
  hipEvent_t last_ev = nullptr;
  hipStream_t last_stream = nullptr;
  bool last_valid = false;
};

// Order this launch after the plan's previous stateful launch when the stream changes: the event is
// recorded on the previous stream at the switch (it covers everything enqueued there so far, the
// plan's launches included), not after every call — an event packet between two kernels of one
// stream idled the GPU ~5 us per encode even without a system-scope fence (rocprofv3 kernel trace).
// So the previous stream must still exist when the plan moves to another one (include/omf_codec.h).
static int plan_enter(omf_plan* p, hipStream_t st) {
  if (p->last_valid && p->last_stream != st) {
    if (!p->last_ev) OMF_HIP(hipEventCreateWithFlags(&p->last_ev, kOrderEventFlags));
    OMF_HIP(hipEventRecord(p->last_ev, p->last_stream));
    OMF_HIP(hipStreamWaitEvent(st, p->last_ev, 0));
  }
  return OMF_OK;
}
static int plan_leave(omf_plan* p, hipStream_t st) {
  p->last_stream = st;
  p->last_valid = true;
  return OMF_OK;
}

// Plan internals shared with omf_topk.hip.
namespace omf_plan_access {
const void* flat_items(const omf_plan* p, int64_t* n) {
  *n = p->n_flat;
  return p->d_flat;
}
int32_t ntensors(const omf_plan* p) { return p->nt; }
int device(const omf_plan* p) { return p->device; }
int64_t arena_end(const omf_plan* p) { return p->arena_end; }
// The decoder's block table (tensor id | bit 31 = the block lies inside it) and its block size.
const uint32_t* dec_blocks(const omf_plan* p, int64_t* n, int64_t* block_elems) {
  *n = p->n_dec_blocks;
  *block_elems = kDecBlk;
  return p->d_dec_binfo;
}
const int64_t* d_sizes(const omf_plan* p) { return p->d_sizes; }
const int64_t* d_begins(const omf_plan* p) { return p->d_begins; }
const std::vector<int64_t>& sizes(const omf_plan* p) { return p->sizes; }
// A plan-owned device buffer of `bytes` for `key` (allocated, and *fresh set, on first use;
// not on the hot path after that), with a host word the caller keeps beside it.  nullptr if
// the allocation fails.
void* topk_table(omf_plan* p, uint64_t key, size_t bytes, bool* fresh, uint64_t** host) {
  *fresh = false;
  for (auto& e : p->topk_tables)
    if (e.key == key) {
      *host = &e.host;
      return e.dev;
    }
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
  p->topk_tables.push_back({key, d, 0, {}});
  *host = &p->topk_tables.back().host;
  *fresh = true;
  return d;
}
// The same for tables keyed by an explicit per-tensor count vector (a received Top-K message's
// k_t): matched on the exact counts.  At most kMaxCountTables are kept; making one more frees the
// oldest (hipFree waits for the device, so no queued launch still reads it).
void* topk_table_counts(omf_plan* p, const int64_t* counts, size_t bytes, bool* fresh, uint64_t** host) {
  constexpr uint64_t kCountsKey = 0xC0C0C0C0C0C0C0C0ull;
  constexpr int kMaxCountTables = 8;
  *fresh = false;
  const size_t nt = (size_t)p->nt;
  int held = 0;
  for (auto& e : p->topk_tables) {
    if (e.key != kCountsKey) continue;
    ++held;
    if (e.counts.size() == nt && std::equal(e.counts.begin(), e.counts.end(), counts)) {
      *host = &e.host;
      return e.dev;
    }
  }
  if (held >= kMaxCountTables) {
    for (auto it = p->topk_tables.begin(); it != p->topk_tables.end(); ++it)
      if (it->key == kCountsKey) {
        (void)hipFree(it->dev);
        p->topk_tables.erase(it);
        break;
      }
  }
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
  p->topk_tables.push_back({kCountsKey, d, 0, std::vector<int64_t>(counts, counts + nt)});
  *host = &p->topk_tables.back().host;
  *fresh = true;
  return d;
}
const std::vector<int64_t>& offsets(const omf_plan* p) { return p->offsets; }
omf::TopkKnobs& topk_knobs(omf_plan* p) { return p->topk_knobs; }
// The plan's device error word (omf_plan_check reports and clears it).
uint32_t* err_word(omf_plan* p) { return reinterpret_cast<uint32_t*>(p->d_sync + 4); }
// Stream ordering of a stateful launch outside this file (plan_enter / plan_leave).
int order_enter(omf_plan* p, hipStream_t st) { return plan_enter(p, st); }
int order_leave(omf_plan* p, hipStream_t st) { return plan_leave(p, st); }
}  // namespace omf_plan_access

static size_t round16(size_t b) { return (b + 15) & ~(size_t)15; }

static bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

// Ticket-order item sequence.  Register-resident tensors (<= cap items of kSub) are
// emitted in place; a larger tensor emits its NORM items in place and its QUANT items
// after the next tensor's items (one tensor of slack for the norm hand-off).
static void build_sequence(const omf_plan& p, bool resident_ok, std::vector<Item>& seq,
                           std::vector<TensorInfo>& tinfo, int64_t& npart) {
  seq.clear();
  tinfo.assign(p.nt, TensorInfo{});
  npart = 0;
  std::vector<Item> deferred;
  for (int32_t t = 0; t < p.nt; ++t) {
    const int64_t n = p.sizes[t], b = p.offsets[t];
    const int64_t es = (int64_t)p.ev * 1024;
    const int64_t ns = (n + es - 1) / es;
    std::vector<Item> q_t;
    if (ns == 1 || (resident_ok && ns <= p.cap)) {
      tinfo[t] = TensorInfo{b, n, es, (int32_t)ns, (int32_t)npart};
      for (int64_t c = 0; c < ns; ++c) {
        const int64_t cb = b + c * es;
        seq.push_back(Item{cb, std::min(b + n, cb + es), t, kResident, (int32_t)c, 0});
      }
      npart += ns;
    } else {
      const int64_t nc = (n + p.chunk - 1) / p.chunk;
      tinfo[t] = TensorInfo{b, n, p.chunk, (int32_t)nc, (int32_t)npart};
      for (int64_t c = 0; c < nc; ++c) {
        const int64_t cb = b + c * p.chunk, ce = std::min(b + n, cb + p.chunk);
        seq.push_back(Item{cb, ce, t, kNorm, (int32_t)c, 0});
        q_t.push_back(Item{cb, ce, t, kQuant, (int32_t)c, 0});
      }
      npart += nc;
    }
    seq.insert(seq.end(), deferred.begin(), deferred.end());
    deferred.swap(q_t);
  }
  seq.insert(seq.end(), deferred.begin(), deferred.end());
}

// Ring sequence: tensors of <= ring_hold_max chunks are HOLD chunks (read once);
// larger ones are NORM chunks (partial only) plus QUANT chunks (second read), the QUANT
// chunks placed ring_gap items later (big_mode 0) or at the very end with every NORM
// chunk first (big_mode 1).  Items are dealt to workgroups round-robin.
// Register-resident encoder (omf_qsgd_ring.hip qsgd_encode_rr): every single-read tensor
// lies inside one row of `grid` consecutive items, so all its chunks are at the same
// position of their workgroups.  Rows are packed first-fit decreasing; gaps are filled
// with NORM items of the multi-row ("big") tensors, or with empty items when none are
// left.  Layout: [whole rows of big NORM items][packed rows][remaining big NORM items]
// [big QUANT items] — every NORM item precedes its tensor's QUANT items.
static void build_rr_sequence(omf_plan& p, int64_t ch, std::vector<omf::ring::Item>& seq,
                              std::vector<omf::ring::Tensor>& tens) {
  namespace R = omf::ring;
  const int64_t G = std::max<int32_t>(p.ring_grid, 1);
  p.ring_hold_max = p.ring_hold_override > 0 ? std::min<int64_t>(G, p.ring_hold_override) : G;
  seq.clear();
  tens.assign(p.nt, R::Tensor{});
  std::vector<R::Item> norm_items, quant_items;
  std::vector<std::pair<int64_t, int32_t>> regular;  // (chunks, tensor)
  int64_t gb = 0;
  p.ring_two_pass = 0;
  auto item = [&](int32_t t, int64_t k, int32_t flags) {
    const int64_t n = p.sizes[t], b = p.offsets[t], cb = b + k * ch;
    return R::Item{cb, std::min(b + n, cb + ch), b, n, t, flags, (int32_t)k, tens[t].nchunks, tens[t].gbase, {0, 0, 0}};
  };
  for (int32_t t = 0; t < p.nt; ++t) {
    const int64_t nc = (p.sizes[t] + ch - 1) / ch;
    tens[t] = R::Tensor{p.offsets[t], p.sizes[t], (int32_t)nc, (int32_t)gb, {0, 0}};
    gb += nc;
    if (nc <= p.ring_hold_max) {
      regular.emplace_back(nc, t);
    } else {
      ++p.ring_two_pass;
      for (int64_t k = 0; k < nc; ++k) norm_items.push_back(item(t, k, R::kPublish));
      for (int64_t k = 0; k < nc; ++k) quant_items.push_back(item(t, k, R::kQuant));
    }
  }
  std::stable_sort(regular.begin(), regular.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
  std::vector<std::vector<int32_t>> rows;
  std::vector<int64_t> room;
  for (const auto& r : regular) {
    size_t i = 0;
    while (i < rows.size() && room[i] < r.first) ++i;
    if (i == rows.size()) {
      rows.emplace_back();
      room.push_back(G);
    }
    rows[i].push_back(r.second);
    room[i] -= r.first;
  }
  // Gap fillers come from the back of the NORM list; whole rows of the rest lead.
  size_t nfill = 0;
  for (size_t i = 0; i + 1 < rows.size(); ++i) nfill += (size_t)room[i];
  nfill = std::min(nfill, norm_items.size());
  const size_t avail = norm_items.size() - nfill;
  const size_t lead = avail / (size_t)G * (size_t)G;
  seq.insert(seq.end(), norm_items.begin(), norm_items.begin() + (ptrdiff_t)lead);
  size_t tail = lead;                           // next NORM item not yet placed (after the lead rows)
  size_t fill = norm_items.size() - nfill;      // next gap filler
  for (size_t i = 0; i < rows.size(); ++i) {
    for (int32_t t : rows[i])
      for (int64_t k = 0; k < tens[t].nchunks; ++k) seq.push_back(item(t, k, R::kPublish | R::kQuant));
    if (i + 1 < rows.size()) {
      for (int64_t g = 0; g < room[i]; ++g) {
        if (fill < norm_items.size()) seq.push_back(norm_items[fill++]);
        else seq.push_back(R::Item{0, 0, 0, 0, 0, 0, 0, 0, 0, {0, 0, 0}});  // empty: keeps rows aligned
      }
    }
  }
  seq.insert(seq.end(), norm_items.begin() + (ptrdiff_t)tail, norm_items.begin() + (ptrdiff_t)(norm_items.size() - nfill));
  seq.insert(seq.end(), quant_items.begin(), quant_items.end());
  p.n_ring_gran = std::max<int64_t>(gb, 1);
}

static void build_ring_sequence(omf_plan& p, std::vector<omf::ring::Item>& seq,
                                std::vector<omf::ring::Tensor>& tens) {
  namespace R = omf::ring;
  const R::Config c = R::config(p.ring_cfg);
  const int64_t ch = R::chunk_elems(c);
  if (c.kind == 1) return build_rr_sequence(p, ch, seq, tens);
  p.ring_hold_max = p.ring_hold_override > 0 ? p.ring_hold_override : (int64_t)c.slots * p.ring_grid;
  const int64_t gap = p.ring_gap >= 0 ? p.ring_gap : p.ring_grid;
  seq.clear();
  tens.assign(p.nt, R::Tensor{});
  std::vector<R::Item> front, back;
  std::vector<std::pair<int64_t, std::vector<R::Item>>> pending;  // (insert when seq.size() >= first, items)
  int64_t gb = 0;
  p.ring_two_pass = 0;
  auto flush = [&](bool all) {
    for (size_t i = 0; i < pending.size();) {
      if (all || (int64_t)seq.size() >= pending[i].first) {
        seq.insert(seq.end(), pending[i].second.begin(), pending[i].second.end());
        pending.erase(pending.begin() + i);
      } else {
        ++i;
      }
    }
  };
  for (int32_t t = 0; t < p.nt; ++t) {
    const int64_t n = p.sizes[t], b = p.offsets[t];
    const int64_t nc = (n + ch - 1) / ch;
    tens[t] = R::Tensor{b, n, (int32_t)nc, (int32_t)gb, {0, 0}};
    gb += nc;
    const bool big = nc > p.ring_hold_max;
    std::vector<R::Item> quant;
    for (int64_t k = 0; k < nc; ++k) {
      const int64_t cb = b + k * ch, ce = std::min(b + n, cb + ch);
      if (!big) {
        seq.push_back(R::Item{cb, ce, b, n, t, R::kPublish | R::kQuant, (int32_t)k, (int32_t)nc, (int32_t)(gb - nc), {0, 0, 0}});
        flush(false);
      } else {
        const R::Item norm_it{cb, ce, b, n, t, R::kPublish, (int32_t)k, (int32_t)nc, (int32_t)(gb - nc), {0, 0, 0}};
        if (p.ring_big_mode == 1) front.push_back(norm_it);
        else seq.push_back(norm_it);
        quant.push_back(R::Item{cb, ce, b, n, t, R::kQuant, (int32_t)k, (int32_t)nc, (int32_t)(gb - nc), {0, 0, 0}});
      }
    }
    if (big) {
      ++p.ring_two_pass;
      if (p.ring_big_mode == 1) back.insert(back.end(), quant.begin(), quant.end());
      else pending.emplace_back((int64_t)seq.size() + gap, std::move(quant));
    }
  }
  flush(true);
  if (p.ring_big_mode == 1) {
    seq.insert(seq.begin(), front.begin(), front.end());
    seq.insert(seq.end(), back.begin(), back.end());
  }
  p.n_ring_gran = std::max<int64_t>(gb, 1);
}

// (Re)build both sequences and upload every table into one device allocation.
static int upload_plan(omf_plan* p) {
  std::vector<Item> seq[2], flat;
  std::vector<TensorInfo> tinfo[2];
  int64_t np[2];
  build_sequence(*p, true, seq[0], tinfo[0], np[0]);
  build_sequence(*p, false, seq[1], tinfo[1], np[1]);
  std::vector<omf::ring::Item> rseq;
  std::vector<omf::ring::Tensor> rtens;
  build_ring_sequence(*p, rseq, rtens);
  p->n_ring = (int64_t)rseq.size();
  // Flat items (decode, norm-supplied quantise, Top-K passes): one 16 Ki sub-chunk each,
  // the fastest decode granularity measured (profiles/r01_notes.md).
  // Bracketed encoder tables: one bracket item per tensor (one workgroup writes its bracket)
  // and fold segments of kSpecSeg wave partials (4 per 4 Ki block, kSub / kSpecBlk = 4 blocks
  // per flat item).
  std::vector<SpecBrItem> br_items;
  std::vector<SpecFoldItem> fold_items;
  std::vector<uint32_t> gpbeg((size_t)p->nt), gpcnt((size_t)p->nt);
  int32_t seg_base = 0;
  for (int32_t t = 0; t < p->nt; ++t) {
    const int64_t n = p->sizes[t], b = p->offsets[t];
    const int64_t p_begin = (int64_t)kWaves * 4 * (int64_t)flat.size();
    for (int64_t c = 0; c * kSub < n; ++c) {
      const int64_t cb = b + c * kSub;
      flat.push_back(Item{cb, std::min(b + n, cb + kSub), t, kQuant, (int32_t)c, 0});
    }
    const int64_t p_end = (int64_t)kWaves * 4 * (int64_t)flat.size();
    gpbeg[(size_t)t] = (uint32_t)(p_begin / (kWaves * 4));  // the grid encoder: one partial per item
    gpcnt[(size_t)t] = (uint32_t)((p_end - p_begin) / (kWaves * 4));
    const int64_t R = std::max<int64_t>(1, std::min<int64_t>(kSpecRuns, n / (2 * kSpecRun)));
    const int64_t Rw = std::max<int64_t>(1, std::min<int64_t>(kSpecRunsWide, n / (2 * kSpecRunWide)));
    br_items.push_back(SpecBrItem{b, n, n / R, (int32_t)R, (int32_t)(n % R), t, (int32_t)Rw});
    const int32_t nsegs = (int32_t)((p_end - p_begin + kSpecSeg - 1) / kSpecSeg);
    for (int32_t q = 0; q < nsegs; ++q)
      fold_items.push_back(SpecFoldItem{p_begin + (int64_t)q * kSpecSeg, std::min(p_end, p_begin + (int64_t)(q + 1) * kSpecSeg),
                                        t, q, nsegs, seg_base});
    seg_base += nsegs;
  }
  static_assert(kSub == 4 * kSpecBlk, "four spec blocks per flat item");
  // decoder block table: the last tensor starting at or before the block, and whether the
  // block lies entirely inside it
  std::vector<uint32_t> binfo((size_t)((p->arena_end + kDecBlk - 1) / kDecBlk));
  {
    int32_t t = 0;
    for (size_t k = 0; k < binfo.size(); ++k) {
      const int64_t base = (int64_t)k * kDecBlk;
      while (t + 1 < p->nt && p->offsets[t + 1] <= base) ++t;
      const bool inside = p->offsets[t] <= base && base + kDecBlk <= p->offsets[t] + p->sizes[t];
      binfo[k] = (uint32_t)t | (inside ? 0x80000000u : 0u);
    }
  }
  p->n_dec_blocks = (int64_t)binfo.size();
  p->n_spec_blocks = 4 * (int64_t)flat.size();
  p->n_spec_br = (int64_t)br_items.size();
  p->n_spec_fold = (int64_t)fold_items.size();
  if ((int64_t)std::max(seq[0].size(), 4 * flat.size()) > 0x7fffffffLL) return fail(OMF_EINVAL, "too many work items");
  p->n_enc[0] = (int64_t)seq[0].size();
  p->n_enc[1] = (int64_t)seq[1].size();
  p->n_flat = (int64_t)flat.size();
  p->n_partials = std::max<int64_t>(std::max(np[0], np[1]), 1);
  p->off_counters = 16;
  p->off_gran = round16(p->off_counters + 4 * (size_t)p->nt);
  p->sync_bytes = round16(p->off_gran + 8 * (size_t)p->nt);
  // the sync block starts the allocation (its per-call memset is 16-byte aligned and sized)
  size_t o = round16(p->sync_bytes);
  const size_t o_enc0 = o; o = round16(o + sizeof(Item) * seq[0].size());
  const size_t o_enc1 = o; o = round16(o + sizeof(Item) * seq[1].size());
  const size_t o_flat = o; o = round16(o + sizeof(Item) * flat.size());
  const size_t o_ti0 = o; o = round16(o + sizeof(TensorInfo) * p->nt);
  const size_t o_ti1 = o; o = round16(o + sizeof(TensorInfo) * p->nt);
  const size_t o_part = o; o = round16(o + 8 * (size_t)p->n_partials);
  const size_t o_sizes = o; o = round16(o + 8 * (size_t)p->nt);
  const size_t o_begins = o; o = round16(o + 8 * (size_t)p->nt);
  const size_t o_ring = o; o = round16(o + sizeof(omf::ring::Item) * rseq.size());
  const size_t o_ring_t = o; o = round16(o + sizeof(omf::ring::Tensor) * rtens.size());
  const size_t o_ring_g = o; o = round16(o + 8 * (size_t)p->n_ring_gran);
  const size_t o_ring_p = o; o = round16(o + 8 * 16);
  const size_t o_sp_bri = o; o = round16(o + sizeof(SpecBrItem) * br_items.size());
  const size_t o_sp_foi = o; o = round16(o + sizeof(SpecFoldItem) * fold_items.size());
  const size_t o_sp_segp = o; o = round16(o + 8 * fold_items.size());
  const size_t o_sp_cnt = o; o = round16(o + 4 * (size_t)p->nt + 4);
  const size_t o_sp_br = o; o = round16(o + sizeof(SpecBracket) * (size_t)p->nt);
  const size_t o_sp_ngran = o; o = round16(o + 8 * (size_t)p->nt);
  const size_t o_sp_part = o; o = round16(o + 8 * (size_t)kWaves * (size_t)p->n_spec_blocks);
  const size_t o_sp_slots = o; o = round16(o + 4 * (size_t)kSpecSlot * (size_t)p->n_spec_blocks);
  const size_t o_sp_heads = o; o = round16(o + 4 * (size_t)kWaves * (size_t)p->n_spec_blocks);
  const size_t o_binfo = o; o = round16(o + 4 * binfo.size());
  const size_t o_sp_recs = o; o = round16(o + 32 * (size_t)kWaves * kSpecPerWave * (size_t)p->n_spec_blocks);
  const size_t o_sp_flags = o; o = round16(o + 4 * (size_t)p->nt);
  const size_t o_sp_status = o; o = round16(o + 4 * (size_t)p->nt);
  const size_t o_g_pbeg = o; o = round16(o + 4 * (size_t)p->nt);
  const size_t o_g_pcnt = o; o = round16(o + 4 * (size_t)p->nt);
  const size_t o_g_bar = o; o = round16(o + 16);
  DeviceGuard g(p->device);
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  if (p->d_block) {
    OMF_HIP(hipDeviceSynchronize());
    (void)hipFree(p->d_block);
    p->d_block = nullptr;
  }
  OMF_HIP(hipMalloc(&p->d_block, o));
  uint8_t* base = static_cast<uint8_t*>(p->d_block);
  p->d_sync = base;
  p->d_enc[0] = reinterpret_cast<Item*>(base + o_enc0);
  p->d_enc[1] = reinterpret_cast<Item*>(base + o_enc1);
  p->d_flat = reinterpret_cast<Item*>(base + o_flat);
  p->d_tinfo[0] = reinterpret_cast<TensorInfo*>(base + o_ti0);
  p->d_tinfo[1] = reinterpret_cast<TensorInfo*>(base + o_ti1);
  p->d_partials = reinterpret_cast<uint64_t*>(base + o_part);
  p->d_sizes = reinterpret_cast<int64_t*>(base + o_sizes);
  p->d_begins = reinterpret_cast<int64_t*>(base + o_begins);
  p->d_ring = reinterpret_cast<omf::ring::Item*>(base + o_ring);
  p->d_ring_t = reinterpret_cast<omf::ring::Tensor*>(base + o_ring_t);
  p->d_ring_gran = reinterpret_cast<uint64_t*>(base + o_ring_g);
  p->d_ring_prof = reinterpret_cast<unsigned long long*>(base + o_ring_p);
  p->d_spec_br_items = reinterpret_cast<SpecBrItem*>(base + o_sp_bri);
  p->d_spec_fold_items = reinterpret_cast<SpecFoldItem*>(base + o_sp_foi);
  p->d_spec_seg_part = reinterpret_cast<uint64_t*>(base + o_sp_segp);
  p->d_spec_cnt = reinterpret_cast<uint32_t*>(base + o_sp_cnt);
  p->d_spec_br = reinterpret_cast<SpecBracket*>(base + o_sp_br);
  p->d_spec_ngran = reinterpret_cast<uint64_t*>(base + o_sp_ngran);
  p->d_spec_part = reinterpret_cast<uint64_t*>(base + o_sp_part);
  p->d_spec_slots = reinterpret_cast<uint32_t*>(base + o_sp_slots);
  p->d_spec_heads = reinterpret_cast<uint32_t*>(base + o_sp_heads);
  p->d_dec_binfo = reinterpret_cast<uint32_t*>(base + o_binfo);
  OMF_HIP(hipMemcpy(p->d_dec_binfo, binfo.data(), 4 * binfo.size(), hipMemcpyHostToDevice));
  p->d_spec_recs = reinterpret_cast<float4*>(base + o_sp_recs);
  p->d_spec_flags = reinterpret_cast<uint32_t*>(base + o_sp_flags);
  p->d_spec_status = reinterpret_cast<uint32_t*>(base + o_sp_status);
  p->d_grid_pbeg = reinterpret_cast<uint32_t*>(base + o_g_pbeg);
  p->d_grid_pcnt = reinterpret_cast<uint32_t*>(base + o_g_pcnt);
  p->d_grid_bar = reinterpret_cast<unsigned long long*>(base + o_g_bar);
  OMF_HIP(hipMemcpy(p->d_grid_pbeg, gpbeg.data(), 4 * gpbeg.size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_grid_pcnt, gpcnt.data(), 4 * gpcnt.size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemset(p->d_grid_bar, 0, 16));
  p->grid_launches = 0;
  OMF_HIP(hipMemcpy(p->d_spec_br_items, br_items.data(), sizeof(SpecBrItem) * br_items.size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_spec_fold_items, fold_items.data(), sizeof(SpecFoldItem) * fold_items.size(),
                    hipMemcpyHostToDevice));
  OMF_HIP(hipMemset(p->d_spec_cnt, 0, 4 * (size_t)p->nt + 4));
  OMF_HIP(hipMemset(p->d_spec_flags, 0, 4 * (size_t)p->nt));
  OMF_HIP(hipMemset(p->d_spec_status, 0, 4 * (size_t)p->nt));  // spec_stats reads them before any encode
  OMF_HIP(hipMemset(p->d_spec_ngran, 0, 8 * (size_t)p->nt));  // epoch 0 is never a launch's tag
  OMF_HIP(hipMemset(p->d_ring_prof, 0, 8 * 16));
  OMF_HIP(hipMemcpy(p->d_enc[0], seq[0].data(), sizeof(Item) * seq[0].size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_enc[1], seq[1].data(), sizeof(Item) * seq[1].size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_flat, flat.data(), sizeof(Item) * flat.size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_tinfo[0], tinfo[0].data(), sizeof(TensorInfo) * p->nt, hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_tinfo[1], tinfo[1].data(), sizeof(TensorInfo) * p->nt, hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_sizes, p->sizes.data(), 8 * (size_t)p->nt, hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_begins, p->offsets.data(), 8 * (size_t)p->nt, hipMemcpyHostToDevice));
  if (!rseq.empty())
    OMF_HIP(hipMemcpy(p->d_ring, rseq.data(), sizeof(omf::ring::Item) * rseq.size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemcpy(p->d_ring_t, rtens.data(), sizeof(omf::ring::Tensor) * rtens.size(), hipMemcpyHostToDevice));
  OMF_HIP(hipMemset(p->d_ring_gran, 0, 8 * (size_t)p->n_ring_gran));  // epoch 0 is never a launch's tag
  OMF_HIP(hipMemset(p->d_sync, 0, p->sync_bytes));
  return OMF_OK;
}

extern "C" {

int omf_plan_create(const int64_t* sizes, const int64_t* offsets, int32_t ntensors, int64_t chunk_elems, int device,
                    omf_plan** out) {
  if (!out) return fail(OMF_EINVAL, "omf_plan_create: out is NULL");
  *out = nullptr;
  if (ntensors <= 0 || !sizes || !offsets) return fail(OMF_EINVAL, "omf_plan_create: need >= 1 tensor");
  if (ntensors >= (1 << 24)) return fail(OMF_EINVAL, "omf_plan_create: at most 2^24 - 1 tensors");
  if (chunk_elems == 0) chunk_elems = 2 * kSub;  // two-pass encode items: 128 KiB of fp32 (32 Ki: 0.579 vs
                                                 // 0.595 ms at 64 Ki on Llama-400M, scripts/exp/ab_chunk.py)
  if (chunk_elems < kSub || chunk_elems % kSub != 0)
    return fail(OMF_EINVAL, "omf_plan_create: chunk_elems must be a positive multiple of 16384");
  for (int32_t t = 0; t < ntensors; ++t) {
    if (sizes[t] <= 0 || offsets[t] < 0 || (offsets[t] & 3))
      return fail(OMF_EINVAL, "omf_plan_create: tensor " + std::to_string(t) +
                                  ": size must be > 0 and offset a non-negative multiple of 4");
    if (t > 0 && offsets[t] < offsets[t - 1] + sizes[t - 1])
      return fail(OMF_EINVAL, "omf_plan_create: tensors must be ordered and non-overlapping");
  }
  auto* p = new (std::nothrow) omf_plan();
  if (!p) return fail(OMF_ENOMEM, "omf_plan_create: host allocation failed");
  p->device = device;
  p->nt = ntensors;
  p->chunk = chunk_elems;
  p->sizes.assign(sizes, sizes + ntensors);
  p->offsets.assign(offsets, offsets + ntensors);
  p->arena_end = offsets[ntensors - 1] + sizes[ntensors - 1];
  {
    // Co-resident capacity of the encoder (occupancy x CUs over every instantiation); a
    // tensor takes the register-resident path only with half of it as margin.
    DeviceGuard g(device);
    hipDeviceProp_t prop;
    if (!g.ok || hipGetDeviceProperties(&prop, device) != hipSuccess) {
      delete p;
      return fail(OMF_EHIP, "omf_plan_create: cannot query the device");
    }
    if (const char* ev = omf::knob("OMF_ENCODE_ROWS")) p->ev = atoi(ev) == 16 ? 16 : 8;  // tuning knob
    const void* k16[5] = {(const void*)qsgd_encode_ordered<1, false, false, 16>,
                          (const void*)qsgd_encode_ordered<1, true, false, 16>,
                          (const void*)qsgd_encode_ordered<4, false, false, 16>,
                          (const void*)qsgd_encode_ordered<4, true, false, 16>,
                          (const void*)qsgd_encode_ordered<1, false, true, 16>};
    const void* k8[5] = {(const void*)qsgd_encode_ordered<1, false, false, 8>,
                         (const void*)qsgd_encode_ordered<1, true, false, 8>,
                         (const void*)qsgd_encode_ordered<4, false, false, 8>,
                         (const void*)qsgd_encode_ordered<4, true, false, 8>,
                         (const void*)qsgd_encode_ordered<1, false, true, 8>};
    const void* const* kerns = p->ev == 8 ? k8 : k16;
    int nb_min = 1 << 30;
    for (int i = 0; i < 5; ++i) {
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kerns[i], kThreads, 0) != hipSuccess || nb < 1) nb = 1;
      nb_min = std::min(nb_min, nb);
    }
    p->cap = std::max<int64_t>(1, (int64_t)nb_min * prop.multiProcessorCount / 2);
    // Ring encoder: configuration and grid (tuning knobs for experiments only).
    if (const char* rc = omf::knob("OMF_RING_CFG")) p->ring_cfg = std::max(0, std::min(atoi(rc), omf::ring::num_configs() - 1));
    if (const char* bm = omf::knob("OMF_RING_BIG")) p->ring_big_mode = atoi(bm) == 1 ? 1 : 0;
    if (const char* gp = omf::knob("OMF_RING_GAP")) p->ring_gap = atoll(gp);
    // Switches that change what an encode writes (skipped launches, no quantisation) are never
    // read from the environment of a release build: tests set them per plan (omf_plan_set_debug);
    // experiment builds (-DOMF_EXPERIMENTS, scripts/exp/build_variants.sh) also take them here.
#ifdef OMF_EXPERIMENTS
    if (const char* dg = omf::knob("OMF_RING_DBG")) p->ring_dbg = (uint32_t)atoi(dg);
    if (const char* sk = omf::knob("OMF_SPEC_SKIP")) p->spec_skip = (uint32_t)atoi(sk);
#endif
    if (const char* zs = omf::knob("OMF_SPEC_ZSIG")) p->spec_zsig = p->spec_zsig_wide = std::max(1.0f, (float)atof(zs));
    // Default strategy by arena size: the bracketed single-read encoder from 2^25 elements
    // (Llama-400M 0.386 ms against the two-pass 0.59 and the ring 0.63; Llama-150M 0.25 against
    // 0.35), the ring below (ResNet-18: 0.032 ms against 0.08 for the bracket's four launches).
    p->strategy = p->arena_end >= ((int64_t)1 << 25) ? 3 : 2;
    if (const char* st = omf::knob("OMF_ENCODE_STRATEGY")) p->strategy = std::max(0, std::min(atoi(st), 4));
    if (const char* sw = omf::knob("OMF_SPEC_WIDE")) p->spec_wide = atoi(sw) != 0 ? 1 : 0;
    if (const char* fb = omf::knob("OMF_SPEC_FB")) p->spec_fb = atoi(fb) != 0 ? 1 : 0;
    {  // grid encoder: one 1024-thread workgroup per CU must fit
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)qsgd_encode_grid<1>, 1024, 0) == hipSuccess &&
          nb >= 1)
        p->grid_wgs = prop.multiProcessorCount;
    }
    p->ring_grid = omf::ring::grid_size(p->ring_cfg, device);
    if (p->ring_grid <= 0) {
      delete p;
      return fail(OMF_EHIP, "omf_plan_create: cannot size the ring encoder grid");
    }
  }
  if (int r = upload_plan(p)) {
    if (p->d_block) (void)hipFree(p->d_block);
    delete p;
    return r;
  }
  *out = p;
  return OMF_OK;
}

int omf_plan_destroy(omf_plan* plan) {
  if (!plan) return OMF_OK;
  DeviceGuard g(plan->device);
  if (plan->last_ev) (void)hipEventDestroy(plan->last_ev);
  if (plan->d_block) (void)hipFree(plan->d_block);
  if (plan->d_spec_slots_w) (void)hipFree(plan->d_spec_slots_w);
  if (plan->d_spec_recs_w) (void)hipFree(plan->d_spec_recs_w);
  if (plan->d_spec_br_part) (void)hipFree(plan->d_spec_br_part);
  if (plan->d_spec_br_cnt) (void)hipFree(plan->d_spec_br_cnt);
  if (plan->d_spec_fb_part) (void)hipFree(plan->d_spec_fb_part);
  if (plan->d_spec_fb_cnt) (void)hipFree(plan->d_spec_fb_cnt);
  if (plan->d_spec_brgran) (void)hipFree(plan->d_spec_brgran);
  for (auto& e : plan->topk_tables) (void)hipFree(e.dev);
  delete plan;
  return OMF_OK;
}

int64_t omf_plan_encode_items(const omf_plan* plan) {
  if (!plan) return -1;
  if (plan->strategy == 3) return plan->n_spec_blocks;
  if (plan->strategy == 4) return plan->grid_wgs;
  return plan->strategy == 2 ? plan->n_ring : plan->n_enc[plan->strategy];
}

int32_t omf_plan_encode_strategy(const omf_plan* plan) { return plan ? plan->strategy : -1; }
int32_t omf_plan_last_encoder(const omf_plan* plan) { return plan ? plan->last_encoder : -1; }
int omf_plan_set_fused_bracket(omf_plan* plan, int32_t on) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  plan->spec_fb = on != 0 ? 1 : 0;
  return OMF_OK;
}
int omf_plan_set_wide_levels(omf_plan* plan, int32_t on) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  plan->spec_wide = on != 0 ? 1 : 0;
  return OMF_OK;
}

int omf_plan_set_encode_strategy(omf_plan* plan, int32_t strategy) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  if (strategy < 0 || strategy > 4)
    return fail(OMF_EINVAL, "strategy must be 0 (resident), 1 (two-pass), 2 (single-read ring), 3 (bracketed "
                            "single-read) or 4 (grid)");
  plan->strategy = strategy;
  return OMF_OK;
}

int64_t omf_plan_resident_capacity(const omf_plan* plan) { return plan ? plan->cap : -1; }

int omf_plan_set_ring(omf_plan* plan, int32_t cfg, int32_t big_mode, int64_t gap, int64_t hold_max) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  if (cfg >= omf::ring::num_configs() || cfg < -1) return fail(OMF_EINVAL, "omf_plan_set_ring: bad configuration");
  if (big_mode < -1 || big_mode > 1 || gap < -2 || hold_max < -1)
    return fail(OMF_EINVAL, "omf_plan_set_ring: bad arguments");
  if (cfg >= 0 && cfg != plan->ring_cfg) {
    DeviceGuard g(plan->device);
    const int grid = omf::ring::grid_size(cfg, plan->device);
    if (grid <= 0) return fail(OMF_EHIP, "omf_plan_set_ring: cannot size the grid");
    plan->ring_cfg = cfg;
    plan->ring_grid = grid;
  }
  if (big_mode >= 0) plan->ring_big_mode = big_mode;
  if (gap >= -1) plan->ring_gap = gap;
  if (hold_max >= 0) plan->ring_hold_override = hold_max;
  return upload_plan(plan);
}

int omf_plan_ring_profile(omf_plan* plan, int64_t* out16) {
  if (!plan || !out16) return fail(OMF_EINVAL, "omf_plan_ring_profile: NULL argument");
  DeviceGuard g(plan->device);
  OMF_HIP(hipDeviceSynchronize());
  OMF_HIP(hipMemcpy(out16, plan->d_ring_prof, 8 * 16, hipMemcpyDeviceToHost));
  OMF_HIP(hipMemset(plan->d_ring_prof, 0, 8 * 16));
  return OMF_OK;
}

int omf_plan_ring_info(const omf_plan* plan, int64_t* out) {
  if (!plan || !out) return fail(OMF_EINVAL, "omf_plan_ring_info: NULL argument");
  out[0] = plan->ring_grid;
  out[1] = omf::ring::chunk_elems(omf::ring::config(plan->ring_cfg));
  out[2] = plan->n_ring;
  out[3] = plan->ring_hold_max;
  out[4] = plan->ring_two_pass;
  out[5] = plan->ring_cfg;
  return OMF_OK;
}

int omf_plan_set_resident_capacity(omf_plan* plan, int64_t cap, int64_t wait_us) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  if (cap < 0 || wait_us < 0) return fail(OMF_EINVAL, "cap and wait_us must be >= 0");
  if (cap > 0) plan->cap = cap;
  plan->wait_ticks = wait_us > 0 ? (uint64_t)wait_us * 100ull : kWaitTicks;
  if (cap > 0) return upload_plan(plan);
  return OMF_OK;
}

int omf_plan_set_debug(omf_plan* plan, uint32_t ring_dbg, uint32_t spec_dbg, int64_t lds_wait_us) {
  if (!plan) return fail(OMF_EINVAL, "plan is NULL");
  if (lds_wait_us < 0) return fail(OMF_EINVAL, "lds_wait_us must be >= 0");
  if ((ring_dbg & ~15u) || (spec_dbg & ~511u)) return fail(OMF_EINVAL, "omf_plan_set_debug: unknown switch bits");
  plan->ring_dbg = ring_dbg;
  plan->spec_skip = spec_dbg;
  plan->lds_wait_ticks = lds_wait_us > 0 ? (uint64_t)lds_wait_us * 100ull : kWaitTicks;
  return OMF_OK;
}

int omf_plan_spec_stats(omf_plan* plan, void* stream, int64_t* out4) {
  if (!plan || !out4) return fail(OMF_EINVAL, "omf_plan_spec_stats: NULL argument");
  DeviceGuard g(plan->device);
  OMF_HIP(hipStreamSynchronize((hipStream_t)stream));
  std::vector<uint32_t> status(plan->nt), heads((size_t)kWaves * (size_t)plan->n_spec_blocks);
  std::vector<SpecBracket> br(plan->nt);
  OMF_HIP(hipMemcpy(status.data(), plan->d_spec_status, 4 * (size_t)plan->nt, hipMemcpyDeviceToHost));
  OMF_HIP(hipMemcpy(br.data(), plan->d_spec_br, sizeof(SpecBracket) * (size_t)plan->nt, hipMemcpyDeviceToHost));
  OMF_HIP(hipMemcpy(heads.data(), plan->d_spec_heads, 4 * heads.size(), hipMemcpyDeviceToHost));
  int64_t whole = 0, deferred = 0, listed = 0, full = 0;
  for (int32_t t = 0; t < plan->nt; ++t) {
    whole += status[t] != 0u;
    deferred += br[t].mode != 0u;
  }
  for (int64_t blk = 0; blk < plan->n_spec_blocks; ++blk)
    for (int w = 0; w < kWaves; ++w) {
      const uint32_t c = heads[(size_t)blk * kWaves + w] & 0xffu;
      listed += c;
      full += c == (uint32_t)plan->spec_last_pw;
    }
  out4[0] = whole;
  out4[1] = deferred;
  out4[2] = listed;
  out4[3] = full;
  return OMF_OK;
}

int omf_plan_check(omf_plan* plan, void* stream) {
  if (!plan) return fail(OMF_EINVAL, "omf_plan_check: plan is NULL");
  DeviceGuard g(plan->device);
  OMF_HIP(hipStreamSynchronize((hipStream_t)stream));
  // the plan's launches on this stream are complete: a later call on another stream needs no
  // ordering against it (and the stream may now be destroyed)
  if (plan->last_valid && plan->last_stream == (hipStream_t)stream) plan->last_valid = false;
  uint32_t err = 0;
  OMF_HIP(hipMemcpy(&err, plan->d_sync + 4, 4, hipMemcpyDeviceToHost));
  if (err) OMF_HIP(hipMemset(plan->d_sync + 4, 0, 4));  // report each event once
  if (err & 4u)
    return fail(OMF_ETIMEOUT, "QSGD encoder: an on-chip wait exceeded its bound (a ring hand-off, or a "
                              "bracketed-encoder fix waiting for its tensor's norm) and was abandoned; the "
                              "payload of that launch is invalid");
  if (err & 8u)
    return fail(OMF_ETIMEOUT, "Top-K encoder: a grid barrier of the exact tail (the device-side fallback) "
                              "exceeded its bound and was abandoned; the selection of that call is invalid");
  if (err & 2u) {
    set_error("encoder recomputed a norm after a bounded wait (items not co-resident); results are exact");
    return 1;
  }
  set_error("");
  return OMF_OK;
}

static int check_bits(int32_t s) {
  if (s < 0 || s > 30) return fail(OMF_EINVAL, "bit_width must be in [0, 30] (levels = 2^bit_width is an int32 on the wire)");
  return OMF_OK;
}

// The fused PS step's last client (omf_ps_accumulate_apply_encode): its payload, width, level
// count and norms, and where acc + decode(q) goes (NULL: nowhere).
struct AccIn {
  const void* q;
  int32_t width, levels;
  const float* norm;
  float* acc_out;
};

static int encode_launch(omf_plan* p, const float* x, float alpha, int32_t s, const float* u, uint64_t seed,
                         uint64_t offset, const float* norm_in, void* q, float* norm_out, bool norm_only, void* stream,
                         float divisor, float* xout, uint32_t fmt, const AccIn* acc_in);

static int encode_impl(omf_plan* p, const float* x, float alpha, int32_t s, const float* u, uint64_t seed,
                       uint64_t offset, const float* norm_in, void* q, float* norm_out, bool norm_only, void* stream,
                       float divisor = 0.0f, float* xout = nullptr, int32_t fmt = 0, const AccIn* acc_in = nullptr) {
  if (!p) return fail(OMF_EINVAL, "plan is NULL");
  if (fmt < 0 || fmt > 2) return fail(OMF_EINVAL, "value_format must be 0 (fp32), 1 (bf16) or 2 (fp16)");
  DeviceGuard g(p->device);
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  if (int r = plan_enter(p, (hipStream_t)stream)) return r;
  if (int r = encode_launch(p, x, alpha, s, u, seed, offset, norm_in, q, norm_out, norm_only, stream, divisor, xout,
                            (uint32_t)fmt, acc_in))
    return r;
  return plan_leave(p, (hipStream_t)stream);
}

// Whether a fused PS step with the last client's decode takes the bracketed encoder's one pass
// (else the caller runs decode-accumulate, then the plain fused step).
static bool spec_serves(const omf_plan* p, int32_t s, const float* u, float divisor, uint32_t fmt, bool wide_ok);

static int encode_launch(omf_plan* p, const float* x, float alpha, int32_t s, const float* u, uint64_t seed,
                         uint64_t offset, const float* norm_in, void* q, float* norm_out, bool norm_only, void* stream,
                         float divisor, float* xout, uint32_t fmt, const AccIn* acc_in) {
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
  a.partials = p->d_partials;
  a.ticket = reinterpret_cast<uint32_t*>(p->d_sync);
  a.err = reinterpret_cast<uint32_t*>(p->d_sync + 4);
  a.counters = reinterpret_cast<uint32_t*>(p->d_sync + p->off_counters);
  a.gran = reinterpret_cast<uint64_t*>(p->d_sync + p->off_gran);
  a.alpha = alpha;
  a.fmt = fmt;
  a.levels = (float)(1u << s);
  a.seed_lo = (uint32_t)seed; a.seed_hi = (uint32_t)(seed >> 32); a.offset = (uint32_t)offset;
  a.wait_ticks = p->wait_ticks;
  const dim3 blk(kThreads);
  if (norm_in && !norm_only) {
    a.items = p->d_flat;
    a.tinfo = p->d_tinfo[0];
    const dim3 grid4((unsigned)(p->n_flat * 4));  // 4 blocks of 4 Ki elements per 16 Ki item
    p->last_encoder = 5;
    if (width == 1) {
      if (u) hipLaunchKernelGGL((qsgd_quant_sub<1, true, 4, false>), grid4, blk, 0, st, a);
      else hipLaunchKernelGGL((qsgd_quant_sub<1, false, 4, false>), grid4, blk, 0, st, a);
    } else {
      if (u) hipLaunchKernelGGL((qsgd_quant_sub<4, true, 4, false>), grid4, blk, 0, st, a);
      else hipLaunchKernelGGL((qsgd_quant_sub<4, false, 4, false>), grid4, blk, 0, st, a);
    }
    OMF_HIP(hipGetLastError());
    return OMF_OK;
  }
  // Grid encoder (strategy 4): on-device draws, any value format and width, arenas of at most
  // grid_wgs x 4 x kGridNB blocks of 4 Ki (larger ones, caller uniforms and the fused PS step
  // take the ring).  One launch.
  if (p->strategy == 4 && !norm_only && !u && divisor == 0.0f && p->grid_wgs > 0 &&
      p->n_spec_blocks <= (int64_t)p->grid_wgs * 4 * kGridNB) {
    GridArgs ga;
    a.items = p->d_flat;
    ga.e = a;
    ga.partials = p->d_spec_part;
    ga.bar = p->d_grid_bar;
    ga.target = (unsigned long long)(p->grid_launches + 1) * (unsigned long long)p->grid_wgs;
    ga.nblocks = p->n_spec_blocks;
    ga.dbg = p->spec_skip;
    const dim3 gg((unsigned)p->grid_wgs), gblk(1024);
    if (width == 1)
      hipLaunchKernelGGL(qsgd_encode_grid<1>, gg, gblk, 0, st, ga, (const Item*)p->d_flat, (const int64_t*)p->d_begins,
                         (const uint32_t*)p->d_grid_pbeg, (const uint32_t*)p->d_grid_pcnt);
    else
      hipLaunchKernelGGL(qsgd_encode_grid<4>, gg, gblk, 0, st, ga, (const Item*)p->d_flat, (const int64_t*)p->d_begins,
                         (const uint32_t*)p->d_grid_pbeg, (const uint32_t*)p->d_grid_pcnt);
    OMF_HIP(hipGetLastError());
    // counted only once the launch is in: the device's monotonic arrival counter advances by
    // grid_wgs per launch that ran, so a failed launch must not move the host's target
    ++p->grid_launches;
    p->last_encoder = 4;
    return OMF_OK;
  }
  // Bracketed single-read encoder: fp32 / bf16 / fp16 values with on-device draws at s <= 4, and
  // fp32 at s = 5-8 with wide levels (the default; int8 at 5-6, the int32 wire at 7-8); the rest
  // (wide levels off: the int32 wire on the ring, s = 5-6 and caller uniforms on the two-pass
  // encoder; the fused PS step is fp32).  No host interaction.
  if (!norm_only && spec_serves(p, s, u, divisor, fmt, acc_in == nullptr)) {
    // (the fused PS step too: the pass divides, stores the average and quantises it)
    SpecArgs sa;
    a.items = p->d_flat;
    a.tinfo = p->d_tinfo[1];
    sa.e = a;
    p->last_encoder = 3;
    sa.begins = p->d_begins;
    sa.sizes = p->d_sizes;
    sa.br_items = p->d_spec_br_items;
    sa.fold_items = p->d_spec_fold_items;
    sa.seg_part = p->d_spec_seg_part;
    sa.fold_cnt = p->d_spec_cnt;
    if (++p->spec_epoch >= 0x80000000u) p->spec_epoch = 1;  // 31-bit tags (the norm granule keeps a status bit)
    sa.epoch = p->spec_epoch;
    sa.wide = s > kSpecMaxBits ? 1u : 0u;
    sa.ngran = p->d_spec_ngran;
    sa.dbg = p->spec_skip;
    sa.zsig = s > kSpecMaxBits ? p->spec_zsig_wide : p->spec_zsig;
    sa.divisor = divisor;
    sa.xout = xout;
    sa.wait_ticks = p->wait_ticks;
    sa.br = p->d_spec_br;
    sa.partials = p->d_spec_part;
    const bool wide = s > kSpecMaxBits;
    if (wide && !p->d_spec_slots_w) {  // once per plan: the wide-level list capacity
      OMF_HIP(hipMalloc(&p->d_spec_slots_w, 4 * (size_t)spec_slot_words(kSpecPerWaveWide) * (size_t)p->n_spec_blocks));
      OMF_HIP(hipMalloc(&p->d_spec_recs_w, 32 * (size_t)kWaves * kSpecPerWaveWide * (size_t)p->n_spec_blocks));
      OMF_HIP(hipMalloc(&p->d_spec_br_part, 16 * (size_t)kBrParts * (size_t)p->nt));
      OMF_HIP(hipMalloc(&p->d_spec_br_cnt, 4 * (size_t)p->nt));
      OMF_HIP(hipMemsetAsync(p->d_spec_br_cnt, 0, 4 * (size_t)p->nt, st));  // left zero by every launch
    }
    const bool fb = p->spec_fb && !wide && !acc_in && fmt == 0 && width == 1 && !(p->spec_skip & 1u);
    const bool wfb = p->spec_fb && wide && !acc_in && fmt == 0 && !(p->spec_skip & 1u);  // wide levels
    if ((fb || wfb) && !p->d_spec_fb_part) {  // once per plan: the fused bracket's sums, counters and granules
      OMF_HIP(hipMalloc(&p->d_spec_fb_part, 16 * (size_t)std::max(kFbParts, kWfbParts) * (size_t)p->nt));
      OMF_HIP(hipMalloc(&p->d_spec_fb_cnt, 4 * (size_t)p->nt));
      OMF_HIP(hipMalloc(&p->d_spec_brgran, 16 * (size_t)p->nt));
      OMF_HIP(hipMemsetAsync(p->d_spec_fb_cnt, 0, 4 * (size_t)p->nt, st));  // left zero by every launch
      OMF_HIP(hipMemsetAsync(p->d_spec_brgran, 0, 16 * (size_t)p->nt, st));  // epoch 0 is never a launch's
    }
    sa.br_part = fb || wfb ? p->d_spec_fb_part : p->d_spec_br_part;
    sa.br_cnt = fb || wfb ? p->d_spec_fb_cnt : p->d_spec_br_cnt;
    sa.brgran = p->d_spec_brgran;
    p->spec_last_pw = wide ? kSpecPerWaveWide : kSpecPerWave;
    sa.slots = wide ? p->d_spec_slots_w : p->d_spec_slots;
    sa.heads = p->d_spec_heads;
    sa.recs = wide ? p->d_spec_recs_w : p->d_spec_recs;
    sa.flags = p->d_spec_flags;
    sa.status = p->d_spec_status;
    sa.nblocks = p->n_spec_blocks;
    sa.aq = acc_in ? acc_in->q : nullptr;
    sa.anorm = acc_in ? acc_in->norm : nullptr;
    sa.aout = acc_in ? acc_in->acc_out : nullptr;
    sa.awidth = acc_in ? acc_in->width : 0;
    sa.alevels = acc_in ? (float)acc_in->levels : 0.0f;
    sa.ainv = acc_in && (acc_in->levels & (acc_in->levels - 1)) == 0 ? 1.0f / (float)acc_in->levels : 0.0f;
    const dim3 gbr((unsigned)(p->n_spec_br * (s > kSpecMaxBits ? kBrParts : 1))), gb((unsigned)p->n_spec_blocks);
    // p->spec_skip: test / experiment switches (omf_plan_set_debug; 0 in production): bit 0
    // skips the bracket launch (the previous brackets stay), bit 1 the finish launch, bits 2/3
    // the fix stores / the fix, bit 4 the fold — the payload is then not the encoder's.
    const bool div = divisor != 0.0f;
    // The wide pass's one-wave workgroups reserve 10 KiB of LDS each (unused): 16 per CU, i.e. four
    // waves per SIMD — 0.556-0.559 ms per Llama-400M s = 8 encode against 0.589 uncapped, 0.565 at 12
    // KiB, 0.635 at 16 KiB (scripts/exp/occ_ab.sh, two interleaved rounds); OMF_SPEC_LDS_W overrides.
    // The s <= 4 pass is co-bound by its VALU and keeps every wave (24 KiB: 0.367 against 0.360 ms).
    static const size_t plds_w = [] { const char* v = omf::knob("OMF_SPEC_LDS_W"); return v ? (size_t)atoi(v) : (size_t)10240; }();
    if (fb) {  // the bracket folded into the pass (its first workgroups)
      const int64_t nbrw = (int64_t)kFbParts * p->n_spec_br;
      const dim3 gfb((unsigned)(nbrw + p->n_spec_blocks));
      if (div) hipLaunchKernelGGL((qsgd_spec_quant_fb<1, true>), gfb, blk, 0, st, sa, sa.br_items, nbrw, sa.begins);
      else hipLaunchKernelGGL((qsgd_spec_quant_fb<1, false>), gfb, blk, 0, st, sa, sa.br_items, nbrw, sa.begins);
    } else if (wfb) {  // wide levels: the bracket's one-wave parts first, then the pass's one-wave blocks
      const int64_t nbrw = (int64_t)kWfbParts * p->n_spec_br;
      const dim3 gw((unsigned)(nbrw + p->n_spec_blocks * kWaves)), bw(64);
      if (width == 1 && !div) hipLaunchKernelGGL((qsgd_spec_quant_wfb<1, false>), gw, bw, plds_w, st, sa, sa.br_items, nbrw, sa.begins);
      else if (width == 1) hipLaunchKernelGGL((qsgd_spec_quant_wfb<1, true>), gw, bw, plds_w, st, sa, sa.br_items, nbrw, sa.begins);
      else if (!div) hipLaunchKernelGGL((qsgd_spec_quant_wfb<4, false>), gw, bw, plds_w, st, sa, sa.br_items, nbrw, sa.begins);
      else hipLaunchKernelGGL((qsgd_spec_quant_wfb<4, true>), gw, bw, plds_w, st, sa, sa.br_items, nbrw, sa.begins);
    } else if (!(p->spec_skip & 1u)) {
      if (wide) hipLaunchKernelGGL(qsgd_spec_bracket_wide, gbr, dim3(kBrThreads), 0, st, sa, sa.br_items);
      else if (sa.aq) hipLaunchKernelGGL((qsgd_spec_bracket<false, true>), gbr, dim3(kBrThreads), 0, st, sa, sa.br_items);
      else hipLaunchKernelGGL((qsgd_spec_bracket<false, false>), gbr, dim3(kBrThreads), 0, st, sa, sa.br_items);
    }
    const float* an = sa.anorm;
    const int aw = acc_in ? (acc_in->width == 32 ? 4 : 1) : 0;
    constexpr int PWW = kSpecPerWaveWide;
    if (fb || wfb) {
      // (the pass ran above)
    } else if (wide) {  // fp32, no fused last client (spec_serves); one wave per workgroup unless OMF_SPEC_WPB=4
      static const bool wpb4 = [] { const char* v = omf::knob("OMF_SPEC_WPB"); return v && atoi(v) == 4; }();
      const dim3 g1((unsigned)(p->n_spec_blocks * kWaves)), b1(64);
      if (wpb4) {
        if (width == 1 && !div) hipLaunchKernelGGL((qsgd_spec_quant<1, false, kFmtF32, 0, PWW>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
        else if (width == 1) hipLaunchKernelGGL((qsgd_spec_quant<1, true, kFmtF32, 0, PWW>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
        else if (!div) hipLaunchKernelGGL((qsgd_spec_quant<4, false, kFmtF32, 0, PWW>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
        else hipLaunchKernelGGL((qsgd_spec_quant<4, true, kFmtF32, 0, PWW>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
      } else {
        if (width == 1 && !div) hipLaunchKernelGGL((qsgd_spec_quant<1, false, kFmtF32, 0, PWW, 1>), g1, b1, plds_w, st, sa, sa.br, sa.begins, an);
        else if (width == 1) hipLaunchKernelGGL((qsgd_spec_quant<1, true, kFmtF32, 0, PWW, 1>), g1, b1, plds_w, st, sa, sa.br, sa.begins, an);
        else if (!div) hipLaunchKernelGGL((qsgd_spec_quant<4, false, kFmtF32, 0, PWW, 1>), g1, b1, plds_w, st, sa, sa.br, sa.begins, an);
        else hipLaunchKernelGGL((qsgd_spec_quant<4, true, kFmtF32, 0, PWW, 1>), g1, b1, plds_w, st, sa, sa.br, sa.begins, an);
      }
    } else if (fmt == kFmtBF16) hipLaunchKernelGGL((qsgd_spec_quant<1, false, kFmtBF16>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    else if (fmt == kFmtF16) hipLaunchKernelGGL((qsgd_spec_quant<1, false, kFmtF16>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    else if (width == 1 && !div) hipLaunchKernelGGL((qsgd_spec_quant<1, false>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    else if (width == 1 && aw == 1) hipLaunchKernelGGL((qsgd_spec_quant<1, true, kFmtF32, 1>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    else if (width == 1 && aw == 4) hipLaunchKernelGGL((qsgd_spec_quant<1, true, kFmtF32, 4>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    else if (width == 1) hipLaunchKernelGGL((qsgd_spec_quant<1, true>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    else if (!div) hipLaunchKernelGGL((qsgd_spec_quant<4, false>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    else hipLaunchKernelGGL((qsgd_spec_quant<4, true>), gb, blk, 0, st, sa, sa.br, sa.begins, an);
    if (p->spec_skip & 2u) {  // experiment: no finish launch (timings only)
      OMF_HIP(hipGetLastError());
      return OMF_OK;
    }
    const int32_t nfold = (int32_t)p->n_spec_fold;
    if (wide) {
#ifndef OMF_FIX_FT  // experiment builds may override it (scripts/exp/s8_variants.sh)
#define OMF_FIX_FT 4
#endif
      constexpr int FT = OMF_FIX_FT, BPW = kThreads / (kWaves * FT);  // fix: 16 blocks per workgroup
      const dim3 gw((unsigned)(nfold + (p->n_spec_blocks + BPW - 1) / BPW));
      if (width == 1)
        hipLaunchKernelGGL((qsgd_spec_finish<1, PWW, FT>), gw, blk, 0, st, sa, (const SpecFoldItem*)sa.fold_items, nfold,
                           (const Item*)a.items, (const int64_t*)sa.begins, (const uint32_t*)sa.slots,
                           (const float4*)sa.recs, (const uint32_t*)sa.heads);
      else
        hipLaunchKernelGGL((qsgd_spec_finish<4, PWW, FT>), gw, blk, 0, st, sa, (const SpecFoldItem*)sa.fold_items, nfold,
                           (const Item*)a.items, (const int64_t*)sa.begins, (const uint32_t*)sa.slots,
                           (const float4*)sa.recs, (const uint32_t*)sa.heads);
      OMF_HIP(hipGetLastError());
      return OMF_OK;
    }
    const dim3 gfin((unsigned)(nfold + (p->n_spec_blocks + kThreads / kWaves - 1) / (kThreads / kWaves)));  // fix: 64 blocks per workgroup
    if (width == 1)
      hipLaunchKernelGGL(qsgd_spec_finish<1>, gfin, blk, 0, st, sa, (const SpecFoldItem*)sa.fold_items, nfold,
                         (const Item*)a.items, (const int64_t*)sa.begins, (const uint32_t*)sa.slots,
                         (const float4*)sa.recs, (const uint32_t*)sa.heads);
    else
      hipLaunchKernelGGL(qsgd_spec_finish<4>, gfin, blk, 0, st, sa, (const SpecFoldItem*)sa.fold_items, nfold,
                         (const Item*)a.items, (const int64_t*)sa.begins, (const uint32_t*)sa.slots,
                         (const float4*)sa.recs, (const uint32_t*)sa.heads);
    OMF_HIP(hipGetLastError());
    return OMF_OK;
  }
  // The ring also serves the fused PS step (divide + encode in one launch) under any strategy,
  // and — with wide levels off (omf_plan_set_wide_levels) — the bracketed plans' int32-wire
  // encodes (s >= 7, fp32, on-device draws): Llama-400M s = 8 0.68 ms against 0.74 for the
  // two-pass encoder, whose second pass rewrites the 4 N payload after re-reading x (round 4).
  // With wide levels on (the default) those take the bracketed encoder above.  bf16 / fp16
  // values and caller uniforms stay on the two-pass encoder (0.61 / 0.78 ms against the ring's
  // 0.70 / 0.83).
  const bool wide_ring = p->strategy == 3 && width == 4 && !u && fmt == 0;
  if ((p->strategy == 2 || p->strategy == 4 || divisor != 0.0f || wide_ring) && !norm_only) {
    omf::ring::Args r;
    r.x = x; r.u = u; r.q = q; r.norm_out = norm_out;
    r.items = p->d_ring; r.tinfo = p->d_ring_t; r.gran = p->d_ring_gran;
    r.err = reinterpret_cast<uint32_t*>(p->d_sync + 4);
    r.n_items = p->n_ring;
    r.alpha = alpha;
    r.fmt = fmt;
    r.round_in = (fmt != 0 && alpha != 1.0f) ? 1u : 0u;
    r.divisor = divisor;
    r.divide = divisor != 0.0f ? 1u : 0u;
    r.xout = xout;
    r.levels = (float)(1u << s);
    r.seed_lo = (uint32_t)seed; r.seed_hi = (uint32_t)(seed >> 32); r.offset = (uint32_t)offset;
    if (++p->ring_epoch == 0) ++p->ring_epoch;
    r.epoch = p->ring_epoch;
    r.wait_ticks = p->wait_ticks;
    r.lds_wait_ticks = p->lds_wait_ticks;
    r.dbg = p->ring_dbg;
    r.prof = p->d_ring_prof;
    const int grid = (int)std::min<int64_t>(p->ring_grid, std::max<int64_t>(p->n_ring, 1));
    p->last_encoder = 2;
    if (omf::ring::launch(p->ring_cfg, width, u != nullptr, r, grid, st) != 0)
      return fail(OMF_EHIP, "ring encoder launch failed");
    OMF_HIP(hipGetLastError());
    return OMF_OK;
  }
  // No per-call memset: tickets and arrival counters are reset in-kernel by their last
  // user, and granules carry this launch's epoch.
  const int strat = p->strategy >= 2 ? 1 : p->strategy;  // norms-only passes use the two-pass tables
  if (++p->epoch == 0) ++p->epoch;
  a.epoch = p->epoch;
  a.n_items = (uint32_t)p->n_enc[strat];
  a.items = p->d_enc[strat];
  a.tinfo = p->d_tinfo[strat];
  const dim3 grid((unsigned)p->n_enc[strat]);
  if (!norm_only) p->last_encoder = strat;
#define OMF_ENC(EV)                                                                              \
  do {                                                                                           \
    if (norm_only) {                                                                             \
      hipLaunchKernelGGL((qsgd_encode_ordered<1, false, true, EV>), grid, blk, 0, st, a);        \
    } else if (width == 1) {                                                                     \
      if (u) hipLaunchKernelGGL((qsgd_encode_ordered<1, true, false, EV>), grid, blk, 0, st, a); \
      else hipLaunchKernelGGL((qsgd_encode_ordered<1, false, false, EV>), grid, blk, 0, st, a);  \
    } else {                                                                                     \
      if (u) hipLaunchKernelGGL((qsgd_encode_ordered<4, true, false, EV>), grid, blk, 0, st, a); \
      else hipLaunchKernelGGL((qsgd_encode_ordered<4, false, false, EV>), grid, blk, 0, st, a);  \
    }                                                                                            \
  } while (0)
  if (p->ev == 8) OMF_ENC(8);
  else OMF_ENC(16);
#undef OMF_ENC
  OMF_HIP(hipGetLastError());
  return OMF_OK;
}

static bool spec_serves(const omf_plan* p, int32_t s, const float* u, float divisor, uint32_t fmt, bool wide_ok) {
  if (p->strategy != 3 || u || s < kSpecMinBits) return false;
  if (s <= kSpecMaxBits) return fmt == 0 || divisor == 0.0f;
  return wide_ok && p->spec_wide && s <= kSpecMaxBitsWide && fmt == 0;  // fp32 wide levels
}

int omf_qsgd_encode(omf_plan* plan, const float* x, float alpha, int32_t bit_width, const float* u, uint64_t seed,
                    uint64_t offset, const float* norm_in, void* q_out, float* norm_out, void* stream) {
  return encode_impl(plan, x, alpha, bit_width, u, seed, offset, norm_in, q_out, norm_out, false, stream);
}

int omf_qsgd_encode_ex(omf_plan* plan, const float* x, float alpha, int32_t bit_width, int32_t value_format,
                       const float* u, uint64_t seed, uint64_t offset, const float* norm_in, void* q_out,
                       float* norm_out, void* stream) {
  return encode_impl(plan, x, alpha, bit_width, u, seed, offset, norm_in, q_out, norm_out, false, stream, 0.0f,
                     nullptr, value_format);
}

int omf_qsgd_norms_ex(omf_plan* plan, const float* x, float alpha, int32_t value_format, float* norm_out,
                      void* stream) {
  return encode_impl(plan, x, alpha, 0, nullptr, 0, 0, nullptr, nullptr, norm_out, true, stream, 0.0f, nullptr,
                     value_format);
}

int omf_ps_apply_encode(omf_plan* p, const float* acc, float divisor, float* avg_out, int32_t bit_width,
                        const float* u, uint64_t seed, uint64_t offset, void* q_out, float* norm_out, void* stream) {
  if (!p) return fail(OMF_EINVAL, "plan is NULL");
  if (!acc || !avg_out) return fail(OMF_EINVAL, "omf_ps_apply_encode: acc and avg_out must be non-NULL");
  if (!(divisor != 0.0f)) return fail(OMF_EINVAL, "omf_ps_apply_encode: divisor must be non-zero");
  if (!aligned(avg_out, 16)) return fail(OMF_EINVAL, "omf_ps_apply_encode: avg_out must be 16-byte aligned");
  const size_t bytes = 4 * (size_t)p->arena_end;
  const uintptr_t a0 = (uintptr_t)acc, o0 = (uintptr_t)avg_out;
  const bool alias = avg_out == acc;
  if (!alias && a0 < o0 + bytes && o0 < a0 + bytes)
    return fail(OMF_EINVAL, "omf_ps_apply_encode: avg_out partially overlaps acc (pass the same pointer or disjoint buffers)");
  // The fused launch reads acc while it writes avg (second-pass chunks of large tensors
  // re-read acc, the bounded-wait fallback recomputes partials from it), so it needs
  // avg_out disjoint from acc; in place it runs as divide + encode.
  if (!alias)  // one ring launch: read acc once, write avg and the payload
    return encode_impl(p, acc, 1.0f, bit_width, u, seed, offset, nullptr, q_out, norm_out, false, stream, divisor,
                       avg_out);
  // in place: the same results as divide, then encode
  DeviceGuard g(p->device);
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  if (avg_out != acc)
    OMF_HIP(hipMemcpyAsync(avg_out, acc, 4 * (size_t)p->arena_end, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  if (int r = omf_div_f32(avg_out, p->arena_end, divisor, stream)) return r;
  return encode_impl(p, avg_out, 1.0f, bit_width, u, seed, offset, nullptr, q_out, norm_out, false, stream);
}

int omf_ps_accumulate_apply_encode(omf_plan* p, const float* acc, const void* q_in, int32_t width_in,
                                   int32_t levels_in, const float* norm_in, float* acc_out, float divisor,
                                   float* avg_out, int32_t bit_width, const float* u, uint64_t seed, uint64_t offset,
                                   void* q_out, float* norm_out, void* stream) {
  if (!p) return fail(OMF_EINVAL, "plan is NULL");
  if (!acc || !avg_out || !q_in || !norm_in)
    return fail(OMF_EINVAL, "omf_ps_accumulate_apply_encode: acc, q_in, norm_in and avg_out must be non-NULL");
  if (width_in != 8 && width_in != 32) return fail(OMF_EINVAL, "width_in must be 8 or 32");
  if (levels_in <= 0) return fail(OMF_EINVAL, "levels_in must be > 0");
  if (!(divisor != 0.0f)) return fail(OMF_EINVAL, "omf_ps_accumulate_apply_encode: divisor must be non-zero");
  if (int r = check_bits(bit_width)) return r;
  if (!aligned(acc, 16) || !aligned(avg_out, 16) || (acc_out && !aligned(acc_out, 16)) ||
      !aligned(q_in, width_in == 8 ? 4 : 16))
    return fail(OMF_EINVAL, "misaligned buffer (fp32/int32 need 16 B, int8 needs 4 B alignment)");
  const size_t bytes = 4 * (size_t)p->arena_end;
  auto overlap = [bytes](const void* x, const void* y) {
    const uintptr_t a0 = (uintptr_t)x, b0 = (uintptr_t)y;
    return a0 < b0 + bytes && b0 < a0 + bytes;
  };
  if (overlap(avg_out, acc) || (acc_out && overlap(avg_out, acc_out)) || (acc_out && acc_out != acc && overlap(acc_out, acc)))
    return fail(OMF_EINVAL, "omf_ps_accumulate_apply_encode: avg_out must be disjoint from acc and acc_out; acc_out is "
                            "acc itself or disjoint from it");
  DeviceGuard g(p->device);
  if (!g.ok) return fail(OMF_EHIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;
  if (spec_serves(p, bit_width, u, divisor, 0u, false)) {  // one pass: acc and the last payload read once
    const AccIn ai{q_in, width_in, levels_in, norm_in, acc_out};
    return encode_impl(p, acc, 1.0f, bit_width, u, seed, offset, nullptr, q_out, norm_out, false, stream, divisor,
                       avg_out, 0, &ai);
  }
  // other encoders: the decoder's accumulate, then the fused step (the same bytes)
  float* sum = acc_out ? acc_out : avg_out;
  if (sum != acc) OMF_HIP(hipMemcpyAsync(sum, acc, bytes, hipMemcpyDeviceToDevice, st));
  if (int r = omf_qsgd_decode(p, q_in, width_in, levels_in, norm_in, sum, 1, stream)) return r;
  return omf_ps_apply_encode(p, sum, divisor, avg_out, bit_width, u, seed, offset, q_out, norm_out, stream);
}

int omf_qsgd_norms(omf_plan* plan, const float* x, float alpha, float* norm_out, void* stream) {
  return encode_impl(plan, x, alpha, 0, nullptr, 0, 0, nullptr, nullptr, norm_out, true, stream);
}

static int decode_blocks(omf_plan* p, const void* q, int32_t width, int32_t levels, const float* norm, float* y,
                         int32_t accumulate, int64_t b0, int64_t b1, void* stream) {
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
  b0 = std::max<int64_t>(b0, 0);
  b1 = std::min<int64_t>(b1, p->n_dec_blocks);
  if (b1 <= b0) return OMF_OK;
  const dim3 blk(kThreads);
  hipStream_t st = (hipStream_t)stream;
  // A plain decode's workgroups reserve 24 KiB of LDS each (unused): six per CU — Llama-400M 0.294-
  // 0.296 ms at s = 4 and 0.482-0.484 at s = 8 against 0.301 / 0.490 uncapped, 0.308 / 0.489 at 28 KiB
  // (scripts/exp/occ_ab.sh); OMF_DEC_LDS overrides.  Accumulating decodes keep every wave.
  static const size_t dlds = [] { const char* v = omf::knob("OMF_DEC_LDS"); return v ? (size_t)atoi(v) : (size_t)24576; }();
  // the last whole quad of the payload the caller holds (width 8: round_up(arena_end, 4) bytes
  // are not promised, so a clamped load never passes the last full quad)
  const int64_t qlast = (p->arena_end & ~(int64_t)3) - 4;  // < 0 only for arenas of < 4 elements
#define OMF_DEC(W, A, P)                                                                                         \
  do {                                                                                                           \
    if (qlast >= 0) {                                                                                            \
      const int64_t per = kDecBlk / (kDecQuads<W, A> * kThreads * 4); /* decode blocks per table block */       \
      hipLaunchKernelGGL((qsgd_decode_arena<W, A, P>), dim3((unsigned)((b1 - b0) * per)), blk, A ? 0 : dlds, st, a, \
                         (const uint32_t*)p->d_dec_binfo, norm, (const int64_t*)p->d_begins,                    \
                         (const int64_t*)p->d_sizes, p->nt, qlast, (uint32_t)(b0 * per));                       \
    } else /* a payload of < 4 elements: the item decoder's byte loads */                                          \
      hipLaunchKernelGGL((qsgd_decode_flat<W, A, P>), dim3((unsigned)p->n_flat), blk, 0, st, a);                \
  } while (0)
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

int omf_qsgd_decode(omf_plan* p, const void* q, int32_t width, int32_t levels, const float* norm, float* y,
                    int32_t accumulate, void* stream) {
  if (!p) return fail(OMF_EINVAL, "plan is NULL");
  return decode_blocks(p, q, width, levels, norm, y, accumulate, 0, p->n_dec_blocks, stream);
}

int omf_qsgd_decode_range(omf_plan* p, const void* q, int32_t width, int32_t levels, const float* norm, float* y,
                          int32_t accumulate, int64_t elem_begin, int64_t elem_end, void* stream) {
  if (!p) return fail(OMF_EINVAL, "plan is NULL");
  if (elem_begin < 0 || elem_end < elem_begin) return fail(OMF_EINVAL, "omf_qsgd_decode_range: bad element range");
  if (p->arena_end < 4)  // the item decoder of tiny payloads has no block ranges: decode it all
    return decode_blocks(p, q, width, levels, norm, y, accumulate, 0, p->n_dec_blocks, stream);
  return decode_blocks(p, q, width, levels, norm, y, accumulate, elem_begin / kDecBlk,
                       (elem_end + kDecBlk - 1) / kDecBlk, stream);
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
