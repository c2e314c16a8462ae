// omf_qsgd_ring.hip — single-read QSGD encoder for the hybrid global hop, MI355X (gfx950).
//
// Semantics: SURVEY.md §8a "Exact QSGD semantics" (reference src/omnifed/hybrid/compression/
// qsgd.py:36-64): one fp32 L2 norm per tensor, then per-element stochastic levels.  The
// norm of a tensor is known only once all of it has been read, so a straightforward
// encoder reads x twice (9 N bytes of HBM traffic for an int8 payload).  This one reads
// it once (5 N):
//
//   * persistent workgroups walk a host-built sequence of chunks (item i -> workgroup
//     i mod grid, so consecutive chunks of a tensor spread over the whole chip);
//   * a chunk is loaded into registers, its partial sum of squares is published as an
//     8-byte {epoch, fp32} granule (sc1 store), and the chunk waits in an LDS ring slot
//     of its workgroup until every granule of its tensor carries this launch's epoch;
//   * every consumer folds the granules in the same fixed order (thread j sums granules
//     j, j + NT, ... in fp64, then a fixed block reduction), so the norm is identical in
//     every workgroup and every run;
//   * the poll for the ring head is issued BEFORE the next chunk's loads, so waiting for
//     it (vmcnt counts in order) leaves the chunk loads in flight while the head is
//     quantised from LDS;
//   * a workgroup only blocks (ring full) after publishing every chunk it has taken, so
//     the sequence is deadlock-free for co-resident workgroups; a bounded wait that
//     expires recomputes the norm from x in the producers' exact order (same bits) and
//     sets err bit 2 (omf_plan_check returns 1) — the kernel cannot hang.
//
// Tensors too large to hold (> slots x grid chunks) are NORM chunks (partial only) plus
// QUANT chunks (re-read once the norm is known), placed by the plan (omf_qsgd.hip).
//
// Element layout inside a chunk (rows of 1024 elements; thread t, float4 k):
//   row = rows_per_thread * (t >> 8) + k,  element = row * 1024 + 4 * (t & 255)
// so a wave reads 1 KiB contiguous per instruction and a thread's four consecutive rows
// form one Philox group of the stream in oracle/philox.py.
#include "../../include/omf_codec.h"
#include "../../include/omf_codec_experimental.h"
#include "omf_common.h"
#include "omf_qsgd_dev.h"
#include "omf_ring.h"

#include <utility>

namespace omf {
namespace ring {
namespace {

// Block-uniform values the compiler cannot prove uniform (barrier votes, LDS reductions):
// readfirstlane keeps them (and the ring bookkeeping that depends on them) in SGPRs.
__device__ __forceinline__ int ufirst(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float ufirst(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ Tensor tensor_of(const Item& it) {
  return Tensor{it.tbegin, it.tn, it.nchunks, it.gbase, {0, 0}};
}

__device__ __forceinline__ float4 scale4(float4 v, float alpha) {
  return make_float4(__fmul_rn(v.x, alpha), __fmul_rn(v.y, alpha), __fmul_rn(v.z, alpha), __fmul_rn(v.w, alpha));
}

// The encoder's input transform: the client weighting x * alpha (global_grpc.py:101-123),
// or the PS average x / total_samples (global_grpc_server.py:155-171), bit-exact.
__device__ __forceinline__ float4 prologue4(const Args& a, float4 v) {
  if (a.divide) return Divisor(a.divisor).div4(v);
  v = scale4(v, a.alpha);
  return a.round_in ? round_fmt4(v, a.fmt) : v;  // bf16/fp16 torch.mul rounds its product
}

__device__ __forceinline__ float sumsq4(float4 v, float acc) {
  acc = fmaf(v.x, v.x, acc);
  acc = fmaf(v.y, v.y, acc);
  acc = fmaf(v.z, v.z, acc);
  return fmaf(v.w, v.w, acc);
}

// Uniforms of Philox group G (3 calls, 16 x 24-bit fields; oracle/philox.py).
__device__ __forceinline__ void philox_group(const Args& a, uint64_t G, int32_t tensor, float4 (&uu)[4]) {
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

// Uniforms for rows 4rg .. 4rg+3 at lane position j of the chunk [cb, ce) of tensor
// `tensor` (chunk offset coff within it): caller draws (parity mode) or Philox group
// G = (coff/4096 + rg)*256 + j (oracle/philox.py).  Independent of the norm, so a claimer
// draws them while the norm is still being resolved.
template <bool HAS_U>
__device__ __forceinline__ void draws_at(const Args& a, int rg, int j, int64_t cb, int64_t ce, int64_t coff,
                                         int32_t tensor, bool full, float4 (&uu)[4]) {
  const int n = (int)(ce - cb);
  if (HAS_U) {
    const float* __restrict__ ub = a.u + cb;
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      const int e = (4 * rg + sl) * 1024 + 4 * j;
      if (full || e + 4 <= n) {
        uu[sl] = *reinterpret_cast<const float4*>(ub + e);
      } else {
        uu[sl] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < n) uu[sl].x = ub[e];
        if (e + 1 < n) uu[sl].y = ub[e + 1];
        if (e + 2 < n) uu[sl].z = ub[e + 2];
      }
    }
  } else {
#ifdef OMF_EXP_NORNG  // experiment builds only: price the RNG
    for (int sl = 0; sl < 4; ++sl) uu[sl] = make_float4(0.5f, 0.25f, 0.75f, 0.125f);
#else
    philox_group(a, ((uint64_t)(coff >> 12) + (uint64_t)rg) * 256u + (uint64_t)j, tensor, uu);
#endif
  }
}

// ---------------------------------------------------------------- buffer-op helpers
// Chunk-relative buffer descriptors, range-checked by the hardware per dword (loads out of
// range read 0, stores out of range are dropped; a descriptor of 0 bytes turns an access
// into a no-op).  Every access of a thread uses ONE 32-bit lane offset plus a scalar row
// offset, a tensor's partial last chunk needs no guard, and a step can issue the same
// memory instructions whatever it has to do — hipcc counts its vmcnt waits only across
// straight-line loads (a branch around a load makes it wait vmcnt(0), draining every
// prefetch in flight: cdna_hip_programming.md §5, trap (c)).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
constexpr int kAuxNT = 2;    // cache policy nt: streamed once
constexpr int kAuxSC1 = 16;  // sc1: agent-coherent (granules cross the XCDs' private L2s)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t chunk_rsrc(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// float4 of row `sl` (byte offset voff + sl * 4 KiB).
__device__ __forceinline__ float4 ld_row(__amdgpu_buffer_rsrc_t r, int voff, int sl) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, sl * 4096, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ void st_row(__amdgpu_buffer_rsrc_t r, int voff, int sl, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(
      (u32x4_t){__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)}, r, voff,
      sl * 4096, kAuxNT);
}
// Four levels of row `sl` (element offset eoff of the row-0 float4).  int8: one packed
// dword (the descriptor spans the chunk rounded up to 4 bytes: the tail of a partial last
// dword lands in the arena's alignment padding as zeros).
template <int WIDTH>
__device__ __forceinline__ void st_levels(__amdgpu_buffer_rsrc_t r, int eoff, int sl, const int32_t (&qq)[4]) {
  if (WIDTH == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(pack_i8x4(qq), r, eoff, sl * 1024, kAuxNT);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128((u32x4_t){(uint32_t)qq[0], (uint32_t)qq[1], (uint32_t)qq[2], (uint32_t)qq[3]},
                                           r, 4 * eoff, sl * 4096, kAuxNT);
  }
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t payload_rsrc(const Args& a, int width, int64_t begin, int64_t n) {
  return chunk_rsrc(static_cast<int8_t*>(a.q) + begin * width, width == 1 ? (n + 3) & ~int64_t(3) : 4 * n);
}

// Quantise and store rows 4rg .. 4rg+3 at lane position j of the chunk [cb, ce); w = those
// four float4, already scaled by alpha; uu = their uniforms (draws_at).  The payload goes
// through a range-checked chunk descriptor, so a tensor's partial last chunk needs no
// per-row guard (its out-of-range elements were loaded as zeros and quantise to 0).  The
// norm is always this launch's own (never caller-supplied): |x| <= norm, so |vn| * L stays
// far below 2^63 and qsgd_quad's overflow test is skipped.
template <int WIDTH>
__device__ __forceinline__ void quant_group_at(const Args& a, const float4 (&w)[4], const float4 (&uu)[4], int rg,
                                               int j, int64_t cb, int64_t ce, const Divisor& dv, bool zero) {
  const __amdgpu_buffer_rsrc_t r = payload_rsrc(a, WIDTH, cb, ce - cb);
  const int eoff = 4 * rg * 1024 + 4 * j;
  if (zero) {  // tile-uniform: keeps the flag out of the per-row code
    const int32_t qz[4] = {0, 0, 0, 0};
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) st_levels<WIDTH>(r, eoff, sl, qz);
    return;
  }
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
    int32_t qq[4];
    qsgd_quad<false>(w[sl], uu[sl], dv, a.levels, false, qq);
    st_levels<WIDTH>(r, eoff, sl, qq);
  }
}

// One Philox group of the register-resident kernel: rows 4rg .. 4rg+3 at float4 column j,
// held in w (already scaled).  The Philox words are consumed as they are produced (same
// stream and bits as philox_group: row sl takes words 3sl .. 3sl+2 of the group's three
// calls), so at most one call's output and two carried words are live beside the chunk
// buffers.  HAS_U: caller uniforms (parity mode) through the chunk-relative descriptor ru.
template <int WIDTH, bool HAS_U>
__device__ __forceinline__ void quant_group_rr(const Args& a, const float4 (&w)[4], int rg, int j, int64_t coff,
                                               int32_t tensor, float norm, __amdgpu_buffer_rsrc_t rq,
                                               __amdgpu_buffer_rsrc_t ru, int voff) {
  const bool zero = !(norm != 0.0f);
  const Divisor dv(norm, a.fmt);
  auto row = [&](int sl, float4 u) {
    int32_t qq[4];
    qsgd_quad(w[sl], u, dv, a.levels, zero, qq);
    st_levels<WIDTH>(rq, voff >> 2, sl, qq);
  };
  if (HAS_U) {
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) row(sl, ld_row(ru, voff, sl));
    return;
  }
  // counter 3G + c, G = ((coff >> 12) + rg) * 256 + j: a uniform 64-bit part plus 3j + c < 2^10
  // (kept 32-bit: a per-lane 64-bit counter base costs two registers for the whole loop)
  const uint64_t base = 3 * ((((uint64_t)(coff >> 12) + (uint64_t)rg)) << 8);
  const uint32_t blo = (uint32_t)base, bhi = (uint32_t)(base >> 32);
  auto call = [&](uint32_t c) {
    const uint32_t add = 3u * (uint32_t)j + c;
    const uint32_t lo = blo + add;
    const uint32_t hi = bhi + (lo < add ? 1u : 0u);
    return philox4x32_10(make_uint4(lo, hi, (uint32_t)tensor, a.offset), a.seed_lo, a.seed_hi);
  };
  const uint4 r0 = call(0);
  row(0, u24x4(r0.x, r0.y, r0.z));
  const uint4 r1 = call(1);
  row(1, u24x4(r0.w, r1.x, r1.y));
  const uint4 r2 = call(2);
  row(2, u24x4(r1.z, r1.w, r2.x));
  row(3, u24x4(r2.y, r2.z, r2.w));
}

// ---------------------------------------------------------------- producer/consumer kernel
//
// One 1024-thread workgroup per CU: waves 0-7 are LOADERS, waves 8-15 QUANTISERS, and
// they synchronise only through LDS flags (no workgroup barrier after the prologue), so
// each role needs only its own registers and a loader's prefetch is never drained by a
// barrier or by another role's wait.
//
// Chunk = ROWS rows of 1024 elements.  Loader wave w owns rows [w*ROWS/8, (w+1)*ROWS/8):
// lane l loads float4 l, l+64, l+128, l+192 of each row (1 KiB contiguous per wave
// instruction), reduces them in that order (fp32 fma chain), stores them into the slot
// (row-major, the same addresses) and publishes its wave partial; the last loader to
// arrive folds the 8 wave partials in order (fp64), publishes the chunk granule and
// marks the slot loaded.  Quantiser thread u (0..511) owns row-groups rg = (u>>8)*GPT+h,
// lane position j = u & 255: the Philox group of oracle/philox.py.
//
// Slot life: loaders wait freed[s] >= k-S+1, fill, loaded[s] = k+1; quantiser wave 0
// resolves the norm (single-chunk partial, cached tensor, or the granule poll) and sets
// qready[s] = k+1; every quantiser wave quantises its groups, the last sets freed[s] = k+1.

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_add(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// This wave's LDS writes have landed (LDS only; in-flight global loads stay in flight).
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Per-workgroup abort word (every kernel below zeroes it before its first barrier): set
// when an LDS wait exceeds its bound.  Every later wait of the workgroup then returns at
// once, so each wave runs its loops (all bounded by the item count) to the end and the
// grid drains; err bit 4 makes omf_plan_check report OMF_ETIMEOUT (payload invalid).
__shared__ uint32_t g_wg_abort;

__device__ __forceinline__ bool wg_aborted() { return ufirst((int)lds_ld(&g_wg_abort)) != 0; }

// Wait until the LDS word *p >= v.  Bounded: the clock is read only every 64 sleeps, so
// the common short wait costs one LDS load per poll; past a.lds_wait_ticks (20 ms) the
// workgroup aborts instead of hanging the GPU (a hand-off logic error, never expected).
// The bound needs both the wall-clock time AND a minimum number of polls (about a quarter
// of the bound spent polling): a context switch of the queue (CWSR) advances the clock
// while the wave is saved, and must not look like a stuck hand-off.
__device__ __forceinline__ void lds_wait_ge(const Args& a, const uint32_t* p, uint32_t v) {
  if (ufirst((int)lds_ld(p)) < (int)v) {
    uint64_t t0 = 0;
    const uint64_t min_polls = a.lds_wait_ticks >> 5;  // a poll is >= ~7 ticks (s_sleep 1 + an LDS load)
    for (uint32_t i = 1;; ++i) {
      __builtin_amdgcn_s_sleep(1);
      if (ufirst((int)lds_ld(p)) >= (int)v) break;
      if ((i & 63) == 0) {
        if (wg_aborted()) break;
        const uint64_t now = wall_clock64();
        if (t0 == 0) {
          t0 = now;
        } else if (now - t0 > a.lds_wait_ticks && i > min_polls) {
          lds_st(&g_wg_abort, 1u);
          if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(a.err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  asm volatile("" ::: "memory");
}

// dbg & 4: per-wave phase cycle totals, accumulated locally and flushed once at exit.
struct Prof {
  uint64_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  __device__ __forceinline__ void add(int ph, uint64_t cycles) { c[ph] += cycles; }
  __device__ __forceinline__ void flush(const Args& a) {
    if ((a.dbg & 4) && (threadIdx.x & 63) == 0)
      for (int i = 0; i < 8; ++i)
        if (c[i]) atomicAdd(&a.prof[i], (unsigned long long)c[i]);
  }
};

// Sum of squares of one loader wave's rows of a chunk, in the loader's exact order.
template <int ROWS, int LW>
__device__ __forceinline__ float loader_sumsq(const Args& a, int64_t cb, int n, int w, int lane) {
  constexpr int RPW = ROWS / LW;
  const float* __restrict__ xb = a.x + cb;
  float acc = 0.0f;
  for (int r = 0; r < RPW; ++r)
    for (int m = 0; m < 4; ++m) {
      const int i = (w * RPW + r) * 1024 + 4 * (lane + 64 * m);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i + 4 <= n) {
        v = *reinterpret_cast<const float4*>(xb + i);
      } else {
        if (i < n) v.x = xb[i];
        if (i + 1 < n) v.y = xb[i + 1];
        if (i + 2 < n) v.z = xb[i + 2];
      }
      acc = sumsq4(prologue4(a, v), acc);
    }
  return acc;
}

// Granule fold of one tensor by ONE wave: lane l sums granules l, l+64, ... (fp64, in
// order), then the fixed butterfly.  Identical in every workgroup.
__device__ __forceinline__ bool poll_norm_wave(const Args& a, const Tensor& ti, int lane, float& norm) {
  double p = 0.0;
  int ok = 1;
  for (int j = lane; j < ti.nchunks; j += 64) {
    const uint64_t g = ld_agent(&a.gran[ti.gbase + j]);
    ok &= (uint32_t)(g >> 32) == a.epoch;
    p += (double)__uint_as_float((uint32_t)g);
  }
  if (!__all(ok)) return false;
  norm = ufirst(finish_norm(wave_sum_f64(p), a.fmt));
  return true;
}

// Bounded poll; on expiry recompute every chunk partial with `partial(cb, n)` (the
// producers' exact order) and fold them like the poll: same bits, err bit 2 set.
template <class Partial>
__device__ __forceinline__ float wait_norm_poll(const Args& a, const Tensor& ti, int lane, int64_t ch,
                                                Partial partial) {
  const uint64_t t0 = wall_clock64();
  float norm;
  for (;;) {
    if (poll_norm_wave(a, ti, lane, norm)) return norm;
    if (wg_aborted()) return 1.0f;  // the payload is already invalid: just drain
    if (ufirst((int)(wall_clock64() - t0 > a.wait_ticks))) break;
    __builtin_amdgcn_s_sleep(2);
  }
  double p = 0.0;
  for (int c = 0; c < ti.nchunks; ++c) {
    const int64_t cb = ti.begin + (int64_t)c * ch;
    const int n = (int)min(ch, ti.begin + ti.n - cb);
    const float part = partial(cb, n);
    if ((c & 63) == lane) p += (double)part;
  }
  if (lane == 0) __hip_atomic_fetch_or(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ufirst(finish_norm(wave_sum_f64(p), a.fmt));
}

// The LDS ring's chunk partial: LW loader-wave partials folded in order.
template <int ROWS, int LW>
__device__ __forceinline__ float wait_norm_wave(const Args& a, const Tensor& ti, int lane) {
  return wait_norm_poll(a, ti, lane, (int64_t)ROWS * 1024, [&](int64_t cb, int n) {
    double fold = 0.0;
    for (int w = 0; w < LW; ++w) fold += wave_sum_f64((double)loader_sumsq<ROWS, LW>(a, cb, n, w, lane));
    return (float)fold;
  });
}

// ROWS rows per chunk, S LDS slots, LW loader waves (the other 16 - LW quantise), DB:
// loaders double-buffer their registers (prefetch two chunks ahead).
template <int ROWS, int S, int LW, bool DB, int WIDTH, bool HAS_U, bool HELP_ = !DB>
__global__ __launch_bounds__(1024, 4) void qsgd_encode_pc(Args a, const Item* __restrict__ items,
                                                          const Tensor* __restrict__ tinfo) {
  // items / tinfo are read-only for the launch: __restrict__ lets the compiler use scalar
  // (SMEM) loads, whose lgkmcnt waits never drain the in-flight chunk loads and payload
  // stores the way a vector table load's vmcnt(0) would.
  constexpr int QW = 16 - LW;               // quantiser waves
  constexpr int RPW = ROWS / LW;            // rows per loader wave
  constexpr int VL = RPW * 4;               // float4 per loader lane
  constexpr int CH = ROWS * 1024;           // chunk elements
  static_assert(ROWS % 4 == 0 && ROWS % LW == 0 && S >= 2, "configuration");
  constexpr int PR = 4;  // partial records (per chunk, decoupled from LDS slots)
  constexpr int NTL = ROWS;   // quantisation tiles per chunk (4 rows x 64 float4 positions each)
  constexpr int QC = QW - 1;  // claiming quantiser waves (quantiser wave 0 polls norms)
  constexpr bool HELP = HELP_;  // loaders claim tiles of a slot's previous chunk before refilling it
  constexpr uint32_t PER_USE = NTL + QC + (HELP ? LW : 0);  // claim tickets per quantised use of a slot
  __shared__ float4 slots[S][ROWS * 256];
  __shared__ double lpart[PR][LW];
  __shared__ float qnorm[S];
  __shared__ uint32_t rarrive[PR], rgen[PR];
  __shared__ uint32_t fill[S], loaded[S], freed[S], qready[S], tclaim[S], tfin[S];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = ufirst(t >> 6);
  if (t < S) {
    fill[t] = 0; loaded[t] = 0; freed[t] = 0; qready[t] = 0; tclaim[t] = 0; tfin[t] = 0;
  }
  if (t < PR) {
    rarrive[t] = 0;
    rgen[t] = (uint32_t)t;  // record r first serves chunk r
  }
  if (t == 0) g_wg_abort = 0;
  __syncthreads();
  const int64_t G = gridDim.x, n_items = a.n_items;
  const uint64_t t_start = __builtin_readcyclecounter();
  Prof prof;

  // Claim and quantise tiles of the chunk in slot s (its `use`-th quantised use, chunk k)
  // until a claim fails.  Every claimer (the QW-1 quantiser waves, and each loader wave
  // before it refills the slot) takes exactly one failing ticket per use.
  auto claim_tiles = [&](int s, uint32_t use, int64_t k, const Item& it) {
    const uint32_t base = PER_USE * use;
    const bool full = it.end - it.begin == CH;
    const int64_t coff = it.begin - it.tbegin;
    float norm = 0.0f;
    Divisor dv(1.0f);
    bool have_norm = false;
    for (;;) {
      const uint32_t c = (uint32_t)ufirst((int)(lane == 0 ? lds_add(&tclaim[s], 1u) : 0u)) - base;
      if (c >= (uint32_t)NTL) break;
      const int rg = (int)(c >> 2), j = 64 * (int)(c & 3) + lane;
      float4 uu[4];
      if (!(a.dbg & 2)) draws_at<HAS_U>(a, rg, j, it.begin, it.end, coff, it.tensor, full, uu);
      if (!have_norm) {  // a tile is held, so the slot cannot be recycled under us
        const uint64_t c2 = __builtin_readcyclecounter();
        lds_wait_ge(a, &qready[s], (uint32_t)(k + 1));
        norm = ufirst(qnorm[s]);
        dv = Divisor(norm, a.fmt);
        have_norm = true;
        prof.add(4, __builtin_readcyclecounter() - c2);
      }
      const uint64_t c3 = __builtin_readcyclecounter();
      if (!(a.dbg & 2)) {
        float4 w4[4];
#pragma unroll
        for (int sl = 0; sl < 4; ++sl) w4[sl] = slots[s][(4 * rg + sl) * 256 + j];
        quant_group_at<WIDTH>(a, w4, uu, rg, j, it.begin, it.end, dv, !(norm != 0.0f));
      }
      lds_drain();
      const uint32_t d = ufirst((int)(lane == 0 ? lds_add(&tfin[s], 1u) : 0u));
      if (d == (uint32_t)NTL * (use + 1) - 1 && lane == 0) lds_st(&freed[s], (uint32_t)(k + 1));
      prof.add(5, __builtin_readcyclecounter() - c3);
    }
  };

  if (wave < LW) {
    // ------------------------------------------------------------ loader
    // A chunk's partial is published as soon as its data lands, before the loader waits
    // for an LDS slot (and the prefetched chunk is published too before any such wait):
    // a workgroup whose quantisers fall behind never delays another workgroup's norms.
    const int w = wave;
    auto issue = [&](float4 (&v)[VL], const Item& it) {
      const float* __restrict__ xb = a.x + it.begin;
      const int n = (int)(it.end - it.begin);
      if (n == CH) {  // block-uniform: every chunk but a tensor's last
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
          for (int m = 0; m < 4; ++m)
            v[4 * r + m] = *reinterpret_cast<const float4*>(xb + (w * RPW + r) * 1024 + 4 * (lane + 64 * m));
      } else {
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int i = (w * RPW + r) * 1024 + 4 * (lane + 64 * m);
            float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i + 4 <= n) {
              z = *reinterpret_cast<const float4*>(xb + i);
            } else {
              if (i < n) z.x = xb[i];
              if (i + 1 < n) z.y = xb[i + 1];
              if (i + 2 < n) z.z = xb[i + 2];
            }
            v[4 * r + m] = z;
          }
      }
    };
    // Scale, reduce and publish chunk k (data in v).
    auto publish = [&](float4 (&v)[VL], const Item& it, int64_t k) {
      const uint64_t c1 = __builtin_readcyclecounter();
      float acc = 0.0f;
#pragma unroll
      for (int q = 0; q < VL; ++q) {
        v[q] = prologue4(a, v[q]);
        acc = sumsq4(v[q], acc);
      }
      if (a.xout && (it.flags & kPublish)) {  // PS fusion: write the averaged parameters once
        float* __restrict__ ob = a.xout + it.begin;
        const int n = (int)(it.end - it.begin);
#pragma unroll
        for (int r2 = 0; r2 < RPW; ++r2)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int i = (w * RPW + r2) * 1024 + 4 * (lane + 64 * m);
            const float4 o = v[4 * r2 + m];
            if (n == CH || i + 4 <= n) {
              store_nt(ob + i, o);
            } else {
              if (i < n) ob[i] = o.x;
              if (i + 1 < n) ob[i + 1] = o.y;
              if (i + 2 < n) ob[i + 2] = o.z;
            }
          }
      }
      const int r = (int)(k % PR);
      if (it.flags & kPublish) {
        const double wp = wave_sum_f64((double)acc);
        lds_wait_ge(a, &rgen[r], (uint32_t)k);  // record free (chunk k-PR folded)
        if (lane == 0) lpart[r][w] = wp;
        lds_drain();
        const uint32_t old = ufirst((int)(lane == 0 ? lds_add(&rarrive[r], 1u) : 0u));
        if (old == LW - 1) {  // last loader wave: fold in wave order, publish the granule
          double fold = 0.0;
#pragma unroll
          for (int j = 0; j < LW; ++j) fold += lpart[r][j];
          if (lane == 0) {
            st_agent(&a.gran[it.gbase + it.chunk], ((uint64_t)a.epoch << 32) | (uint64_t)__float_as_uint((float)fold));
            lds_st(&rarrive[r], 0u);
            lds_drain();
            lds_st(&rgen[r], (uint32_t)(k + PR));
          }
        }
      } else if (w == 0) {  // QUANT chunk: no partial, retire the record
        lds_wait_ge(a, &rgen[r], (uint32_t)k);
        if (lane == 0) lds_st(&rgen[r], (uint32_t)(k + PR));
      }
      prof.add(1, __builtin_readcyclecounter() - c1);
    };
    // Step on chunk k (already published): wait for its slot (publishing the in-flight
    // chunk k+1 first if the slot is busy), fill the slot, issue the loads of k+2, then
    // publish k+1 as soon as its data lands.  So a workgroup's published chunks run one
    // step ahead of its slot turnover, and a blocked loader holds no unpublished chunk.
    uint32_t uses[S];  // quantised uses of each slot so far (identical in every wave)
#pragma unroll
    for (int q = 0; q < S; ++q) uses[q] = 0;
    auto step = [&](float4 (&v)[VL], Item& it, int64_t& idx, int64_t& k, float4 (&vo)[VL], const Item& ito,
                    int64_t idxo, int64_t ko, bool& pubo) {
      const int s = (int)(k % S);
      const uint64_t c0 = __builtin_readcyclecounter();
      if (k >= S) {
        const Item prev = items[idx - (int64_t)S * G];  // the slot's current occupant, chunk k - S
        if (HELP && (prev.flags & kQuant)) {  // (single-buffered: no other chunk is held)
          uint32_t use = 0;
#pragma unroll
          for (int q = 0; q < S; ++q)
            if (q == s) use = uses[q]++;
          // Like every claimer: not before all claimers have left the slot's previous use.
          // (freed only says its tiles are done; a late claimer's failing ticket may still
          // be outstanding, and a ticket taken before it would steal this use's tile 0.)
          lds_wait_ge(a, &tclaim[s], PER_USE * use);
          claim_tiles(s, use, k - S, prev);  // help quantise it (takes this wave's failing ticket)
        }
        if (ufirst((int)lds_ld(&freed[s])) < (int)(k - S + 1) && DB && idxo < n_items && !pubo) {
          publish(vo, ito, ko);  // never hold an unpublished chunk while waiting
          pubo = true;
        }
        lds_wait_ge(a, &freed[s], (uint32_t)(k - S + 1));
      }
      prof.add(0, __builtin_readcyclecounter() - c0);
      if (it.flags & kQuant) {
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
          for (int m = 0; m < 4; ++m) slots[s][(w * RPW + r) * 256 + lane + 64 * m] = v[4 * r + m];
        lds_drain();
        const uint32_t old = ufirst((int)(lane == 0 ? lds_add(&fill[s], 1u) : 0u));
        if (old == LW - 1 && lane == 0) {
          lds_st(&fill[s], 0u);
          lds_drain();
          // test hook (omf_plan_set_debug ring bit 8): the slot is never marked loaded, so the
          // poller's hand-off wait expires and the workgroup aborts (err bit 4, OMF_ETIMEOUT)
          if (!(a.dbg & 8)) lds_st(&loaded[s], (uint32_t)(k + 1));
        }
      } else if (w == 0 && lane == 0) {
        lds_st(&freed[s], (uint32_t)(k + 1));  // NORM chunk: the slot stays free
      }
      idx += (DB ? 2 : 1) * G;
      k += DB ? 2 : 1;
      if (idx < n_items) {
        it = items[idx];
        issue(v, it);
      }
      if (DB && idxo < n_items && !pubo) {
        publish(vo, ito, ko);
        pubo = true;
      }
    };
    if (DB) {
      int64_t ia = blockIdx.x, ib = ia + G, ka = 0, kb = 1;
      bool pa = true, pb = false;  // chunk 0 is published in the prologue
      float4 va[VL], vb[VL];
      Item ita{}, itb{};
      if (ia < n_items) { ita = items[ia]; issue(va, ita); }
      if (ib < n_items) { itb = items[ib]; issue(vb, itb); }
      if (ia < n_items) publish(va, ita, ka);
      for (;;) {
        if (ia >= n_items) break;
        pa = false;  // the chunk step() loads into va next is unpublished
        step(va, ita, ia, ka, vb, itb, ib, kb, pb);
        if (ib >= n_items) break;
        pb = false;
        step(vb, itb, ib, kb, va, ita, ia, ka, pa);
      }
    } else {
      int64_t ia = blockIdx.x, ka = 0;
      bool pn = true;
      float4 va[VL];
      Item ita{};
      if (ia < n_items) { ita = items[ia]; issue(va, ita); publish(va, ita, ka); }
      while (ia < n_items) {
        step(va, ita, ia, ka, va, ita, n_items, ka, pn);
        if (ia < n_items) publish(va, ita, ka);
      }
    }
    prof.add(6, __builtin_readcyclecounter() - t_start);
    prof.flush(a);
    return;
  }

  // -------------------------------------------------------------- quantiser
  // Wave LW is a dedicated POLLER: it resolves each chunk's norm (its only memory
  // operations are granule polls, so a poll returns at load latency — a wave with payload
  // stores in flight would wait for them first: vmcnt retires in order) and publishes it
  // in the slot's norm record.  The other QW-1 waves CLAIM 64-group tiles of the chunk
  // (ROWS tiles per chunk) from a per-slot counter: every claimer takes tickets until one
  // fails, so each use of a slot advances the counter by exactly ROWS + QW - 1 and it
  // never needs resetting.
  const int qw = wave - LW;
  int64_t k = 0;
  Item nx = blockIdx.x < n_items ? items[blockIdx.x] : Item{};
  if (qw == 0) {
    int32_t cached_t = -1;
    float cached_norm = 0.0f;
    for (int64_t idx = blockIdx.x; idx < n_items; idx += G, ++k) {
      const Item it = nx;
      if (idx + G < n_items) nx = items[idx + G];
      if (!(it.flags & kQuant)) continue;
      const int s = (int)(k % S);
      const uint64_t c0 = __builtin_readcyclecounter();
      float norm;
      if (it.tensor == cached_t) {
        norm = cached_norm;
      } else if (a.dbg & 1) {
        norm = 1.0f;
      } else {
        norm = wait_norm_wave<ROWS, LW>(a, tensor_of(it), lane);
        cached_t = it.tensor;
        cached_norm = norm;
      }
      const uint64_t c1 = __builtin_readcyclecounter();
      prof.add(3, c1 - c0);
      lds_wait_ge(a, &loaded[s], (uint32_t)(k + 1));  // the slot's previous chunk is finished
      prof.add(2, __builtin_readcyclecounter() - c1);
      if (lane == 0) {
        qnorm[s] = norm;
        lds_drain();
        lds_st(&qready[s], (uint32_t)(k + 1));
        if (it.chunk == 0) a.norm_out[it.tensor] = norm;
      }
    }
  } else {
    uint32_t uses[S];  // quantised uses of each slot so far (identical in every claimer)
#pragma unroll
    for (int q = 0; q < S; ++q) uses[q] = 0;
    for (int64_t idx = blockIdx.x; idx < n_items; idx += G, ++k) {
      const Item it = nx;
      if (idx + G < n_items) nx = items[idx + G];  // prefetch: the scalar load overlaps this chunk
      if (!(it.flags & kQuant)) continue;
      const int s = (int)(k % S);
      uint32_t use = 0;
#pragma unroll
      for (int q = 0; q < S; ++q)
        if (q == s) use = uses[q]++;
      const uint64_t c0 = __builtin_readcyclecounter();
      // Claim before the chunk has landed: the first tile's draws are computed while the
      // slot fills and the norm resolves (the data is read only after qready, which the
      // poller sets after `loaded`, which the loaders set after every tile of the slot's
      // previous use is finished).
      lds_wait_ge(a, &tclaim[s], PER_USE * use);  // every claimer has left the slot's previous use
      prof.add(2, __builtin_readcyclecounter() - c0);
      claim_tiles(s, use, k, it);
    }
  }
  prof.add(7, __builtin_readcyclecounter() - t_start);
  prof.flush(a);
}

// ---------------------------------------------------------------- register-resident kernel
//
// Every wave streams its own part of each chunk through registers: no LDS staging and no
// producer/consumer hand-off.  Thread t owns the Philox group (rg = t >> 8, j = t & 255)
// of every 64 KiB chunk: rows 4rg .. 4rg+3 at float4 column j (a wave reads 1 KiB
// contiguous per instruction).  Position p of a workgroup is its p-th item (sequence index
// blockIdx.x + p * grid).  With D register buffers per thread, step p:
//   1. issues the loads of position p+D-1 (its buffer was freed by step p-1);
//   2. publishes position p+1 as soon as it lands (prologue; thread fp32 chain -> wave
//      fp64 butterfly -> the 16 wave partials folded in wave order in LDS -> one granule);
//   3. resolves the norm of position p's tensor: wave 0 (the poller) consumes the granule
//      poll it issued at the end of step p-1 (or polls again) and hands the norm to the
//      other waves through LDS;
//   4. quantises position p from registers and stores the payload;
//   5. (poller) issues the granule poll for position p+1's tensor.  It is consumed in step
//      p+1 before anything else waits on memory, so its wait (vmcnt retires in issue
//      order) covers only what was issued before it, never step p+1's chunk loads.
// The plan packs every single-read tensor inside one sequence row (all its chunks share
// one position; omf_qsgd.hip build_ring_sequence), so position p's norm needs only
// position-p publishes, which every workgroup makes one step before it needs a norm:
// deadlock-free, with a quantisation step of slack for workgroups that lag.  Tensors of
// more than one row are NORM items (publish only, never wait) ahead of their QUANT items.

// The register-resident chunk partial (fallback recompute): thread (w, lane)'s four
// float4 in row order, wave butterfly, waves folded in order — the publish order exactly.
__device__ __forceinline__ float rr_chunk_partial(const Args& a, int64_t cb, int n, int lane) {
  const __amdgpu_buffer_rsrc_t rx = chunk_rsrc(a.x + cb, 4 * (int64_t)n);
  double fold = 0.0;
  for (int w = 0; w < 16; ++w) {
    const int voff = 4 * ((w >> 2) * 4096 + 4 * (((w & 3) << 6) + lane));
    float acc = 0.0f;
    for (int sl = 0; sl < 4; ++sl) acc = sumsq4(prologue4(a, ld_row(rx, voff, sl)), acc);
    fold += wave_sum_f64((double)acc);
  }
  return (float)fold;
}

template <int D, int L, int WIDTH, bool HAS_U>
__global__ __launch_bounds__(1024, 4) void qsgd_encode_rr(Args a, const Item* __restrict__ items,
                                                          const Tensor* __restrict__ tinfo) {
  static_assert(L >= 1 && D >= L + 2, "step p publishes p+L while p+L+1 .. p+D-1 stay in flight");
  constexpr int CH = 16 * 1024, NW = 16, PR = 4;
  constexpr int NP = 4;  // granules per lane of an early poll (tensors of <= 256 chunks)
  __shared__ double lpart[PR][NW];
  __shared__ uint32_t rarrive[PR], rgen[PR];
  __shared__ float qnorm[2];
  __shared__ uint32_t qflag[2], qdone[2];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = ufirst(t >> 6);
  const int rg = wave >> 2, j = ((wave & 3) << 6) + lane;
  const int voff = 4 * (rg * 4096 + 4 * j);  // byte offset of this thread's row-0 float4 in a chunk
  if (t < PR) {
    rarrive[t] = 0;
    rgen[t] = (uint32_t)t;
  }
  if (t < 2) {
    qflag[t] = 0;
    qdone[t] = 0;
    qnorm[t] = 0.0f;
  }
  if (t == 0) g_wg_abort = 0;
  __syncthreads();
  const int64_t G = gridDim.x, n_items = a.n_items;
  const int64_t npos = (n_items - (int64_t)blockIdx.x + G - 1) / G;
  // Position p's item; past the end an empty item (no flags, no elements), so that every
  // step issues the same memory instructions (zero-size descriptors) without a branch.
  auto item_at = [&](int64_t p) __attribute__((always_inline)) -> Item {
    Item it = items[(int64_t)blockIdx.x + min(p, npos - 1) * G];
    if (p >= npos) {
      it.flags = 0;
      it.end = it.begin;
    }
    return it;
  };

  auto load = [&](float4 (&v)[4], int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const __amdgpu_buffer_rsrc_t rx = chunk_rsrc(a.x + it.begin, 4 * (it.end - it.begin));
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) v[sl] = ld_row(rx, voff, sl);
  };

  uint32_t npub = 0;  // publishes so far (identical in every wave)
  auto publish = [&](float4 (&v)[4], int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const bool pub = (it.flags & kPublish) != 0;
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) v[sl] = prologue4(a, v[sl]);
    // PS fusion: the averaged parameters, written once (a no-op descriptor otherwise)
    const __amdgpu_buffer_rsrc_t ro =
        chunk_rsrc(a.xout ? a.xout + it.begin : a.x, a.xout && pub ? 4 * (it.end - it.begin) : 0);
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) st_row(ro, voff, sl, v[sl]);
    bool last = false;
    double fold = 0.0;
    if (pub) {
      float acc = 0.0f;
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) acc = sumsq4(v[sl], acc);
      const double wp = wave_sum_f64((double)acc);
      const int r = (int)(npub % PR);
      lds_wait_ge(a, &rgen[r], npub);  // record free (publish npub - PR folded)
      if (lane == 0) lpart[r][wave] = wp;
      lds_drain();
      const uint32_t old = ufirst((int)(lane == 0 ? lds_add(&rarrive[r], 1u) : 0u));
      if (old == NW - 1) {  // last wave in: fold in wave order
        last = true;
#pragma unroll
        for (int w = 0; w < NW; ++w) fold += lpart[r][w];
        if (lane == 0) {
          lds_st(&rarrive[r], 0u);
          lds_drain();
          lds_st(&rgen[r], npub + PR);
        }
      }
      ++npub;
    }
    // the granule (sc1 store of lane 0 of the last wave; every other lane stores nothing)
    const __amdgpu_buffer_rsrc_t rgr = chunk_rsrc(a.gran + it.gbase + it.chunk, last && lane == 0 ? 8 : 0);
    __builtin_amdgcn_raw_buffer_store_b64((u32x2_t){__float_as_uint((float)fold), a.epoch}, rgr, 0, 0, kAuxSC1);
  };

  // Norm hand-off: resolution r uses LDS slot r & 1; wave 0 writes it once the other 15
  // waves have read the slot's previous use (qdone), and raises qflag.
  int32_t cached_t = -1;
  float cached_norm = 0.0f;
  uint32_t nres = 0;
  u32x2_t pg[NP];
  int32_t pend_t = -1;  // tensor of wave 0's outstanding early poll
  auto consume_poll = [&](const Item& it, float& norm) __attribute__((always_inline)) -> bool {
    double sum = 0.0;  // poll_norm_wave's fold
    int ok = 1;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (lane + 64 * i < it.nchunks) {
        ok &= pg[i].y == a.epoch;
        sum += (double)__uint_as_float(pg[i].x);
      }
    }
    if (!__all(ok)) return false;
    norm = ufirst(finish_norm(wave_sum_f64(sum), a.fmt));
    return true;
  };
  auto resolve = [&](const Item& it) __attribute__((always_inline)) -> float {
    if (it.tensor == cached_t) return cached_norm;
    const int s = (int)(nres & 1);
    const uint32_t use = nres >> 1;
    ++nres;
    float norm = 1.0f;
    if (wave == 0) {
      bool ok = (a.dbg & 1) != 0;
      if (!ok && pend_t == it.tensor) ok = consume_poll(it, norm);
      if (!ok)
        norm = wait_norm_poll(a, tensor_of(it), lane, CH,
                              [&](int64_t cb, int n) { return rr_chunk_partial(a, cb, n, lane); });
      lds_wait_ge(a, &qdone[s], (uint32_t)(NW - 1) * use);
      if (lane == 0) {
        qnorm[s] = norm;
        lds_drain();
        lds_st(&qflag[s], use + 1);
      }
    } else {
      lds_wait_ge(a, &qflag[s], use + 1);
      norm = ufirst(qnorm[s]);
      if (lane == 0) lds_add(&qdone[s], 1u);
    }
    cached_t = it.tensor;
    cached_norm = norm;
    return norm;
  };

  auto quantise = [&](const float4 (&v)[4], int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const int64_t n = it.end - it.begin;
    if (it.flags & kQuant) {
      const float norm = resolve(it);
      if (it.chunk == 0 && wave == 0 && lane == 0) a.norm_out[it.tensor] = norm;
      const __amdgpu_buffer_rsrc_t ru = chunk_rsrc(HAS_U ? a.u + it.begin : a.x, HAS_U ? 4 * n : 0);
      if (!(a.dbg & 2))
        quant_group_rr<WIDTH, HAS_U>(a, v, rg, j, it.begin - it.tbegin, it.tensor, norm,
                                     payload_rsrc(a, WIDTH, it.begin, n), ru, voff);
    } else {  // the same stores, through a no-op descriptor
      const __amdgpu_buffer_rsrc_t rq = chunk_rsrc(a.q, 0);
      const int32_t zq[4] = {0, 0, 0, 0};
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) st_levels<WIDTH>(rq, voff >> 2, sl, zq);
    }
  };

  // Early poll for position p's tensor: wave 0 reads the granules when p needs a new norm;
  // every other wave (and wave 0 otherwise) issues the same loads through a no-op descriptor.
  auto poll_next = [&](int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const bool need = wave == 0 && (it.flags & kQuant) && it.tensor != cached_t && it.nchunks <= 64 * NP &&
                      !(a.dbg & 1);
    const __amdgpu_buffer_rsrc_t rp = chunk_rsrc(a.gran + it.gbase, need ? 8 * (int64_t)it.nchunks : 0);
#pragma unroll
    for (int i = 0; i < NP; ++i) pg[i] = __builtin_amdgcn_raw_buffer_load_b64(rp, 8 * (lane + 64 * i), 0, kAuxSC1);
    pend_t = need ? it.tensor : -1;
  };

  // Buffer indices must be compile-time constants (registers, not scratch): each step of a
  // D-step round is instantiated with its own index.  Steps past the end are empty.
  float4 buf[D][4];
  auto step = [&](int64_t p0, auto bc) __attribute__((always_inline)) {
    constexpr int b = decltype(bc)::value;
    const int64_t p = p0 + b;
    load(buf[(b + D - 1) % D], p + D - 1);
    publish(buf[(b + L) % D], p + L);
    quantise(buf[b], p);
    poll_next(p + 1);
  };
  auto round = [&](int64_t p0, auto seq) __attribute__((always_inline)) {
    [&]<int... B>(std::integer_sequence<int, B...>) __attribute__((always_inline)) {
      (step(p0, std::integral_constant<int, B>{}), ...);
    }(seq);
  };
  auto prologue = [&]<int... B>(std::integer_sequence<int, B...>) __attribute__((always_inline)) {
    (load(buf[B], B), ...);
  };
  auto prologue_pub = [&]<int... B>(std::integer_sequence<int, B...>) __attribute__((always_inline)) {
    (publish(buf[B], B), ...);
  };
  prologue(std::make_integer_sequence<int, D - 1>{});
  prologue_pub(std::make_integer_sequence<int, L>{});
  for (int64_t p0 = 0; p0 < npos; p0 += D) round(p0, std::make_integer_sequence<int, D>{});
}

template <int WIDTH, bool HAS_U>
__global__ __launch_bounds__(1024, 4) void qsgd_encode_rr2(Args a, const Item* __restrict__ items,
                                                          const Tensor* __restrict__ tinfo) {
  constexpr int L = 2;  // step p publishes p+2
  constexpr int CH = 16 * 1024, NW = 16, PR = 4;
  constexpr int NP = 4;  // granules per lane of an early poll (tensors of <= 256 chunks)
  __shared__ float4 hold[2][4][1024];  // published chunks p+1, p+2 wait here for their norms
  __shared__ double lpart[PR][NW];
  __shared__ uint32_t rarrive[PR], rgen[PR];
  __shared__ float qnorm[2];
  __shared__ uint32_t qflag[2], qdone[2];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = ufirst(t >> 6);
  const int rg = wave >> 2, j = ((wave & 3) << 6) + lane;
  const int voff = 4 * (rg * 4096 + 4 * j);  // byte offset of this thread's row-0 float4 in a chunk
  if (t < PR) {
    rarrive[t] = 0;
    rgen[t] = (uint32_t)t;
  }
  if (t < 2) {
    qflag[t] = 0;
    qdone[t] = 0;
    qnorm[t] = 0.0f;
  }
  if (t == 0) g_wg_abort = 0;
  __syncthreads();
  const int64_t G = gridDim.x, n_items = a.n_items;
  const int64_t npos = (n_items - (int64_t)blockIdx.x + G - 1) / G;
  // Position p's item; past the end an empty item (no flags, no elements), so that every
  // step issues the same memory instructions (zero-size descriptors) without a branch.
  auto item_at = [&](int64_t p) __attribute__((always_inline)) -> Item {
    Item it = items[(int64_t)blockIdx.x + min(p, npos - 1) * G];
    if (p >= npos) {
      it.flags = 0;
      it.end = it.begin;
    }
    return it;
  };

  auto load = [&](float4 (&v)[4], int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const __amdgpu_buffer_rsrc_t rx = chunk_rsrc(a.x + it.begin, 4 * (it.end - it.begin));
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) v[sl] = ld_row(rx, voff, sl);
  };

  uint32_t npub = 0;  // publishes so far (identical in every wave)
  auto publish = [&](float4 (&v)[4], int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const bool pub = (it.flags & kPublish) != 0;
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) v[sl] = prologue4(a, v[sl]);
    // PS fusion: the averaged parameters, written once (a no-op descriptor otherwise)
    const __amdgpu_buffer_rsrc_t ro =
        chunk_rsrc(a.xout ? a.xout + it.begin : a.x, a.xout && pub ? 4 * (it.end - it.begin) : 0);
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) st_row(ro, voff, sl, v[sl]);
    bool last = false;
    double fold = 0.0;
    if (pub) {
      float acc = 0.0f;
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) acc = sumsq4(v[sl], acc);
      const double wp = wave_sum_f64((double)acc);
      const int r = (int)(npub % PR);
      lds_wait_ge(a, &rgen[r], npub);  // record free (publish npub - PR folded)
      if (lane == 0) lpart[r][wave] = wp;
      lds_drain();
      const uint32_t old = ufirst((int)(lane == 0 ? lds_add(&rarrive[r], 1u) : 0u));
      if (old == NW - 1) {  // last wave in: fold in wave order
        last = true;
#pragma unroll
        for (int w = 0; w < NW; ++w) fold += lpart[r][w];
        if (lane == 0) {
          lds_st(&rarrive[r], 0u);
          lds_drain();
          lds_st(&rgen[r], npub + PR);
        }
      }
      ++npub;
    }
    // the granule (sc1 store of lane 0 of the last wave; every other lane stores nothing)
    const __amdgpu_buffer_rsrc_t rgr = chunk_rsrc(a.gran + it.gbase + it.chunk, last && lane == 0 ? 8 : 0);
    __builtin_amdgcn_raw_buffer_store_b64((u32x2_t){__float_as_uint((float)fold), a.epoch}, rgr, 0, 0, kAuxSC1);
  };

  // Norm hand-off: resolution r uses LDS slot r & 1.  At the START of step p wave 0
  // resolves position p's norm (consuming the poll it issued a whole step earlier, or
  // polling again) and writes the slot once the other 15 waves have read its previous use
  // (qdone); the other waves read it when they reach the quantisation of p.
  int32_t cached_t = -1;
  float cached_norm = 0.0f;
  uint32_t nres = 0;
  int rd_slot = -1;      // other waves: the slot holding a norm not read yet
  uint32_t rd_use = 0;
  u32x2_t pg[NP];
  int32_t pend_t = -1;   // tensor of wave 0's outstanding early poll
  auto consume_poll = [&](const Item& it, float& norm) __attribute__((always_inline)) -> bool {
    double sum = 0.0;  // poll_norm_wave's fold
    int ok = 1;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (lane + 64 * i < it.nchunks) {
        ok &= pg[i].y == a.epoch;
        sum += (double)__uint_as_float(pg[i].x);
      }
    }
    if (!__all(ok)) return false;
    norm = ufirst(finish_norm(wave_sum_f64(sum), a.fmt));
    return true;
  };
  auto resolve_early = [&](int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    if (!(it.flags & kQuant) || it.tensor == cached_t) return;
    const int s = (int)(nres & 1);
    const uint32_t use = nres >> 1;
    ++nres;
    cached_t = it.tensor;
    if (wave == 0) {
      float norm = 1.0f;
      bool ok = (a.dbg & 1) != 0;
      if (!ok && pend_t == it.tensor) ok = consume_poll(it, norm);
      if (!ok)
        norm = wait_norm_poll(a, tensor_of(it), lane, CH,
                              [&](int64_t cb, int n) { return rr_chunk_partial(a, cb, n, lane); });
      lds_wait_ge(a, &qdone[s], (uint32_t)(NW - 1) * use);
      if (lane == 0) {
        qnorm[s] = norm;
        lds_drain();
        lds_st(&qflag[s], use + 1);
      }
      cached_norm = norm;
    } else {
      rd_slot = s;
      rd_use = use;
    }
  };
  auto quantise = [&](const float4 (&v)[4], int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const int64_t n = it.end - it.begin;
    if (it.flags & kQuant) {
      if (rd_slot >= 0) {
        lds_wait_ge(a, &qflag[rd_slot], rd_use + 1);
        cached_norm = ufirst(qnorm[rd_slot]);
        if (lane == 0) lds_add(&qdone[rd_slot], 1u);
        rd_slot = -1;
      }
      const float norm = cached_norm;
      if (it.chunk == 0 && wave == 0 && lane == 0) a.norm_out[it.tensor] = norm;
      const __amdgpu_buffer_rsrc_t ru = chunk_rsrc(HAS_U ? a.u + it.begin : a.x, HAS_U ? 4 * n : 0);
      if (!(a.dbg & 2))
        quant_group_rr<WIDTH, HAS_U>(a, v, rg, j, it.begin - it.tbegin, it.tensor, norm,
                                     payload_rsrc(a, WIDTH, it.begin, n), ru, voff);
    } else {  // the same stores, through a no-op descriptor
      const __amdgpu_buffer_rsrc_t rq = chunk_rsrc(a.q, 0);
      const int32_t zq[4] = {0, 0, 0, 0};
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) st_levels<WIDTH>(rq, voff >> 2, sl, zq);
    }
  };

  // Early poll for position p's tensor (issued after p-1's norm is resolved): wave 0 reads
  // the granules when p needs a new norm; every other wave (and wave 0 otherwise) issues
  // the same loads through a no-op descriptor.
  auto poll_next = [&](int64_t p) __attribute__((always_inline)) {
    const Item it = item_at(p);
    const bool need = wave == 0 && (it.flags & kQuant) && it.tensor != cached_t && it.nchunks <= 64 * NP &&
                      !(a.dbg & 1);
    const __amdgpu_buffer_rsrc_t rp = chunk_rsrc(a.gran + it.gbase, need ? 8 * (int64_t)it.nchunks : 0);
#pragma unroll
    for (int i = 0; i < NP; ++i) pg[i] = __builtin_amdgcn_raw_buffer_load_b64(rp, 8 * (lane + 64 * i), 0, kAuxSC1);
    pend_t = need ? it.tensor : -1;
  };

  // Chunk c is loaded into register buffer rb[c % 3] (chunks p+3, p+4 in flight during step
  // p), published from there into LDS slot hold[c % 2], and quantised from registers after
  // its step reads it back.  Indices are compile-time constants: a round is 6 steps.
  float4 rb[3][4], qb[4];
  auto park = [&](const float4 (&v)[4], int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) hold[slot][sl][t] = v[sl];
  };
  auto unpark = [&](float4 (&v)[4], int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) v[sl] = hold[slot][sl][t];
  };
  auto step = [&](int64_t p0, auto bc) __attribute__((always_inline)) {
    constexpr int b = decltype(bc)::value;
    const int64_t p = p0 + b;
    resolve_early(p);                // consumes the poll issued a step ago
    poll_next(p + 1);                // publishes of p+1 were made a step ago, everywhere
    unpark(qb, b % 2);               // chunk p leaves its slot ...
    publish(rb[(b + 2) % 3], p + 2);  // ... which chunk p+2 takes
    park(rb[(b + 2) % 3], b % 2);
    load(rb[(b + 2) % 3], p + 5);
    quantise(qb, p);
  };
  auto round = [&](int64_t p0, auto seq) __attribute__((always_inline)) {
    [&]<int... B>(std::integer_sequence<int, B...>) __attribute__((always_inline)) {
      (step(p0, std::integral_constant<int, B>{}), ...);
    }(seq);
  };
  load(rb[0], 0);
  load(rb[1], 1);
  load(rb[2], 2);
  publish(rb[0], 0);
  park(rb[0], 0);
  load(rb[0], 3);
  publish(rb[1], 1);
  park(rb[1], 1);
  load(rb[1], 4);
  for (int64_t p0 = 0; p0 < npos; p0 += 6) round(p0, std::make_integer_sequence<int, 6>{});
}

// Instantiated configurations: {rows of 1024 elements per chunk, LDS slots, loader
// waves, loader double-buffering}.  cfg 0 is the default (fastest measured).
constexpr Config kConfigs[] = {
    {16, 2, 8, 0},  // 64 KiB chunks x 2 slots, 8 loader + 1 poller + 7 claimer waves, loaders help
    {16, 2, 8, 1},  // same with double-buffered loaders (no spare registers to help: they only load)
    {8, 4, 8, 1},   // 32 KiB chunks x 4 slots (per-chunk synchronisation dominates: slower)
    {16, 4, 0, 0, 1},  // register-resident: 64 KiB chunks, 4 register buffers per thread, lookahead 1
    {16, 3, 0, 0, 1},  // register streams + 2 LDS slots for published chunks: lookahead 2
};
// Measured and dropped (Llama-400M, round 2): 48 KiB x 3 slots with 4 / 6 / 12
// loader waves 0.84 / 0.63 / 0.78 ms, 32 KiB x 4 slots with 8 / 4 loader waves 0.78 / 0.71 ms,
// 64 KiB x 2 with 4 loader waves 0.85 ms; double-buffered loaders that also help quantise
// 0.68 ms (64 KiB x 2), 0.70 (48 KiB x 3, 12 one-row loaders), 0.76 (32 KiB x 4) — against
// cfg 0's 0.63 ms.  With quantisation and norm waits switched off (OMF_RING_DBG=3) every one
// of them still takes 0.40-0.55 ms: the hand-off machinery, not the slot count, sets the pace.

template <int ROWS, int S, int LW, bool DB, bool HELP = !DB>
const void* kernel_ptr(int width, bool has_u) {
  if (width == 1) {
    return has_u ? (const void*)qsgd_encode_pc<ROWS, S, LW, DB, 1, true, HELP>
                 : (const void*)qsgd_encode_pc<ROWS, S, LW, DB, 1, false, HELP>;
  }
  return has_u ? (const void*)qsgd_encode_pc<ROWS, S, LW, DB, 4, true, HELP>
               : (const void*)qsgd_encode_pc<ROWS, S, LW, DB, 4, false, HELP>;
}

// Caller uniforms (parity mode) hold 16 more registers per thread: 3 buffers keep them unspilled.
template <int D, int L>
const void* kernel_ptr_rr(int width, bool has_u) {
  if (width == 1) return has_u ? (const void*)qsgd_encode_rr<3, 1, 1, true> : (const void*)qsgd_encode_rr<D, L, 1, false>;
  return has_u ? (const void*)qsgd_encode_rr<3, 1, 4, true> : (const void*)qsgd_encode_rr<D, L, 4, false>;
}

const void* kernel_for(int cfg, int width, bool has_u) {
  switch (cfg) {
    case 3: return kernel_ptr_rr<4, 1>(width, has_u);
    case 4:
      if (width == 1) return has_u ? (const void*)qsgd_encode_rr2<1, true> : (const void*)qsgd_encode_rr2<1, false>;
      return has_u ? (const void*)qsgd_encode_rr2<4, true> : (const void*)qsgd_encode_rr2<4, false>;
    case 1: return kernel_ptr<16, 2, 8, true>(width, has_u);
    case 2: return kernel_ptr<8, 4, 8, true>(width, has_u);
    default: return kernel_ptr<16, 2, 8, false>(width, has_u);
  }
}

}  // namespace

int num_configs() { return (int)(sizeof(kConfigs) / sizeof(kConfigs[0])); }

Config config(int cfg) { return kConfigs[(cfg >= 0 && cfg < num_configs()) ? cfg : 0]; }

int grid_size(int cfg, int device) {
  (void)cfg;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  return prop.multiProcessorCount;  // one 1024-thread workgroup per CU (the LDS ring fills it)
}

int launch(int cfg, int width, bool has_u, const Args& a, int grid, hipStream_t st) {
  const void* k = kernel_for(cfg, width == 1 ? 1 : 4, has_u);
  if (!k) return -1;
  Args args = a;
  const Item* items = a.items;
  const Tensor* tinfo = a.tinfo;
  void* params[] = {&args, &items, &tinfo};
  return hipLaunchKernel(k, dim3((unsigned)grid), dim3(1024), params, 0, st) == hipSuccess ? 0 : -1;
}

}  // namespace ring
}  // namespace omf
