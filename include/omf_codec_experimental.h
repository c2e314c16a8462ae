/*
 * omf_codec_experimental.h — test and experiment hooks of the MI355X codec library.
 *
 * NOT part of the drop-in boundary (include/omf_codec.h): these entry points tune or
 * instrument the encoders — switches that skip launches or quantisation, ring / bracket /
 * Top-K tuning, per-phase counters — for the GPU test suite and the measurements recorded
 * in DESIGN.md.  Production callers never need them; every default is the measured choice.
 * The product library also ignores its environment (the OMF_* tuning variables are read by
 * experiment builds only, -DOMF_EXPERIMENTS).
 */
#ifndef OMF_CODEC_EXPERIMENTAL_H
#define OMF_CODEC_EXPERIMENTAL_H

#include "omf_codec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Test / experiment hook, never set in production (all 0): switches that change what an
 * encode writes.  ring_dbg (ring encoder): 1 no norm wait (norm := 1), 2 no quantisation,
 * 4 phase cycle counters, 8 slots never marked loaded (every hand-off wait of the poller
 * expires: OMF_ETIMEOUT).  spec_dbg (bracketed encoder): 1 no bracket launch, 2 no finish
 * launch, 4 no fix stores, 8 no fix, 16 no fold (every fix wait expires: OMF_ETIMEOUT);
 * grid encoder: 32 arrive after the wait (every wait expires, exact recovery), 64 no barrier
 * wait, 128 no norm fold (norm := 1), 256 no quantisation (phase timings).
 * lds_wait_us > 0 replaces the ring's 20 ms hand-off bound (0 restores it); the norm-wait
 * bound is omf_plan_set_resident_capacity's wait_us. */
int omf_plan_set_debug(omf_plan* plan, uint32_t ring_dbg, uint32_t spec_dbg, int64_t lds_wait_us);
/* Ring encoder tuning / test hook (rebuilds the chunk sequence; not for the hot path):
 * cfg = kernel configuration (-1 keep), big_mode 0/1 (placement of second-read chunks,
 * -1 keep), gap = items between a large tensor's first and second pass (-2 keep, -1 one
 * grid), hold_max = largest tensor (chunks) read once (0 = slots x grid, -1 keep). */
int omf_plan_set_ring(omf_plan* plan, int32_t cfg, int32_t big_mode, int64_t gap, int64_t hold_max);
/* Ring encoder facts: out[0] grid, out[1] chunk elements, out[2] items, out[3] hold limit
 * (chunks), out[4] tensors taking two passes, out[5] configuration. */
int omf_plan_ring_info(const omf_plan* plan, int64_t* out6);
/* Experiment hook: per-phase cycle totals of ring launches made with omf_plan_set_debug
 * ring bit 4 (zeros otherwise); read and reset. */
int omf_plan_ring_profile(omf_plan* plan, int64_t* out16);
/* Largest tensor (in 16 Ki-element items) that takes the register-resident path: half the
 * encoder's co-resident workgroups (occupancy x CUs). */
int64_t omf_plan_resident_capacity(const omf_plan* plan);
/* Tuning / test hook: cap > 0 replaces the capacity (rebuilds the item sequence; not for
 * the hot path); wait_us > 0 bounds each norm wait (default 20 ms) after which a workgroup
 * recomputes the norm itself (exact, reported by omf_plan_check). */
int omf_plan_set_resident_capacity(omf_plan* plan, int64_t cap, int64_t wait_us);
/* Wide levels on a bracketed plan (strategy 3): on (the default; an experiment build's
 * OMF_SPEC_WIDE=0 turns it off for new plans) the fp32 encodes at bit_width 5-8 (int8 at 5-6, the int32 wire at 7-8) take the
 * bracketed encoder with a 32-quad undecided list per wave; off, they take the ring (7-8) or the
 * two-pass encoder (5-6).  Identical payloads either way. */
int omf_plan_set_wide_levels(omf_plan* plan, int32_t on);
/* The bracketed encoder's bracket folded into its pass (on: the pass's first workgroups sample the
 * tensors and publish the brackets, the pass's blocks poll for theirs after issuing their loads — the
 * default; off: a launch of its own before the pass; an experiment build's OMF_SPEC_FB=0 turns it off for new
 * plans).  fp32 encodes
 * without a fused last client: bit_width 1-4, and 5-8 when wide levels are on (one-wave workgroups); identical
 * payloads either way. */
int omf_plan_set_fused_bracket(omf_plan* plan, int32_t on);
/* Diagnostics of the last bracketed single-read encode (strategy 3; synchronises `stream`,
 * not for the hot path): out[0] tensors requantised whole (norm outside the sampled bracket,
 * a wave's undecided-quad slot overflowed, or a degenerate sample), out[1] of those the
 * deferred ones (degenerate sample), out[2] undecided quads fixed from the slots, out[3]
 * wave slots filled to capacity. */
int omf_plan_spec_stats(omf_plan* plan, void* stream, int64_t* out4);
/* Test / experiment hook of the plan's Top-K encoder (never needed in production; an experiment
 * build also reads them from the OMF_TOPK_* environment, once, at the plan's first Top-K call).  Every
 * setting changes only how the exact selection is found, never what it is: groups (>= 1) = the
 * two-stream group pipeline, force_fallback (0 / 1) = always the exact tail's device-wide radix sort
 * (2: the same, with one tail workgroup skipping its first barrier arrival — the test of the bound's
 * expiry: the call's selection is invalid and omf_plan_check reports OMF_ETIMEOUT),
 * sample_runs (0 = default, or 64..2^20) = sampled runs per tensor, sure_z / sure_c = the sure
 * bin's margin.  A negative argument keeps the current setting. */
int omf_plan_set_topk(omf_plan* plan, int32_t groups, int32_t force_fallback, int64_t sample_runs, float sure_z,
                      float sure_c);

#ifdef __cplusplus
}
#endif

#endif /* OMF_CODEC_EXPERIMENTAL_H */
