/*
 * omf_codec.h — C ABI of the MI355X-native OmniFed gradient-compression codec.
 *
 * Drop-in boundary for the hybrid engine's global gRPC hop.  The reference is
 * pure Python/PyTorch (no native code, no FFI): its codec entry points are the
 * Python functions cited on each declaration below
 * (paths relative to at-aaims/OmniFed).  The Python host layer
 * `omnifed_amd.hybrid.compression` / `omnifed_amd.hybrid.communicator.
 * global_grpc_compression` keeps those names and signatures and binds this ABI
 * with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every pointer argument is DEVICE memory owned by the caller unless noted.
 *    The library allocates only in omf_plan_create (its own workspace) and, once per
 *    (plan, Top-K ratio), a small constant table on the first Top-K call at that ratio
 *    (synchronous, not on the hot path after that).  The hot-path calls never allocate or
 *    copy host memory, and never synchronise — except omf_topk_torch_order (host work on
 *    the tied tensors) and omf_plan_check / omf_plan_spec_stats / omf_topk_stats, which exist
 *    to synchronise.  Since ABI 1.11 omf_topk_encode is stream-asynchronous too (its fallback
 *    is decided and run on the device) and may be captured into a HIP graph after its first
 *    call at a ratio.
 *  - `stream` is a hipStream_t (NULL = the legacy default stream).  Calls are
 *    asynchronous on that stream; results are ready when the stream is.
 *  - Return value: 0 (OMF_OK) or a negative OMF_E* code; the message for the
 *    calling thread is in omf_last_error().  No C++ exception crosses the ABI.
 *  - Reentrant: no global mutable state.  A plan is driven by one host thread at
 *    a time; its stateful launches (QSGD encode, norms, fused PS step, Top-K
 *    duplicate check) may go to any stream: a launch on a different stream than
 *    the plan's previous one is ordered after everything enqueued so far on
 *    that previous stream (an event recorded there at the switch,
 *    hipStreamWaitEvent), never run concurrently.
 *    The previous stream must therefore still exist when the plan moves to
 *    another stream (PyTorch's pooled streams always do): before destroying the
 *    stream of a plan's last stateful launch, call omf_plan_check on it (which
 *    synchronises it and drops the plan's reference to it).
 *
 * Data layout ("update arena"): the named tensors of one client, flattened in
 * named_parameters() order into one fp32 buffer, tensor t occupying elements
 * [offsets[t], offsets[t] + sizes[t]).  offsets[t] must be a multiple of 4
 * (16-byte aligned starts; gaps between tensors are padding that is never
 * read as data).  Payload arenas (int8 / int32 QSGD levels, fp32 decoded
 * values) use the SAME element offsets.  Base pointers: fp32 and int32 buffers
 * 16-byte aligned, int8 buffers 4-byte aligned.  An int8 payload is written in
 * whole dwords: the bytes from the end of a tensor up to the next multiple of 4
 * (padding, inside the next tensor's aligned start) may be written as zero, so an
 * int8 payload buffer must hold round_up(arena_end, 4) elements.
 */
#ifndef OMF_CODEC_H
#define OMF_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMF_OK 0
#define OMF_EINVAL (-1)   /* bad argument (maps to Python ValueError) */
#define OMF_EHIP (-2)     /* HIP runtime error */
#define OMF_ETIMEOUT (-3) /* an in-kernel wait hit its bound (reported by omf_plan_check) */
#define OMF_ENOMEM (-4)

typedef struct omf_plan omf_plan;

/* ABI version (major*100 + minor). */
#define OMF_ABI_VERSION 112
int omf_abi_version(void);

/* Last error message of the calling thread ("" if none). */
const char* omf_last_error(void);

/*
 * Plan over a fixed list of named tensors (one client's update dict).
 * sizes/offsets are HOST arrays of ntensors elements; chunk_elems is the work unit of
 * one workgroup in the two-pass encoder (0 = default 32768; a multiple of 16384).
 * Decode and the other passes use 16384-element items; tensors of <= 8192 elements
 * (the encoder's rows x 1024) are encoded by one workgroup each (norm and levels from
 * registers).
 * Replaces the per-call Python loop of encode_updates_dict /
 * decode_updates_dict (src/omnifed/hybrid/communicator/global_grpc_compression.py:207-223).
 */
int omf_plan_create(const int64_t* sizes, const int64_t* offsets, int32_t ntensors,
                    int64_t chunk_elems, int device, omf_plan** out);
int omf_plan_destroy(omf_plan* plan);
/* Number of workgroups one encode launch uses (diagnostics / roofline bookkeeping). */
int64_t omf_plan_encode_items(const omf_plan* plan);
/* Synchronise `stream` and report what the plan's launches since the previous check hit:
 * OMF_ETIMEOUT when an on-chip wait exceeded its bound (a ring encoder hand-off: that
 * workgroup aborted and drained; a bracketed-encoder fix thread waiting for its tensor's norm:
 * the quad kept its guess) — the payload of that launch is invalid; 1 (results still exact)
 * when an encoder recomputed a norm after a bounded wait; 0 otherwise.  Clears what it
 * reports.  The Python layer calls it at the synchronisation each product path already makes
 * (the norms' device-to-host copy) and raises RuntimeError on OMF_ETIMEOUT, so the PS turns
 * it into UpdateResponse(success=False) like any codec exception
 * (src/omnifed/hybrid/communicator/global_grpc_server.py:138-145).  Every bound needs both
 * its wall-clock time (20 ms) and a minimum number of polls, so a queue context switch does
 * not fake an expiry. */
int omf_plan_check(omf_plan* plan, void* stream);
/* Encoder strategy: 0 = register-resident items for tensors of at most
 * omf_plan_resident_capacity() items (x read once; the workgroup holds its 16 Ki elements
 * while the tensor norm is published) and two-pass items for larger tensors;
 * 1 = two-pass for every tensor (x re-read after the norm);
 * 2 = single-read "ring" encoder: persistent workgroups keep each chunk in an LDS ring
 * until its tensor's norm is complete; tensors larger than the ring's
 * hold limit take a second read;
 * 3 = bracketed single-read encoder (fp32 values, on-device draws; otherwise as 1): a sampled
 * bracket of each tensor's norm, one pass that reads x once and writes every level that is
 * the same for every norm in the bracket, a fold of the exact norm, and a fix pass for the
 * few undecided quads.  Identical payloads given the norm; the norms fold
 * partials over different chunk sizes, so strategies agree to rounding. */
int omf_plan_set_encode_strategy(omf_plan* plan, int32_t strategy);
/* The plan's encode strategy (0-3 as above).  A new plan picks 3 (bracketed single-read) for
 * arenas of >= 2^25 elements and 2 (the ring) below: the measured crossover;
 * omf_plan_set_encode_strategy overrides.  Strategy 3 serves fp32 / bf16 / fp16 values with on-device
 * draws at bit_width 1-4 and fp32 values at 5-8 (omf_plan_set_wide_levels); its other int32-wire
 * encodes take the ring (2), the rest (caller uniforms, half values at s = 5, 6) the two-pass
 * encoder (1). */
int32_t omf_plan_encode_strategy(const omf_plan* plan);
/* The encoder the plan's latest encode (or fused PS step) launched: 0 register-resident +
 * two-pass, 1 two-pass, 2 ring, 3 bracketed, 4 grid, 5 levels with caller norms (norm_in);
 * -1 before the first.  Lets a test assert which path a configuration takes (e.g. the int32
 * wire of a bracketed plan: the ring). */
int32_t omf_plan_last_encoder(const omf_plan* plan);

/*
 * QSGD encode, all tensors of the plan in ONE launch.
 * Replaces QSGDQuantCompression.quantize_vector / compress
 * (src/omnifed/hybrid/compression/qsgd.py:36-82) as called per tensor by
 * _encode_qsgd_layer (global_grpc_compression.py:101-123), with the client
 * weighting of GrpcCommunicator.aggregate (global_grpc.py:101-123) fused in:
 *   xs = fl32(x * alpha)                      (alpha = 1.0f: identity)
 *   norm[t] = fp32 L2 norm of xs over tensor t  (or norm_in[t] if norm_in != NULL)
 *   q_i = sign(xs_i/norm) * clamp(floor(|xs_i/norm|*L) + (u_i < frac), 0, L),  L = 2^bit_width
 * bit_width in [0, 30]; payload element = int8 if L <= 127 else int32 (qsgd.py:18-21).
 * u: NULL = on-device Philox4x32-10 uniforms from (seed, offset) — see
 * oracle/philox.py for the exact counter layout; non-NULL = caller-supplied
 * fp32 uniforms in the arena layout (parity mode, e.g. the MT19937 stream of
 * torch.rand_like).  A zero norm yields an all-zero payload (the Python layer
 * then emits the reference's dense passthrough LayerState).
 * norm_out (ntensors fp32) receives the norm used for every tensor.
 */
int omf_qsgd_encode(omf_plan* plan, const float* x, float alpha, int32_t bit_width,
                    const float* u, uint64_t seed, uint64_t offset, const float* norm_in,
                    void* q_out, float* norm_out, void* stream);

/* Only the per-tensor norms of xs = fl32(x*alpha) (parity-mode helper: lets the host
 * know which tensors consume MT19937 draws before it builds u). */
int omf_qsgd_norms(omf_plan* plan, const float* x, float alpha, float* norm_out, void* stream);

/*
 * omf_qsgd_encode / omf_qsgd_norms for tensors whose dtype is bf16 or fp16.  The reference
 * quantises in the tensor's own dtype (qsgd.py:46-58 on a bf16/fp16 tensor; the weighting
 * torch.mul(param, batch_samples) of global_grpc.py:104/121 too).  x still holds fp32 (the
 * exact upcast of the tensor); value_format 0 = fp32 (= omf_qsgd_encode), 1 = bf16,
 * 2 = fp16, and the encoder rounds (to nearest even) where torch's CPU ops round:
 *   xs   = round(fl32(x * alpha))                (exact when alpha = 1)
 *   norm = round(fp32 L2 norm of xs)             (norm_out receives it; the wire's float32)
 *   vn   = round(fl32(xs / norm))
 * and an fp16 |vn| * L of 65520 or more (inf in fp16) gives level 0, as the reference's
 * int64 conversion of inf does.  The rest of the chain is exact in fp32.
 */
int omf_qsgd_encode_ex(omf_plan* plan, const float* x, float alpha, int32_t bit_width, int32_t value_format,
                       const float* u, uint64_t seed, uint64_t offset, const float* norm_in, void* q_out,
                       float* norm_out, void* stream);
int omf_qsgd_norms_ex(omf_plan* plan, const float* x, float alpha, int32_t value_format, float* norm_out,
                      void* stream);

/*
 * Fused PS step: avg_out = acc / divisor (IEEE fp32 division, as the reference's
 * `acc / total_samples` in CentralServerServicer._apply_model_updates,
 * src/omnifed/hybrid/communicator/global_grpc_server.py:155-171) and the QSGD encode of avg
 * for the downlink (_send_current_model, :213-234 -> encode_layer_state), acc read once:
 * the bracketed encoder's pass divides, stores the average and quantises it (strategy 3 at
 * bit_width 1-4; its rare whole-tensor requantisation reads the average back), or one ring
 * launch (other plans; tensors larger than the on-chip ring re-read acc); the two-pass
 * strategies run divide + encode.  Arguments after avg_out as omf_qsgd_encode (no alpha,
 * no norm_in).  avg_out must be disjoint from acc for the one-launch paths; avg_out == acc
 * is accepted and runs as divide (in place) + encode; a partial overlap is OMF_EINVAL.
 */
int omf_ps_apply_encode(omf_plan* plan, const float* acc, float divisor, float* avg_out, int32_t bit_width,
                        const float* u, uint64_t seed, uint64_t offset, void* q_out, float* norm_out, void* stream);

/*
 * The PS round's last step in one pass: the last arriving client's decode-accumulate
 * (SendUpdate: acc[name] += update, global_grpc_server.py:108-111, 147-153), the average
 * (_apply_model_updates, :155-171) and its downlink encode (_send_current_model, :213-234):
 *   sum_i   = fl32(acc_i + fl32(fl32(norm_in[t] * q_in_i) / levels_in))   (omf_qsgd_decode's accumulate)
 *   avg_out = sum / divisor,  q_out / norm_out = the QSGD encode of avg_out (as omf_ps_apply_encode)
 * acc_out: where sum is stored (acc itself, a disjoint arena, or NULL: not stored — the caller
 * no longer needs the accumulator).  q_in: the last client's payload arena (width_in 8 or 32,
 * LayerState.width; levels_in = LayerState.level), norm_in its per-tensor norms (0 for a tensor
 * absent from its message).  avg_out disjoint from acc and acc_out.  Bracketed plans (bit_width
 * 1-4, on-device draws) read acc and q_in once in the encoder's pass (10 B per element at s = 4
 * instead of 18 for decode-accumulate then omf_ps_apply_encode); other plans run those two.
 * Bytes equal to omf_qsgd_decode(accumulate=1) followed by omf_ps_apply_encode.
 */
int omf_ps_accumulate_apply_encode(omf_plan* plan, const float* acc, const void* q_in, int32_t width_in,
                                   int32_t levels_in, const float* norm_in, float* acc_out, float divisor,
                                   float* avg_out, int32_t bit_width, const float* u, uint64_t seed, uint64_t offset,
                                   void* q_out, float* norm_out, void* stream);

/*
 * QSGD decode, all tensors in one launch.
 * Replaces QSGDQuantCompression.decompress_quantized (qsgd.py:84-96) as called by
 * _decode_qsgd_layer (global_grpc_compression.py:163-182), and — with
 * accumulate != 0 — the PS accumulate step acc[name] += update
 * (src/omnifed/hybrid/communicator/global_grpc_server.py:147-153):
 *   y_i = fl32(fl32(norm[t] * q_i) / fl32(levels));   accumulate: y_out_i = fl32(y_out_i + y_i)
 * width: 8 (int8 payload) or 32 (int32), the LayerState.width field; levels > 0 is
 * LayerState.level (any positive value; powers of two take an exact multiply path).
 */
int omf_qsgd_decode(omf_plan* plan, const void* q, int32_t width, int32_t levels, const float* norm,
                    float* y_out, int32_t accumulate, void* stream);
/* omf_qsgd_decode over the arena's 4096-element decode blocks that overlap [elem_begin,
 * elem_end) only (every element of those blocks is written, so the payload of those whole blocks
 * must be in place).  Lets a caller decode an arena chunk by chunk as its payload arrives and
 * copy each decoded chunk out while the next is staged (the CPU placement of
 * decode_updates_dict, global_grpc_compression.py:214-223).  Same results as one full decode. */
int omf_qsgd_decode_range(omf_plan* plan, const void* q, int32_t width, int32_t levels, const float* norm,
                          float* y_out, int32_t accumulate, int64_t elem_begin, int64_t elem_end, void* stream);

/*
 * y_i = fl32(y_i / divisor) over n elements (PS averaging,
 * CentralServerServicer._apply_model_updates, global_grpc_server.py:155-171).
 */
int omf_div_f32(float* y, int64_t n, float divisor, void* stream);

/*
 * Opt-in bit-packed QSGD wire (NOT reference-compatible, a new
 * compression_type "QSGDBitPackedCompression" that replaces the int8/int32 values_data
 * of _encode_qsgd_layer, global_grpc_compression.py:111-123, only when enabled).
 * Level q in [-L, L] -> code q + L in b = omf_qsgd_packed_bits(L) = ceil(log2(2L+1))
 * bits, LSB-first: element i of a tensor at bits [i*b, (i+1)*b) of its stream; tensor t's
 * stream starts at 32-bit word offsets[t] * b / 32 of the packed arena, ceil(arena_end / 32) * b
 * words (32 elements = b words, the last partial group of a tensor included, its padding
 * packed as code 0; groups of arena padding are neither written nor decoded).  Both calls
 * need every tensor offset to be a multiple of 32 elements (OMF_EINVAL otherwise; the
 * Python arena_layout's are multiples of 64).
 * omf_qsgd_pack: payload (width 8 or 32, as omf_qsgd_encode wrote it) -> packed arena (8-byte
 * aligned: even widths are stored as 8-byte word pairs; omf_qsgd_decode_packed needs 4).
 * omf_qsgd_decode_packed: y = fl32(fl32(norm * (code - L)) / L), bit-identical to
 * omf_qsgd_decode of the unpacked payload (accumulate: y += that).
 */
int32_t omf_qsgd_packed_bits(int32_t levels);
int omf_qsgd_pack(omf_plan* plan, const void* q, int32_t width, int32_t levels, uint32_t* packed, void* stream);
int omf_qsgd_decode_packed(omf_plan* plan, const uint32_t* packed, int32_t levels, const float* norm, float* y,
                           int32_t accumulate, void* stream);

/*
 * Top-K sparsification with error feedback, all tensors of the plan in one call.
 * Replaces TopKCompression.compress (src/omnifed/hybrid/compression/topk.py:33-42)
 * with ResidualUpdates.compensate/update (src/omnifed/hybrid/compression/core.py:26-37)
 * and topk_sparse (topk.py:10-15):
 *   a = fl32(alpha * x): the client weighting param * batch_samples
 *       (global_grpc.py:101-123) fused in; alpha = 1 leaves x's bits unchanged.
 *   residual_mode 0: t' = a                       (no error-feedback state)
 *   residual_mode 1: t' = residual + a, then residual := t' - desparse(selection)
 *   residual_mode 2: t' = a,            then residual := t' - desparse(selection)
 *                    (first call for a name: the reference has no residual yet)
 *   k_t = max(1, int(n_t * ratio))  (omf_topk_k); the k_t largest |t'| of tensor t;
 *   values (fp32 t') / indices (tensor-local int64) of tensor t are written at
 *   [K_t, K_t + k_t) with K_t = sum_{u<t} k_u (packed in plan order).
 * Order within a tensor: descending |t'|, ties by ascending index (torch.topk's
 * order for k*64 <= n on the reference CPU path; ties there are unspecified).
 * ws: caller workspace of omf_topk_workspace_bytes(plan, ratio) bytes.
 * Stream-asynchronous: the plan kernel's verdict is read by the launches queued behind it (the
 * bucket kernels, the zero fill and the exact tail, each leaving at once when the verdict does
 * not need it); the rare fallback (a sampled threshold too high, or an over-full fine bin) runs
 * on the device in the exact tail — a grid-barrier kernel, one workgroup per CU, sized by the
 * device's own candidate count.  A tail barrier that exceeded its bound (never expected) is
 * reported by omf_plan_check as OMF_ETIMEOUT.  The first call at a ratio builds the plan's
 * constant tables synchronously (not capturable); later calls launch only.
 */
int64_t omf_topk_k(int64_t numel, double ratio);
/* The plan's Top-K encoder counters (diagnostics; waits for the device, hipDeviceSynchronize,
 * since the device counts the path each call took): out6[0] calls of the sampled path, [1] of
 * those that took the bucket-sort fast path, [2] of those that completed a tensor with its
 * lowest-index exact zeros (zero mode: fewer than k non-zero t', e.g. the PS re-encoding an
 * average of sparse Top-K updates), [3] calls that took the exact tail's fallback (device-wide
 * radix sort), [4] of those that redid a tensor exactly, [5] calls of the exact path (plans of
 * > 256 tensors or a tensor over 2^25 elements).  reset != 0 zeroes them after reading. */
int omf_topk_stats(omf_plan* plan, int64_t* out6, int32_t reset);
size_t omf_topk_workspace_bytes(const omf_plan* plan, double ratio);
int omf_topk_encode(omf_plan* plan, const float* x, float* residual, int32_t residual_mode, double ratio,
                    float alpha, float* values, int64_t* indices, void* ws, size_t ws_bytes, void* stream);
/*
 * The reference's own selection where magnitudes tie.  The reference selects with
 * torch.topk(|t'|, k, sorted=False) on the CPU (topk.py:13; its compressor is always built on
 * "cpu": grpc_leader_comm.py:59).  torch's CPU kernel (ATen TopKImpl.h) runs libstdc++'s
 * partial_sort (heap select + heap sort) when k*64 <= n and nth_element otherwise, so among equal
 * magnitudes both WHICH are selected at rank k and their ORDER in the selection are that
 * algorithm's, not omf_topk_encode's (|t'| descending, index ascending).
 * omf_topk_torch_order rewrites a finished omf_topk_encode (same plan, x, residual,
 * residual_mode, ratio, alpha, values, indices and ws) into torch's bytes: a census on the device
 * flags each tensor whose selection may differ (two selected values with one magnitude, an
 * unselected element with the k-th magnitude, or the nth_element regime with k > 1; NaNs are one
 * magnitude); for those, t' is fetched, torch's selection recomputed on the host (threads over
 * tensors, omf_topk_select_host's algorithm) and values / indices — and the residual, when the
 * selected SET changed (t' - t' on the new selection, t' back on the old) — written back.
 * Synchronises `stream` (not stream-asynchronous: the host work is the point).
 * *n_reordered (HOST, may be NULL) receives the number of tensors rewritten.
 */
int omf_topk_torch_order(omf_plan* plan, const float* x, float* residual, int32_t residual_mode, double ratio,
                         float alpha, float* values, int64_t* indices, void* ws, size_t ws_bytes, void* stream,
                         int64_t* n_reordered);
/*
 * HOST-only (no device, no plan): indices[0, k) = torch.topk(|t|, k, sorted=False).indices of the
 * HOST array t[0, n) as the reference's CPU torch computes it (1 <= k <= n < 2^32), order included.
 */
int omf_topk_select_host(const float* t, int64_t n, int64_t k, int64_t* indices);

/*
 * Top-K decode of ONE tensor of n elements: topk_desparse (topk.py:18-21),
 * _decode_topk_layer (global_grpc_compression.py:140-160) and the sparse
 * scatter-add of layerwise_decompress (core.py:62-71):
 *   mode 0: y := 0, then y[idx_j] = val_j       (PS uplink decode)
 *   mode 1: y[idx_j] = val_j, y holds the base  (client overlay decode)
 *   mode 2: y[idx_j] += val_j                   (scatter-add; indices unique per call)
 * Indices outside [0, n) are skipped.
 */
int omf_topk_decode(const float* values, const int64_t* indices, int64_t k, float* y,
                    int64_t n, int32_t mode, void* stream);

/*
 * Top-K decode of ONE client's whole selection (omf_topk_encode's packed layout for the
 * plan's tensors at `ratio`) into an arena y, one launch: the per-layer _decode_topk_layer
 * loop of decode_updates_dict (global_grpc_compression.py:140-160, 214-223) and, with
 * mode 2, one client's term of layerwise_decompress's scatter-add (core.py:62-71) as
 * torch_mpi.sparse_aggregate applies it to every parameter (torch_mpi.py:302-359).
 * mode 0: y := 0 then set; 1: set over y (overlay); 2: y += v.  Index -1 (padding) and
 * indices outside a tensor are skipped.  Plans of at most 4096 tensors.
 */
int omf_topk_decode_arena(omf_plan* plan, double ratio, const float* values, const int64_t* indices, float* y,
                          int32_t mode, void* stream);
/* omf_topk_decode_arena with a caller workspace of omf_topk_decode_workspace_bytes(plan, ratio)
 * bytes (256-byte aligned): mode 0 then writes the arena in ONE streaming pass — the values are
 * placed into per-super-tile buckets (64 Ki arena elements; capacity twice the expected count +
 * 256, an overflow list past it) and each 8 Ki-element sub-tile is built in LDS (zeros + its
 * values) and stored whole — instead of a fill followed by scattered 4-byte stores (which reach
 * HBM as partial-line read-modify-writes).  Same bytes as omf_topk_decode_arena (indices unique
 * per tensor; the reference's zeros().scatter_ leaves a duplicate's last value, which neither
 * decoder promises).  The first call of a plan at a ratio uploads the plan's bucket tables
 * (synchronous, once).  Modes 1/2 and arenas over 2^30 elements ignore the workspace.
 * The workspace must be zero-filled before its first use (its bucket counters); every call
 * leaves them zero again, so it needs no clearing between calls (a workspace used by one call
 * at a time: one per stream). */
size_t omf_topk_decode_workspace_bytes(const omf_plan* plan, double ratio);
int omf_topk_decode_arena_ws(omf_plan* plan, double ratio, const float* values, const int64_t* indices, float* y,
                             int32_t mode, void* ws, size_t ws_bytes, void* stream);

/*
 * The whole-arena decode of ONE received message, whose per-tensor selection sizes are whatever
 * its layers carry (k_t = len(values_data) / 4) rather than a ratio's: the per-layer
 * _decode_topk_layer loop of decode_updates_dict (global_grpc_compression.py:140-160, 214-223),
 * the PS's accumulate of a Top-K update (global_grpc_server.py:108-111, 147-153: with mode 2) and
 * the client downlink overlay (global_grpc_client.py:98-111: mode 1) in one call.
 * counts: HOST array of ntensors, 0 <= counts[t] <= sizes[t] (0: the tensor is absent from the
 * message — mode 0 leaves it zero, modes 1 / 2 untouched); values / indices packed in plan order
 * at K_t = sum_{u<t} counts[u].  Otherwise as omf_topk_decode_arena_ws (modes, workspace of
 * omf_topk_decode_counts_workspace_bytes(plan, counts) bytes for the tiled mode 0, or NULL).
 * The plan keeps the tables of the last 8 count vectors it saw (uploaded on first use).
 */
size_t omf_topk_decode_counts_workspace_bytes(const omf_plan* plan, const int64_t* counts);
int omf_topk_decode_counts(omf_plan* plan, const int64_t* counts, const float* values, const int64_t* indices,
                           float* y, int32_t mode, void* ws, size_t ws_bytes, void* stream);
/*
 * Index check of a received selection (layout as omf_topk_decode_counts), before it is decoded:
 * the reference decoder indexes with numpy (`dense[indices] = values`,
 * global_grpc_compression.py:154/158), which wraps an index in [-n_t, 0) to i + n_t — rewritten
 * here in place in the DEVICE array `indices` — and raises IndexError for one outside
 * [-n_t, n_t).  *bad (device int32) receives the lowest such tensor t, or 0x7f7f7f7f (>= ntensors)
 * when every index is in range.  Asynchronous on `stream`.
 */
int omf_topk_check_indices(omf_plan* plan, const int64_t* counts, int64_t* indices, int32_t* bad, void* stream);
/*
 * Repeated indices of the same received message (after omf_topk_check_indices has wrapped them):
 * flags[t] (DEVICE int32[ntensors], written) = 1 when an in-range index of tensor t appears more
 * than once.  The reference decodes a layer as dense[indices] = values, where numpy keeps the LAST
 * value of a repeated index (global_grpc_compression.py:140-160); the scatter decodes do not, so the
 * Python layer decodes a flagged layer by itself with that rule.  Never true for a selection an
 * encoder produced.  Uses a plan-owned bitmap of arena_end bits (made on first use), so it is one
 * of the plan's stateful launches: ordered after the previous one when the stream changes.
 * Asynchronous.
 */
int omf_topk_check_duplicates(omf_plan* plan, const int64_t* counts, const int64_t* indices, int32_t* flags,
                              void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OMF_CODEC_H */
