"""Host-inclusive wire path timing: the drop-in's user-visible API on Llama-400M.

QSGD (s = 4) and Top-K (k = 1 %, the reference's default scheme, conf/base.yaml:197):
encode_updates_dict : device gradients -> one encode call -> chunked pinned D2H of the payload
                      buffer -> bytes filled by worker threads -> 183 LayerState messages
decode_updates_dict : LayerStates -> pinned staging (worker threads) -> chunked H2D -> one
                      decode call (device="cuda": stays on the GPU; default: CPU tensors)
decode_updates_into : client downlink straight into the model's device tensors
accumulate_layers   : the PS's SendUpdate decode-accumulate of one client (DeviceAggregator)
apply_and_encode    : the PS's GetUpdatedModel: average + re-encode + LayerStates (Top-K: the
                      sparse average of two clients' Top-K decodes, the reference's steady state;
                      the dense accumulator is timed beside it)
host round trip     : host fp32 tensors in -> LayerStates -> host fp32 tensors out (the rate
                      including the H<->D copies, north_star)

usage: python scripts/wire_bench.py [config] [out.json]
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, hostio, shapes  # noqa: E402
from omnifed_amd.hybrid.communicator.global_grpc_compression import (  # noqa: E402
    build_global_compressor, decode_updates_dict, decode_updates_into, encode_layer_state, encode_updates_dict)
from omnifed_amd.ps import DeviceAggregator  # noqa: E402

dev = torch.device("cuda", 0)
cfg = sys.argv[1] if len(sys.argv) > 1 else "llama400m"
out_path = sys.argv[2] if len(sys.argv) > 2 else None
named = shapes.model_shapes(cfg)
g = torch.Generator(device=dev).manual_seed(0)
upd = {n: torch.randn(s, device=dev, generator=g) * 1e-3 for n, s in named}
N = sum(t.numel() for t in upd.values())
targets = {n: torch.empty_like(t) for n, t in upd.items()}


def progress(msg):
    print(f"[wire {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def tm(fn, reps=7, warm=3):
    for _ in range(warm):  # steady state: the retained host memory and the copy threads warmed up
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(sorted(ts)[len(ts) // 2] * 1e3, 2)


TK_ORDER = "index"  # the Top-K legs time the device order; "topk_torch_order" below the reference's


def topk_comp(**kw):
    c = build_global_compressor(enabled=True, scheme="topk", compress_ratio=0.01, device=dev, **kw)
    c.tie_order = TK_ORDER
    return c


def leg(comp, tag):
    """The wire legs of one compressor; returns a dict of medians (ms) and rates."""
    r = {}
    st = {}
    progress(f"{tag} legs")
    layers = encode_updates_dict(upd, comp, stats=st)
    r["wire"] = st
    r["encode_updates_dict_ms"] = tm(lambda: encode_updates_dict(upd, comp))
    r["decode_updates_dict_gpu_ms"] = tm(lambda: decode_updates_dict(layers, device=dev))
    r["decode_updates_into_ms"] = tm(lambda: decode_updates_into(layers, targets))
    r["decode_updates_dict_cpu_ms"] = tm(lambda: decode_updates_dict(layers), reps=3, warm=1)  # pageable pool
    hostio.set_pinned_arenas(4 << 30)  # the opt-in page-locked result arenas (OMF_PIN_HOST_ARENAS)
    r["decode_updates_dict_cpu_pinned_ms"] = tm(lambda: decode_updates_dict(layers), reps=3, warm=1)
    hostio.set_pinned_arenas(0)
    agg = DeviceAggregator(named, device=dev)
    r["agg_accumulate_layers_ms"] = tm(lambda: agg.accumulate_layers(layers, number_samples=1))
    # GetUpdatedModel: the server's compressor re-encodes the average (apply_and_encode).  A dense
    # accumulator (QSGD decodes are dense; a Top-K average over many clients' updates):
    srv = (topk_comp() if tag == "topk" else
           build_global_compressor(enabled=True, scheme=tag, bit_width=4, compress_ratio=0.01, device=dev))
    agg.acc.copy_(torch.randn(agg.acc.numel(), device=dev, generator=g) * 4e-2)
    agg.total_samples = 40
    r["ps_apply_and_encode_dense_ms"] = tm(lambda: agg.apply_and_encode(srv, total_samples=40))
    r["ps_apply_and_encode_ms"] = r["ps_apply_and_encode_dense_ms"]
    del agg
    if tag == "topk":
        # The reference's steady state for Top-K (scheme: topk, aggregate_payload: params,
        # conf/base.yaml:194-198): the PS sums the clients' zero-filled Top-K decodes
        # (global_grpc_server.py:147-153), divides (:155-171) and re-encodes that SPARSE average per
        # request (:213-234) — at most C k non-zeros per tensor.  Two clients with error feedback on
        # (their second call's selections), overlapping (client 1 = client 0's gradient + 5 % noise)
        # and disjoint (independent gradients) selections.
        plan_t = codec.Plan.get([t.numel() for t in upd.values()], device=dev)
        for label, noise in (("overlap", 0.05), ("disjoint", None)):
            agg2 = DeviceAggregator(named, device=dev)
            for c in range(2):
                cc = topk_comp()
                if noise is None:  # disjoint: independent gradients
                    u = upd if c == 0 else {n: torch.randn(t.shape, device=dev, generator=g) * 1e-3
                                            for n, t in upd.items()}
                else:
                    u = {n: t + (noise * c) * torch.randn(t.shape, device=dev, generator=g) * 1e-3
                         for n, t in upd.items()}
                encode_updates_dict(u, cc)
                agg2.accumulate_layers(encode_updates_dict(u, cc), number_samples=1)
                del u, cc
            nnz = int((agg2.acc != 0).sum())
            srv2 = topk_comp()
            plan_t.topk_stats(reset=True)
            r[f"ps_apply_and_encode_sparse_{label}_ms"] = tm(lambda: agg2.apply_and_encode(srv2, total_samples=2))
            r[f"sparse_{label}_nnz_per_k"] = round(nnz / sum(plan_t.topk_ks(0.01)), 3)
            r[f"sparse_{label}_topk_stats"] = plan_t.topk_stats(reset=True)
            del agg2, srv2
        r["ps_apply_and_encode_ms"] = r["ps_apply_and_encode_sparse_overlap_ms"]
    # host round trip: host fp32 tensors in, LayerStates, host fp32 tensors out
    host = {n: t.cpu().pin_memory() for n, t in upd.items()}
    r["host_roundtrip_ms"] = tm(lambda: decode_updates_dict(encode_updates_dict(host, comp)), reps=3, warm=1)
    for k in ("encode_updates_dict_ms", "decode_updates_dict_gpu_ms", "decode_updates_into_ms",
              "decode_updates_dict_cpu_ms", "host_roundtrip_ms"):
        r[k.replace("_ms", "_fp32_GBs")] = round(4 * N / (r[k] * 1e-3) / 1e9, 2)
    r["device_roundtrip_ms"] = round(r["encode_updates_dict_ms"] + r["decode_updates_dict_gpu_ms"], 2)
    return r, layers


res = {"config": cfg, "elements": N, "tensors": len(named), "copy_threads": hostio.workers()}
qcomp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev)
res["qsgd_s4"], layers = leg(qcomp, "qsgd")
tcomp = topk_comp()
res["topk_1pct"], tlayers = leg(tcomp, "topk")
progress("per-layer Top-K loop, copy threads, device-side steps")
# the round-3 per-layer Top-K loop (one encode + host wait + small D2H per tensor), for comparison
tper = topk_comp()
res["topk_1pct"]["per_layer_encode_ms"] = tm(lambda: [encode_layer_state(n, t, tper) for n, t in upd.items()],
                                             reps=3, warm=1)
# an fp16 model's update (the reference's default scheme on a half-precision model): one batched
# selection launch over the dict, residuals in fp16 (round 4), against the per-layer loop
upd16 = {n: t.half() for n, t in upd.items()}
t16 = topk_comp()
res["topk_1pct"]["fp16_encode_updates_dict_ms"] = tm(lambda: encode_updates_dict(upd16, t16), reps=5, warm=2)
t16p = topk_comp()
res["topk_1pct"]["fp16_per_layer_encode_ms"] = tm(lambda: [encode_layer_state(n, t, t16p) for n, t in upd16.items()],
                                                  reps=3, warm=1)
del upd16, t16, t16p
# the drop-in's default Top-K order (tie_order="torch": the reference's bytes where magnitudes tie,
# omf_topk_torch_order's host rewrite of the tied tensors) on the client encode and the PS re-encode
progress("Top-K in torch order")
TK_ORDER = "torch"
ttc = topk_comp()
res["topk_torch_order"] = {"encode_updates_dict_ms": tm(lambda: encode_updates_dict(upd, ttc), reps=3, warm=1)}
plan_tt = codec.Plan.get([t.numel() for t in upd.values()], device=dev)
res["topk_torch_order"]["tensors_rewritten"] = plan_tt.topk_reordered
agg_t = DeviceAggregator(named, device=dev)
agg_t.accumulate_layers(encode_updates_dict(upd, topk_comp()), number_samples=1)
srv_t = topk_comp()
res["topk_torch_order"]["ps_apply_and_encode_sparse_ms"] = tm(lambda: agg_t.apply_and_encode(srv_t, total_samples=1),
                                                              reps=3, warm=1)
TK_ORDER = "index"
del ttc, agg_t, srv_t
# the host copies on the calling thread vs worker threads (hostio.set_workers), same process
res["by_copy_threads"] = {}
for nthr in (0, 2, 4, 8):
    hostio.set_workers(nthr)
    res["by_copy_threads"][str(nthr)] = {
        "qsgd_encode_updates_dict_ms": tm(lambda: encode_updates_dict(upd, qcomp)),
        "qsgd_decode_updates_dict_gpu_ms": tm(lambda: decode_updates_dict(layers, device=dev)),
        "topk_encode_updates_dict_ms": tm(lambda: encode_updates_dict(upd, tcomp)),
        "topk_decode_updates_dict_gpu_ms": tm(lambda: decode_updates_dict(tlayers, device=dev))}
hostio.set_workers(None)

# fused PS step (omf_ps_apply_encode) vs divide + encode, device-resident
plan = codec.Plan.get([t.numel() for t in upd.values()], device=dev)
acc = torch.randn(plan.arena_end, device=dev, generator=g)
avg = torch.empty_like(acc)
q = torch.empty(plan.arena_end, dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)


def separate():
    avg.copy_(acc)
    codec.div_(avg, 40.0)
    plan.qsgd_encode(avg, 4, q_out=q, norm_out=nr, seed=1)


res["ps_fused_apply_encode_ms"] = round(tm(lambda: plan.ps_apply_encode(acc, 40.0, 4, avg_out=avg, q_out=q,
                                                                         norm_out=nr, seed=1), reps=10), 4)
res["ps_divide_then_encode_ms"] = round(tm(separate, reps=10), 4)
# the last client's SendUpdate + the first GetUpdatedModel (global_grpc_server.py:108-125, 147-171,
# 213-234): its decode-accumulate fused into the PS step (omf_ps_accumulate_apply_encode) against
# decode-accumulate then the fused PS step; device-resident, then through the drop-in's messages
q_last, n_last = plan.qsgd_encode(torch.randn(plan.arena_end, device=dev, generator=g), 4, seed=2)
acc_keep = acc.clone()


def last_two_calls():
    acc_keep.copy_(acc)
    plan.qsgd_decode(q_last, 8, 16, n_last, y_out=acc_keep, accumulate=True)
    plan.ps_apply_encode(acc_keep, 40.0, 4, avg_out=avg, q_out=q, norm_out=nr, seed=1)


def last_fused():
    plan.ps_accumulate_apply_encode(acc, q_last, 8, 16, n_last, 40.0, 4, avg_out=avg, q_out=q, norm_out=nr, seed=1)


res["ps_last_client_fused_ms"] = round(tm(last_fused, reps=10), 4)
res["ps_last_client_two_calls_ms"] = round(tm(last_two_calls, reps=10) - tm(lambda: acc_keep.copy_(acc), reps=10), 4)
del acc_keep
agg_f = DeviceAggregator(named, device=dev)
agg_s = DeviceAggregator(named, device=dev)
srv_f = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev)
srv_s = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev)
res["ps_last_update_and_get_model_fused_ms"] = tm(lambda: agg_f.accumulate_apply_encode(layers, 1, srv_f), reps=5)
res["ps_last_update_and_get_model_two_calls_ms"] = tm(
    lambda: (agg_s.accumulate_layers(layers, 1), agg_s.apply_and_encode(srv_s)), reps=5)
del agg_f, agg_s
# opt-in bit-packed wire (s = 4: 6 bits per element instead of 8)
pcomp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev, packed_wire=True)
players = encode_updates_dict(upd, pcomp)
res["packed_encode_updates_dict_ms"] = tm(lambda: encode_updates_dict(upd, pcomp))
res["packed_decode_updates_dict_gpu_ms"] = tm(lambda: decode_updates_dict(players, device=dev))
res["packed_wire_bytes"] = sum(len(L.values_data) for L in players)
res["int8_wire_bytes"] = sum(len(L.values_data) for L in layers)
qq, nn = plan.qsgd_encode(acc, 4, seed=1)
pk = plan.qsgd_pack(qq, 8, 16)
res["device_pack_ms"] = round(tm(lambda: plan.qsgd_pack(qq, 8, 16, packed_out=pk), reps=10), 4)
res["device_decode_packed_ms"] = round(tm(lambda: plan.qsgd_decode_packed(pk, 16, nn, y_out=avg), reps=10), 4)
res["device_decode_int8_ms"] = round(tm(lambda: plan.qsgd_decode(qq, 8, 16, nn, y_out=avg), reps=10), 4)
line = json.dumps(res)
print(line, flush=True)
if out_path:
    with open(out_path, "w") as f:
        f.write(json.dumps(res, indent=1) + "\n")
