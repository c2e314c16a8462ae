"""Host-inclusive wire path timing: the drop-in's user-visible API on Llama-400M.

encode_updates_dict : device gradients -> one encode launch -> chunked pinned D2H of the
                      int8 payload arena -> bytes filled by worker threads -> 183 LayerState
                      messages (omnifed_amd.hostio)
decode_updates_dict : LayerStates -> pinned staging (worker threads) -> chunked H2D -> one
                      decode launch (device="cuda": stays on the GPU; default: CPU tensors)
decode_updates_into : client downlink straight into the model's device tensors
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from omnifed_amd import shapes  # noqa: E402
from omnifed_amd.hybrid.communicator.global_grpc_compression import (  # noqa: E402
    build_global_compressor, decode_updates_dict, decode_updates_into, encode_updates_dict)

dev = torch.device("cuda", 0)
cfg = sys.argv[1] if len(sys.argv) > 1 else "llama400m"
named = shapes.model_shapes(cfg)
g = torch.Generator(device=dev).manual_seed(0)
upd = {n: torch.randn(s, device=dev, generator=g) * 1e-3 for n, s in named}
N = sum(t.numel() for t in upd.values())
comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev)
targets = {n: torch.empty_like(t) for n, t in upd.items()}


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
    return sorted(ts)[len(ts) // 2]


stats = {}
layers = encode_updates_dict(upd, comp, stats=stats)
from omnifed_amd import hostio  # noqa: E402
res = {"config": cfg, "elements": N, "tensors": len(named), "wire": stats, "copy_threads": hostio.workers(),
       "agg_accumulate_layers_ms": None, "by_copy_threads": {},
       "encode_updates_dict_ms": tm(lambda: encode_updates_dict(upd, comp)) * 1e3,
       "decode_updates_dict_gpu_ms": tm(lambda: decode_updates_dict(layers, device=dev)) * 1e3,
       "decode_updates_into_ms": tm(lambda: decode_updates_into(layers, targets)) * 1e3,
       "decode_updates_dict_cpu_ms": tm(lambda: decode_updates_dict(layers)) * 1e3}
# the host copies on the calling thread vs worker threads (hostio.set_workers), same process
for nthr in (0, 2, 4, 8):
    hostio.set_workers(nthr)
    res["by_copy_threads"][str(nthr)] = {
        "encode_updates_dict_ms": round(tm(lambda: encode_updates_dict(upd, comp)) * 1e3, 2),
        "decode_updates_dict_gpu_ms": round(tm(lambda: decode_updates_dict(layers, device=dev)) * 1e3, 2)}
hostio.set_workers(None)
# the PS uplink: one client's LayerStates decode-accumulated into the aggregator arena
from omnifed_amd import codec  # noqa: E402
from omnifed_amd.ps import DeviceAggregator  # noqa: E402

agg = DeviceAggregator(named, device=dev)
res["agg_accumulate_layers_ms"] = round(tm(lambda: agg.accumulate_layers(layers, number_samples=1)) * 1e3, 2)
del agg
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


res["ps_fused_apply_encode_ms"] = tm(lambda: plan.ps_apply_encode(acc, 40.0, 4, avg_out=avg, q_out=q, norm_out=nr,
                                                                   seed=1), reps=10) * 1e3
res["ps_divide_then_encode_ms"] = tm(separate, reps=10) * 1e3
res["ps_fused_apply_encode_ms"] = round(res["ps_fused_apply_encode_ms"], 4)
res["ps_divide_then_encode_ms"] = round(res["ps_divide_then_encode_ms"], 4)
# opt-in bit-packed wire (s = 4: 6 bits per element instead of 8)
pcomp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev, packed_wire=True)
players = encode_updates_dict(upd, pcomp)
res["packed_encode_updates_dict_ms"] = round(tm(lambda: encode_updates_dict(upd, pcomp)) * 1e3, 2)
res["packed_decode_updates_dict_gpu_ms"] = round(tm(lambda: decode_updates_dict(players, device=dev)) * 1e3, 2)
res["packed_wire_bytes"] = sum(len(L.values_data) for L in players)
res["int8_wire_bytes"] = sum(len(L.values_data) for L in layers)
qq, nn = plan.qsgd_encode(acc, 4, seed=1)
pk = plan.qsgd_pack(qq, 8, 16)
res["device_pack_ms"] = round(tm(lambda: plan.qsgd_pack(qq, 8, 16, packed_out=pk), reps=10) * 1e3, 4)
res["device_decode_packed_ms"] = round(tm(lambda: plan.qsgd_decode_packed(pk, 16, nn, y_out=avg), reps=10) * 1e3, 4)
res["device_decode_int8_ms"] = round(tm(lambda: plan.qsgd_decode(qq, 8, 16, nn, y_out=avg), reps=10) * 1e3, 4)
for k in ("encode_updates_dict_ms", "decode_updates_dict_gpu_ms", "decode_updates_into_ms",
          "decode_updates_dict_cpu_ms"):
    res[k.replace("_ms", "_fp32_GBs")] = round(4 * N / (res[k] * 1e-3) / 1e9, 2)
    res[k] = round(res[k], 2)
print(json.dumps(res), flush=True)
