"""Where the host-inclusive wire path's time goes (Llama-400M, s = 4, int8 payload): each stage of
encode_updates_dict / decode_updates_dict timed alone, median of 5 (experiment harness)."""
import json
import os
import sys
import time

os.environ["OMF_RETAIN_HOST_MEMORY"] = "0"  # glibc defaults first; retained explicitly at the end

import numpy as np
import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, hostio, shapes  # noqa: E402
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb  # noqa: E402
from omnifed_amd.hybrid.communicator.global_grpc_compression import (  # noqa: E402
    build_global_compressor, decode_updates_dict, encode_updates_dict, qsgd_layer_from_payload)

dev = torch.device("cuda", 0)
named = shapes.model_shapes(sys.argv[1] if len(sys.argv) > 1 else "llama400m")
sizes = [shapes.numel(s) for _, s in named]
plan = codec.Plan.get(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3
upd = {n: x[o:o + k].view(s) for (n, s), o, k in zip(named, plan.offsets, sizes)}
comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev)
q, norms = plan.qsgd_encode(x, 4, seed=1)
spans = [(o, k) for o, k in zip(plan.offsets, sizes)]
staged = hostio.STAGING.get("probe", q.numel())


def tm(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(sorted(ts)[len(ts) // 2] * 1e3, 2)


res = {"elements": sum(sizes), "copy_threads": hostio.workers()}
res["encode_kernel_ms"] = tm(lambda: plan.qsgd_encode(x, 4, q_out=q, norm_out=norms, seed=1))
res["d2h_payload_pinned_ms"] = tm(lambda: staged.copy_(q.view(torch.uint8)[:staged.numel()], non_blocking=True))
res["device_to_bytes_only_ms"] = tm(lambda: [None for _ in hostio.device_to_bytes(q, spans, key="probe2")])
payloads = [bytes(k) for k in sizes]  # host bytes of the right sizes (contents irrelevant here)
res["layerstate_build_only_ms"] = tm(lambda: [qsgd_layer_from_payload(n, s, p, 1.0, 8, 16)
                                              for (n, s), p in zip(named, payloads)])


def assign_only():
    for p in payloads:
        L = pb.layer_state(layer_name="x")
        L.values_data = p


res["values_data_assign_only_ms"] = tm(assign_only)
res["encode_updates_dict_ms"] = tm(lambda: encode_updates_dict(upd, comp))
layers = encode_updates_dict(upd, comp)
res["values_data_get_only_ms"] = tm(lambda: [L.values_data for L in layers])
dst = torch.empty(plan.arena_end, dtype=torch.int8, device=dev)
items = [(o, (lambda L=L: L.values_data)) for L, o in zip(layers, plan.offsets)]
res["stage_payloads_only_ms"] = tm(lambda: hostio.stage_payloads(items, staged.data_ptr(), staged.numel(),
                                                                 lambda a, b: None))
res["bytes_to_device_ms"] = tm(lambda: hostio.bytes_to_device(items, dst, plan.arena_end, key="probe3"))
res["decode_updates_dict_gpu_ms"] = tm(lambda: decode_updates_dict(layers, device=dev))
# the same with the process's freed memory retained (hostio.retain_host_memory, opt-in)
res["retain_host_memory"] = hostio.retain_host_memory()
res["retained_layerstate_build_only_ms"] = tm(lambda: [qsgd_layer_from_payload(n, s, p, 1.0, 8, 16)
                                                       for (n, s), p in zip(named, payloads)])
res["retained_encode_updates_dict_ms"] = tm(lambda: encode_updates_dict(upd, comp))
res["retained_decode_updates_dict_gpu_ms"] = tm(lambda: decode_updates_dict(layers, device=dev))
print(json.dumps(res), flush=True)
