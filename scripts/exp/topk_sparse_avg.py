"""The PS's Top-K downlink on the sparse average of two clients' Top-K decodes (the reference's
steady state, conf/base.yaml:194-198) through the drop-in API, as scripts/wire_bench.py times it:
each client's second error-feedback encode_updates_dict, accumulate_layers on the PS, then repeated
apply_and_encode (the PS re-encodes the average for every client's GetUpdatedModel), with the plan's
verdict counters per call; OMF_TOPK_DBG=12 prints the verdicts and over-full fine bins.
usage: topk_sparse_avg.py [overlap|disjoint]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402
from omnifed_amd.hybrid.communicator.global_grpc_compression import (  # noqa: E402
    build_global_compressor, encode_updates_dict)
from omnifed_amd.ps import DeviceAggregator  # noqa: E402

dev = torch.device("cuda", 0)
mode = sys.argv[1] if len(sys.argv) > 1 else "disjoint"
named = shapes.model_shapes("llama400m")
g = torch.Generator(device=dev).manual_seed(0)
upd = {n: torch.randn(s, device=dev, generator=g) * 1e-3 for n, s in named}
plan = codec.Plan.get([t.numel() for t in upd.values()], device=dev)
agg = DeviceAggregator(named, device=dev)
for c in range(2):
    cc = build_global_compressor(enabled=True, scheme="topk", compress_ratio=0.01, device=dev)
    if mode == "disjoint":
        u = upd if c == 0 else {n: torch.randn(t.shape, device=dev, generator=g) * 1e-3 for n, t in upd.items()}
    else:
        u = {n: t + (0.05 * c) * torch.randn(t.shape, device=dev, generator=g) * 1e-3 for n, t in upd.items()}
    encode_updates_dict(u, cc)
    agg.accumulate_layers(encode_updates_dict(u, cc), number_samples=1)
srv = build_global_compressor(enabled=True, scheme="topk", compress_ratio=0.01, device=dev)
out = []
for call in range(12):
    plan.topk_stats(reset=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    agg.apply_and_encode(srv, total_samples=2)
    b.record()
    torch.cuda.synchronize()
    st = plan.topk_stats(reset=True)
    out.append({"call": call, "ms": round(a.elapsed_time(b), 3), **{k: st[k] for k in ("fast", "fallback", "zero_fill", "redo")}})
print(json.dumps({"mode": mode, "nnz_per_k": round(int((agg.acc != 0).sum()) / sum(plan.topk_ks(0.01)), 3),
                  "calls": out}))
