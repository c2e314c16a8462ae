"""Fused PS step (omf_ps_apply_encode: avg = acc / total and its QSGD payload) by strategy, Llama-400M
(experiment; interleaved)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(os.environ.get("MODEL", "llama400m"))]
plans = {}
for sn in ("bracket", "ring", "ordered"):
    p = codec.Plan(sizes, device=dev)
    p.set_encode_strategy(sn)
    plans[sn] = p
acc = torch.randn(plans["ring"].arena_end, device=dev) * 1e-2
avg = torch.empty_like(acc)
q = torch.empty(plans["ring"].payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
res = {sn: [] for sn in plans}
for rnd in range(6):
    for sn, p in plans.items():
        p.ps_apply_encode(acc, 7.0, 4, avg_out=avg, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(10):
            p.ps_apply_encode(acc, 7.0, 4, avg_out=avg, q_out=q, norm_out=nr, seed=1, offset=i)
        e1.record()
        torch.cuda.synchronize()
        res[sn].append(e0.elapsed_time(e1) / 10)
for sn, v in res.items():
    v = sorted(v)
    print(f"fused PS step {sn:8s}: median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}", flush=True)
