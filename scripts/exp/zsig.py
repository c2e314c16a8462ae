"""Bracketed encode time vs the bracket's width (OMF_SPEC_ZSIG sigmas; experiment, interleaved)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
zs = ["2", "3", "4", "6", "9"]
plans = {}
for z in zs:
    os.environ["OMF_SPEC_ZSIG"] = z
    p = codec.Plan(sizes, device=dev)
    p.set_encode_strategy("bracket")
    plans[z] = p
os.environ.pop("OMF_SPEC_ZSIG")
x = torch.randn(plans["6"].arena_end, device=dev) * 1e-3
q = torch.empty(plans["6"].payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
res = {z: [] for z in zs}
for rnd in range(7):
    for z, p in plans.items():
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=i)
        e1.record()
        torch.cuda.synchronize()
        res[z].append(e0.elapsed_time(e1) / 10)
for z, p in plans.items():
    v = sorted(res[z])
    p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
    print(f"zsig {z}: median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}  {p.spec_stats()}", flush=True)
