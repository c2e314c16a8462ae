"""Two-pass encoder with 8 vs 16 rows per thread (OMF_ENCODE_ROWS, read at plan creation), interleaved (experiment)."""
import os
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
plans = {}
for rows in ("16", "8"):
    os.environ["OMF_ENCODE_ROWS"] = rows
    plans[rows] = codec.Plan(sizes, device=dev)
    plans[rows].set_encode_strategy("ordered")
x = torch.randn(plans["16"].arena_end, device=dev) * 1e-3
q = torch.empty(plans["16"].payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
res = {r: [] for r in plans}
for rnd in range(6):
    for r, p in plans.items():
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=rnd)
        e1.record()
        torch.cuda.synchronize()
        res[r].append(e0.elapsed_time(e1) / 10)
for r in res:
    t = sorted(res[r])
    print(f"ordered rows {r}: median {t[len(t) // 2]:.4f} ms min {t[0]:.4f}", flush=True)
