"""Two-pass encoder: items between a tensor's NORM and QUANT items (OMF_TWOPASS_GAP, read at plan
creation; -1 = one tensor of slack, the default), interleaved (experiment)."""
import os
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(os.environ.get("MODEL", "llama400m"))]
gaps = sys.argv[1:] or ["-1", "0", "64", "256", "1024"]
plans = {}
for gp in gaps:
    os.environ["OMF_TWOPASS_GAP"] = gp
    plans[gp] = codec.Plan(sizes, device=dev)
    plans[gp].set_encode_strategy("ordered")
x = torch.randn(plans[gaps[0]].arena_end, device=dev) * 1e-3
q = torch.empty(plans[gaps[0]].payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
res = {g: [] for g in gaps}
for rnd in range(8):
    for g, p in plans.items():
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=rnd)
        e1.record()
        torch.cuda.synchronize()
        assert p.check() is not None
        res[g].append(e0.elapsed_time(e1) / 10)
for g in res:
    t = sorted(res[g])
    print(f"gap {g:>5s}: median {t[len(t) // 2]:.4f} ms min {t[0]:.4f}", flush=True)
