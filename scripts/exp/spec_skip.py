"""Marginal cost of each bracketed-encoder launch: encode timings with spec debug bits (Plan.set_debug)
(experiment; each setting in its own plan, interleaved)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(os.environ.get("MODEL", "llama400m"))]
settings = [0, 2, 4, 8]
plans = {}
for sk in settings:
    p = codec.Plan(sizes, device=dev)
    p.set_encode_strategy("bracket")
    plans[sk] = p
x = torch.randn(plans[0].arena_end, device=dev) * 1e-3
q = torch.empty(plans[0].payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
for sk, p in plans.items():
    p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)  # brackets exist before skipping them
    p.set_debug(spec=sk)
res = {sk: [] for sk in settings}
for rnd in range(7):
    for sk in settings:
        p = plans[sk]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(20):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=i)
        e1.record()
        torch.cuda.synchronize()
        res[sk].append(e0.elapsed_time(e1) / 20)
names = {0: "all three", 2: "bracket+quant", 4: "fix: no stores", 8: "fix: heads only"}
for sk in settings:
    v = sorted(res[sk])
    print(f"{names[sk]:14s}: median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}", flush=True)
