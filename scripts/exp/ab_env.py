"""A/B one environment switch the library reads per launch (e.g. OMF_QUANT_NT=0/1) on the default
encoder, interleaved in one process (experiment).  Usage: ab_env.py VAR [values...]"""
import os
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

var = sys.argv[1]
vals = sys.argv[2:] or ["0", "1"]
dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
res = {v: [] for v in vals}
for rnd in range(8):
    for v in vals:
        os.environ[var] = v
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=rnd)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 10)
for v in vals:
    t = sorted(res[v])
    print(f"{p.strategy} {var}={v}: median {t[len(t) // 2]:.4f} ms min {t[0]:.4f}", flush=True)
