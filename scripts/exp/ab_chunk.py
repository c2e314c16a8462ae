"""Ordered (two-pass) encoder: NORM/QUANT item size sweep, interleaved in one process (experiment)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(sys.argv[1] if len(sys.argv) > 1 else "llama400m")]
chunks = [16384 * m for m in (2, 4)]
plans = {c: codec.Plan(sizes, device=dev, chunk=c) for c in chunks}
for p in plans.values():
    p.set_encode_strategy("ordered")
p0 = plans[chunks[0]]
x = torch.randn(p0.arena_end, device=dev) * 1e-3
q = torch.empty(p0.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
res = {c: [] for c in chunks}
for rnd in range(12):
    for c in chunks:
        p = plans[c]
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=rnd)
        e1.record()
        torch.cuda.synchronize()
        res[c].append(e0.elapsed_time(e1) / 10)
for c in chunks:
    t = sorted(res[c])
    print(f"chunk {c // 1024:5d} Ki: median {t[len(t) // 2]:.4f} ms min {t[0]:.4f}", flush=True)
