"""Top-K encode: GPU time per call in a back-to-back loop vs the host time each call takes
(experiment: is the host path, which waits for the plan's verdict, the bottleneck?)."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan.get(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
res = torch.zeros(p.arena_end, device=dev)
K = sum(p.topk_ks(0.01))
vals = torch.empty(K, device=dev)
idx = torch.empty(K, dtype=torch.int64, device=dev)
for _ in range(3):
    p.topk_encode(x, 0.01, residual=res, residual_mode=1, values=vals, indices=idx)
torch.cuda.synchronize()
n = 20
host = []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record()
for _ in range(n):
    h0 = time.perf_counter()
    p.topk_encode(x, 0.01, residual=res, residual_mode=1, values=vals, indices=idx)
    host.append(time.perf_counter() - h0)
e1.record()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / n
print(f"per call: GPU events {e0.elapsed_time(e1) / n:.3f} ms, wall {wall * 1e3:.3f} ms, host inside call "
      f"median {sorted(host)[n // 2] * 1e3:.3f} ms", flush=True)
