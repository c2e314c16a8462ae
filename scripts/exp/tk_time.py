"""Top-K encode (k = 1 %, error feedback, Llama-400M) timed in back-to-back loops (experiment)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
res = torch.zeros(p.arena_end, device=dev)
K = sum(p.topk_ks(0.01))
vals = torch.empty(K, device=dev)
idx = torch.empty(K, dtype=torch.int64, device=dev)
f = lambda: p.topk_encode(x, 0.01, residual=res, residual_mode=1, values=vals, indices=idx, alpha=2.0)
ts = []
for rnd in range(6):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        f()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10)
ts.sort()
print(f"topk encode: median {ts[len(ts) // 2]:.4f} ms  min {ts[0]:.4f}", flush=True)
