"""Top-K encode on the Llama-400M arena (k = 1 %), for rocprofv3 (experiment).  Error-feedback
calls take a fresh gradient each call (t' = residual + x_i), as in training."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(sys.argv[1] if len(sys.argv) > 1 else "llama400m")]
p = codec.Plan.get(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
xs = [torch.randn(p.arena_end, device=dev, generator=g) * 1e-3 for _ in range(6)]
res = torch.zeros(p.arena_end, device=dev)
p.topk_encode(xs[0], 0.01, residual=res, residual_mode=2)
torch.cuda.synchronize()
for mode in (1, 0):
    t0 = time.perf_counter()
    for i in range(5):
        p.topk_encode(xs[1 + i], 0.01, residual=res if mode else None, residual_mode=mode)
    torch.cuda.synchronize()
    print(f"topk mode {mode}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms", flush=True)
