"""Top-K fast-path coverage (experiment): how often the bucket plan falls back, over random
Llama-400M-shaped inputs and error-feedback sequences (OMF_TOPK_DBG=4 prints the flags)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan.get(sizes, device=dev)
res = torch.zeros(p.arena_end, device=dev)
for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(p.arena_end, device=dev, generator=g) * 1e-3
    p.topk_encode(x, 0.01)
    for call in range(3):
        p.topk_encode(x, 0.01, residual=res, residual_mode=2 if call == 0 else 1)
    torch.cuda.synchronize()
print("done", flush=True)
