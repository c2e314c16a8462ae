"""Top-K encode + arena decode, back to back (experiment, for rocprofv3 --kernel-trace
--hip-runtime-trace): where the GPU idles between the two calls."""
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
xs = [torch.randn(p.arena_end, device=dev, generator=g) * 1e-3 for _ in range(2)]
res = torch.zeros(p.arena_end, device=dev)
K = sum(p.topk_ks(0.01))
vals = torch.empty(K, device=dev)
idx = torch.empty(K, dtype=torch.int64, device=dev)
y = torch.empty(p.arena_end, device=dev)
for i in range(30):
    p.topk_encode(xs[i % 2], 0.01, residual=res, residual_mode=1, values=vals, indices=idx, alpha=2.0)
    p.topk_decode_arena(vals, idx, 0.01, y=y, mode=0)
torch.cuda.synchronize()
print("ok", flush=True)
