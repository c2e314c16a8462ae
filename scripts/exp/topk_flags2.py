"""Top-K fast-path coverage by input distribution (experiment; run with OMF_TOPK_DBG=4, which
prints each call's redo / overflow flags on stderr): Llama-400M shapes, k = 1 %, 4 error-feedback
calls per distribution and seed."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan.get(sizes, device=dev)
res = torch.zeros(p.arena_end, device=dev)
n = p.arena_end


def dist(name, g):
    z = torch.randn(n, device=dev, generator=g)
    if name == "gauss":
        return z * 1e-3
    if name == "laplace":
        u = torch.rand(n, device=dev, generator=g) - 0.5
        return -torch.sign(u) * torch.log1p(-2 * u.abs()) * 1e-3
    if name == "student3":  # heavy tails: z / sqrt(chi2_3 / 3)
        c = (torch.randn(n, device=dev, generator=g) ** 2 + torch.randn(n, device=dev, generator=g) ** 2
             + torch.randn(n, device=dev, generator=g) ** 2) / 3
        return z / c.sqrt() * 1e-3
    if name == "uniform":
        return (torch.rand(n, device=dev, generator=g) - 0.5) * 1e-3
    raise ValueError(name)


for name in ("gauss", "laplace", "student3", "uniform"):
    for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        g = torch.Generator(device=dev).manual_seed(seed)
        x = dist(name, g)
        print(f"== {name} {seed}", file=sys.stderr, flush=True)
        for call in range(4):
            p.topk_encode(x, 0.01, residual=res, residual_mode=2 if call == 0 else 1)
        torch.cuda.synchronize()
        del x
print("done", flush=True)
