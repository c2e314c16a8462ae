"""Bracketed-encoder diagnostics (spec_stats) on Llama-400M for fp32 / bf16 / fp16 values, s = 4."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(1000)
x0 = torch.randn(p.arena_end, device=dev, generator=g) * 1e-3
out = {}
for fmt, dt in ((0, None), (1, torch.bfloat16), (2, torch.float16)):
    x = x0 if dt is None else x0.to(dt).float()
    for alpha in (1.0, 3.0):
        p.qsgd_encode(x, 4, alpha=alpha, seed=7, offset=1, value_format=fmt)
        out[f"fmt{fmt}_a{alpha:g}"] = p.spec_stats()
p.check()
print(json.dumps(out), flush=True)
