"""Bracketed encode and the flat quantiser (norms given), 10 launches each on Llama-400M (counter passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(os.environ.get("MODEL", "llama400m"))]
p = codec.Plan(sizes, device=dev)
p.set_encode_strategy("bracket")
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
for i in range(10):
    p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=i)
for i in range(10):
    p.qsgd_encode(x, 4, q_out=q, norm_in=nr, seed=1, offset=i)
torch.cuda.synchronize()
print("ok")
