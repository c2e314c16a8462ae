"""Run the encoders (ring, flat with norms supplied) and the decoder a few times each on
Llama-400M s=4 — a short program for rocprofv3 --pmc passes (experiment)."""
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.arena_end, dtype=torch.int8, device=dev)
nr = torch.empty(p.nt, device=dev)
y = torch.empty_like(x)
p.set_encode_strategy("ring")
for _ in range(4):
    p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
nin = nr.clone()
for _ in range(4):
    p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, norm_in=nin)
for _ in range(4):
    p.qsgd_decode(q, 8, 16, nr, y_out=y)
torch.cuda.synchronize()
print("ok", flush=True)
