"""Encode/decode time per plan chunk size on the L400 arena (HIP events, interleaved rounds)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "llama400m"
chunks = [int(c) for c in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["16384", "65536", "131072", "262144"])]
dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(cfg)]
N = sum(sizes)
plans = {c: codec.Plan.get(sizes, device=dev, chunk=c) for c in chunks}
p0 = plans[chunks[0]]
x = torch.randn(p0.arena_end, device=dev) * 1e-3
q = torch.empty(p0.arena_end, dtype=torch.int8, device=dev)
y = torch.empty(p0.arena_end, device=dev)
nrm = torch.empty(p0.nt, device=dev)
res = {c: ([], []) for c in chunks}
for rnd in range(8):
    for c, p in plans.items():
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        p.qsgd_encode(x, 4, q_out=q, norm_out=nrm, seed=1, offset=rnd)
        e[1].record()
        p.qsgd_decode(q, 8, 16, nrm, y_out=y)
        e[2].record()
        torch.cuda.synchronize()
        if rnd:
            res[c][0].append(e[0].elapsed_time(e[1]))
            res[c][1].append(e[1].elapsed_time(e[2]))
    p.check()
for c in chunks:
    em, dm = np.median(res[c][0]), np.median(res[c][1])
    print(f"chunk {c:7d} items {plans[c].encode_items:6d}  encode {em:.4f} ms {5*N/em/1e6:7.1f} GB/s"
          f"  decode {dm:.4f} ms {5*N/dm/1e6:7.1f} GB/s  step {10*N/(em+dm)/1e6:7.1f} GB/s")
