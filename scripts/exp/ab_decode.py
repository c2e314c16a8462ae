"""A/B the QSGD decoder's payload-load policy (OMF_DEC_NTL=0/1, read per call), interleaved (experiment)."""
import os
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
y = torch.empty(p.arena_end, device=dev)
res = {"0": [], "1": []}
VAR = sys.argv[1] if len(sys.argv) > 1 else "OMF_DEC_NTL"
for rnd in range(8):
    for v in ("0", "1"):
        os.environ[VAR] = v
        p.qsgd_decode(q, 8, 16, nr, y_out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_decode(q, 8, 16, nr, y_out=y)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 10)
for v in res:
    t = sorted(res[v])
    print(f"decode {VAR}={v}: median {t[len(t) // 2]:.4f} ms min {t[0]:.4f}", flush=True)
