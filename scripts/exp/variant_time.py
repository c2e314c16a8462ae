"""Time encoders under an experiment library (OMF_CODEC_LIB_EXPERIMENT) — RNG cost sensitivity."""
import os
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


def tm(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


lib = os.environ.get("OMF_CODEC_LIB_EXPERIMENT", "base")
p.set_encode_strategy("ordered")
p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
nin = nr.clone()
row = {"ordered": tm(lambda: p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)),
       "flat(norm in)": tm(lambda: p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, norm_in=nin))}
p.set_encode_strategy("ring")
for cfg in (2, 4):
    p.set_ring(cfg=cfg, big_mode=1)
    row[f"ring{cfg}"] = tm(lambda: p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1))
print(lib.split("/")[-2] if "/" in lib else lib, " ".join(f"{k} {v:.4f}" for k, v in row.items()), flush=True)
