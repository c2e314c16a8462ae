"""A/B the flat quantiser (norms given) variants OMF_QUANT_VARIANT=0..4, interleaved (experiment; the
variants were removed once variant 1, 4 Ki-element blocks, became the quantiser)."""
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
p.qsgd_norms(x, norm_out=nr)
ref = None
vals = sys.argv[1:] or ["0", "1", "2", "3", "4"]
res = {v: [] for v in vals}
for rnd in range(6):
    for v in vals:
        os.environ["OMF_QUANT_VARIANT"] = v
        p.qsgd_encode(x, 4, q_out=q, norm_in=nr, seed=1)
        torch.cuda.synchronize()
        if rnd == 0:
            if ref is None:
                ref = q.clone()
            assert torch.equal(q, ref), v
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_in=nr, seed=1)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 10)
for v in vals:
    t = sorted(res[v])
    print(f"quant variant {v}: median {t[len(t) // 2]:.4f} ms min {t[0]:.4f}", flush=True)
