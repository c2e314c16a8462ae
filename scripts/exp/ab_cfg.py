"""A/B the ring configurations given on the command line, interleaved in one process (experiment)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
cfgs = [int(c) for c in sys.argv[1:]] or [0, 5]
plans = {}
for c in cfgs:
    p = codec.Plan(sizes, device=dev)
    p.set_ring(cfg=c, big_mode=1)
    plans[c] = p
x = torch.randn(plans[cfgs[0]].arena_end, device=dev) * 1e-3
q = torch.empty(plans[cfgs[0]].payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
res = {c: [] for c in cfgs}
for rnd in range(6):
    for c in cfgs:
        p = plans[c]
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=rnd)
        e1.record()
        torch.cuda.synchronize()
        res[c].append(e0.elapsed_time(e1) / 10)
        assert p.check()
for c in cfgs:
    v = sorted(res[c])
    print(f"cfg {c}: median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}  all {' '.join(f'{t:.4f}' for t in res[c])}", flush=True)
