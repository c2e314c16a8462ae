"""A/B the encode strategies (ring / ordered two-pass / resident) and the flat quantiser with the
norms given, interleaved in one process (experiment)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
MODEL = __import__("os").environ.get("MODEL", "llama400m")
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(MODEL)]
strats = sys.argv[1:] or ["ring", "ordered"]
plans = {}
for sname in strats:
    p = codec.Plan(sizes, device=dev)
    if sname not in ("flat", "norms"):
        p.set_encode_strategy(sname)
    elif sname == "norms":
        p.set_encode_strategy("ordered")
    plans[sname] = p
x = torch.randn(plans[strats[0]].arena_end, device=dev) * 1e-3
q = torch.empty(plans[strats[0]].payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
plans[strats[0]].qsgd_norms(x, norm_out=nr)
res = {sn: [] for sn in strats}
for rnd in range(6):
    for sn in strats:
        p = plans[sn]

        def run(o):
            if sn == "flat":
                p.qsgd_encode(x, 4, q_out=q, norm_in=nr, seed=1, offset=o)
            elif sn == "norms":
                p.qsgd_norms(x, norm_out=nr)
            else:
                p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=o)
        run(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run(rnd)
        e1.record()
        torch.cuda.synchronize()
        res[sn].append(e0.elapsed_time(e1) / 10)
for sn in strats:
    v = sorted(res[sn])
    print(f"{MODEL} {sn:8s}: median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}", flush=True)
if "bracket" in plans:
    plans["bracket"].qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, offset=99)
    print(f"{MODEL} bracket stats: {plans['bracket'].spec_stats()}", flush=True)
