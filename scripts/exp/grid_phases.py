"""Grid encoder phase costs on ResNet-18 s = 3 (experiment): the encode loop timed with phases
switched off through omf_plan_set_debug (64 no barrier wait, 128 no fold, 256 no quantisation).
Outputs of the switched runs are meaningless; the plan is checked clean afterwards."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes(sys.argv[1] if len(sys.argv) > 1 else "resnet18")]
plan = codec.Plan(sizes, device=dev)
plan.set_encode_strategy("grid")
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
res = {}
for bits in (0, 256, 128 | 256, 64 | 128 | 256, 64, 64 | 128, 0):
    plan.set_debug(spec=bits)
    ts = []
    for rnd in range(7):
        for i in range(3):
            plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(50):
            plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 50 * 1e3)
    res[str(bits)] = round(sorted(ts)[3], 2)
    print(json.dumps({bits: res[str(bits)]}), flush=True)
plan.set_debug()
plan.qsgd_encode(x, 3, q_out=q, norm_out=nr)
plan.check()
print(json.dumps(res), flush=True)
