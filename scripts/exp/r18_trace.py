"""ResNet-18 s = 3 encode + decode, back to back (experiment, for rocprofv3 --kernel-trace): the
kernels' durations and the idle gaps between them come from the trace (scripts/exp/trace_gaps.py)."""
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
strategy = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "-" else None
pattern = sys.argv[2] if len(sys.argv) > 2 else "ed"  # e = encode, d = decode, per step
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("resnet18")]
plan = codec.Plan(sizes, device=dev)
if strategy:
    plan.set_encode_strategy(strategy)
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
y = torch.empty(plan.arena_end, device=dev)
for i in range(300):
    for c in pattern:
        if c == "e":
            plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)
        else:
            plan.qsgd_decode(q, 8, 8, nr, y_out=y)
torch.cuda.synchronize()
plan.check()
print("ok", flush=True)
