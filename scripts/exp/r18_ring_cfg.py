"""ResNet-18 ring encoder configurations (omf_plan_set_ring cfg 0-4: 64 KiB x 2 slots, double-
buffered loaders, 32 KiB x 4, register-resident 4 buffers, register + 2 LDS slots), interleaved:
HIP events around 50 encodes, median over rounds.  s from argv (default 3)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

s = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rounds = 7
dev = torch.device("cuda", 0)
sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes("resnet18")]
plans = {}
for c in range(5):
    p = codec.Plan(sizes, device=dev)
    p.set_encode_strategy("ring")
    p.set_ring(cfg=c)
    plans[c] = p
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(plans[0].arena_end, device=dev, generator=g) * 1e-3
w = 8 if 2**s <= 127 else 32
q = torch.empty(plans[0].payload_elems(w), dtype=torch.int8 if w == 8 else torch.int32, device=dev)
nr = torch.empty(len(sizes), device=dev)
st = torch.cuda.current_stream(dev)


def timed(p, reps=50):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    p.qsgd_encode(x, s, q_out=q, norm_out=nr, seed=7, offset=0)
    a.record(st)
    for i in range(reps):
        p.qsgd_encode(x, s, q_out=q, norm_out=nr, seed=7, offset=i)
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


res = {c: [] for c in plans}
for _ in range(rounds):
    for c, p in plans.items():
        res[c].append(timed(p))
for p in plans.values():
    p.check()
print(json.dumps({"s": s, **{f"cfg{c}_enc_us": round(sorted(v)[len(v) // 2], 2) for c, v in res.items()}}), flush=True)
