"""ResNet-18 s = 3: the ring encoder against norms-then-quantise as two launches (experiment;
events around 200 back-to-back encodes, median of 7 rounds, interleaved)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("resnet18")]
plan = codec.Plan(sizes, device=dev)
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
n2 = torch.empty(plan.nt, device=dev)
y = torch.empty(plan.arena_end, device=dev)


def ring(i):
    plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)


def two(i):
    plan.qsgd_norms(x, alpha=2.0, norm_out=n2)
    plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i, norm_in=n2)


def norms_only(i):
    plan.qsgd_norms(x, alpha=2.0, norm_out=n2)


def quant_only(i):
    plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i, norm_in=n2)


fns = {"ring": ring, "norms+quant": two, "norms": norms_only, "quant(norms given)": quant_only}
ts = {k: [] for k in fns}
for f in fns.values():
    for i in range(5):
        f(i)
torch.cuda.synchronize()
for rnd in range(7):
    for k, f in fns.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(200):
            f(i)
        e1.record()
        torch.cuda.synchronize()
        ts[k].append(e0.elapsed_time(e1) / 200 * 1e3)
ring(0)
torch.cuda.synchronize()
n_ring = nr.clone()
plan.qsgd_norms(x, alpha=2.0, norm_out=n2)
torch.cuda.synchronize()
print(json.dumps({k: round(sorted(v)[3], 2) for k, v in ts.items()}), flush=True)
print(json.dumps({"norms_equal_ring": bool(torch.equal(n_ring, n2)),
                  "max_rel": float(((n_ring - n2).abs() / n_ring.abs().clamp_min(1e-30)).max())}), flush=True)
