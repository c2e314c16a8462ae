"""ResNet-18 (BASELINE config 2) encoder variants, interleaved in one process (HIP events around
`reps` back-to-back calls, median over rounds): the ring encoder (default below 2^25 elements), the
grid encoder, the bracketed single-read encoder (fused bracket), and two launches — the norms pass (omf_qsgd_norms) then the quantiser with those
norms (omf_qsgd_encode norm_in) — plus the decoder and encode + decode steps.  s = 3 (8 levels)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

s = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 9
reps = 50
dev = torch.device("cuda", 0)
sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes("resnet18")]
plans = {name: codec.Plan(sizes, device=dev) for name in ("ring", "grid", "two", "bracket")}
plans["grid"].set_encode_strategy("grid")
plans["two"].set_encode_strategy("ordered")
plans["bracket"].set_encode_strategy("bracket")  # the fused-bracket single-read encoder
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(plans["ring"].arena_end, device=dev, generator=g) * 1e-3
L = 2**s
w = 8 if L <= 127 else 32
q = torch.empty(plans["ring"].payload_elems(w), dtype=torch.int8 if w == 8 else torch.int32, device=dev)
nr = torch.empty(len(sizes), device=dev)
y = torch.empty(plans["ring"].arena_end, device=dev)
st = torch.cuda.current_stream(dev)


def enc(name, i):
    p = plans[name]
    if name == "two":
        p.qsgd_norms(x, norm_out=nr)
        p.qsgd_encode(x, s, q_out=q, norm_out=nr, norm_in=nr, seed=7, offset=i)
    else:
        p.qsgd_encode(x, s, q_out=q, norm_out=nr, seed=7, offset=i)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)
    a.record(st)
    for i in range(reps):
        fn(i)
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


res = {}
for r in range(rounds):
    for name in plans:
        res.setdefault(f"{name}_enc_us", []).append(timed(lambda i: enc(name, i)))
        res.setdefault(f"{name}_step_us", []).append(
            timed(lambda i: (enc(name, i), plans["ring"].qsgd_decode(q, w, L, nr, y_out=y))))
    res.setdefault("decode_us", []).append(timed(lambda i: plans["ring"].qsgd_decode(q, w, L, nr, y_out=y)))
    for p in plans.values():
        p.check()
out = {"s": s, "rounds": rounds, "reps": reps, "elements": sum(sizes)}
for k, v in res.items():
    v = sorted(v)
    out[k] = round(v[len(v) // 2], 2)
# the variants' payloads: the ring's and the grid's equal given their norms; the two-launch one too
outs = {}
for name in plans:
    enc(name, 3)
    torch.cuda.synchronize()
    outs[name] = (q.clone(), nr.clone())
out["norms_equal_ring_grid"] = bool(torch.equal(outs["ring"][1], outs["grid"][1]))
out["bracket_encoder"] = plans["bracket"].last_encoder
print(json.dumps(out), flush=True)
