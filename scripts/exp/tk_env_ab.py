"""Interleaved A/B of Top-K encode (and arena decode) time against per-call environment switches
(Llama-400M, k = 1 %, error feedback, a fresh gradient per call); experiment harness.

  python scripts/exp/tk_env_ab.py VAR=a,b[,c] [rounds]
Each round times 20 calls of every variant in turn (events on the stream); medians over rounds.
Also checks that every variant produced the same values / indices / residual on one call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

var, vals_s = sys.argv[1].split("=", 1)
# variants separated by ',' (or by ';' when a value itself needs commas: write those as ':')
variants = [v.replace(":", ",") for v in vals_s.split(";")] if ";" in vals_s else vals_s.split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
xs = [torch.randn(p.arena_end, device=dev, generator=g) * 1e-3 for _ in range(4)]
res = torch.zeros(p.arena_end, device=dev)
K = sum(p.topk_ks(0.01))
vals = torch.empty(K, device=dev)
idx = torch.empty(K, dtype=torch.int64, device=dev)
y = torch.empty(p.arena_end, device=dev)


def enc(i):
    p.topk_encode(xs[i % 4], 0.01, residual=res, residual_mode=1, values=vals, indices=idx, alpha=2.0)


# equality: the same call (same residual in, same x) under every variant
r0 = torch.randn(p.arena_end, device=dev, generator=g) * 1e-3
outs = {}
for v in variants:
    os.environ[var] = v
    res.copy_(r0)
    enc(1)
    torch.cuda.synchronize()
    p.topk_decode_arena(vals, idx, 0.01, y=y, mode=0)
    torch.cuda.synchronize()
    outs[v] = (vals.clone(), idx.clone(), res.clone(), y.clone())
same = all(all(torch.equal(a, b) for a, b in zip(outs[variants[0]], outs[v])) for v in variants[1:])
print(json.dumps({"identical_outputs": same}), flush=True)
del outs

ts = {v: [] for v in variants}
td = {v: [] for v in variants}
for v in variants:
    os.environ[var] = v
    for i in range(6):
        enc(i)
torch.cuda.synchronize()
for rnd in range(rounds):
    for v in variants:
        os.environ[var] = v
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        for i in range(20):
            enc(i)
        e1.record()
        for i in range(20):
            p.topk_decode_arena(vals, idx, 0.01, y=y, mode=0)
        e2.record()
        torch.cuda.synchronize()
        ts[v].append(e0.elapsed_time(e1) / 20)
        td[v].append(e1.elapsed_time(e2) / 20)
out = {}
for v in variants:
    a, b = sorted(ts[v]), sorted(td[v])
    out[v] = {"encode_median_ms": round(a[len(a) // 2], 4), "encode_min_ms": round(a[0], 4),
              "decode_median_ms": round(b[len(b) // 2], 4)}
print(json.dumps({var: out}), flush=True)
