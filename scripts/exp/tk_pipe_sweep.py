"""Top-K encode time (Llama-400M, k = 1 %, error feedback, a fresh gradient per call) against the
pipeline group count (OMF_TOPK_GROUPS) and the sample size (OMF_TOPK_SAMPLE_RUNS); every
configuration's output is checked equal to the one-group run's (experiment harness)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
xs = [torch.randn(p.arena_end, device=dev, generator=g) * 1e-3 for _ in range(4)]
K = sum(p.topk_ks(0.01))
vals = torch.empty(K, device=dev)
idx = torch.empty(K, dtype=torch.int64, device=dev)
ref = None
out = {}
for groups, runs in [(1, 2048), (2, 2048), (4, 2048), (8, 2048), (4, 4096), (4, 16384), (8, 16384)]:
    os.environ["OMF_TOPK_GROUPS"] = str(groups)
    os.environ["OMF_TOPK_SAMPLE_RUNS"] = str(runs)
    res = torch.zeros(p.arena_end, device=dev)
    # correctness: three EF calls from a zero residual give the same bytes in every configuration
    for i in range(3):
        p.topk_encode(xs[i], 0.01, residual=res, residual_mode=1, values=vals, indices=idx, alpha=2.0)
    got = (vals.clone(), idx.clone(), res.clone())
    if ref is None:
        ref = got
    same = all(torch.equal(a, b) for a, b in zip(ref, got))
    f = lambda i: p.topk_encode(xs[i % 4], 0.01, residual=res, residual_mode=1, values=vals, indices=idx, alpha=2.0)
    for i in range(8):
        f(i)
    torch.cuda.synchronize()
    ts = []
    for rnd in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(20):
            f(i)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20)
    ts.sort()
    key = f"g{groups}_r{runs}"
    out[key] = {"median_ms": round(ts[2], 4), "min_ms": round(ts[0], 4), "same_as_g1": same}
    print(json.dumps({key: out[key]}), flush=True)
print(json.dumps(out), flush=True)
