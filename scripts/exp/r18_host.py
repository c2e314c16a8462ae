"""ResNet-18 s = 3: host issue time of one encode / decode call (wall clock per call with the
GPU kept busy, no sync inside the loop) against the GPU time (events); experiment harness."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes("resnet18")]
plan = codec.Plan(sizes, device=dev)
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
y = torch.empty(plan.arena_end, device=dev)
res = {}
for st in ("ring", "grid"):
    plan.set_encode_strategy(st)
    enc = lambda i: plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)
    dec = lambda i: plan.qsgd_decode(q, 8, 8, nr, y_out=y)
    for name, fn in (("enc", enc), ("dec", dec)):
        for i in range(20):
            fn(i)
        torch.cuda.synchronize()
        # host issue cost: the GPU is held busy by a long kernel first so the loop never waits
        torch.cuda._sleep(50_000_000)
        t0 = time.perf_counter()
        for i in range(200):
            fn(i)
        host_us = (time.perf_counter() - t0) / 200 * 1e6
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(200):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        res[f"{st}_{name}"] = {"host_issue_us": round(host_us, 2), "event_us": round(e0.elapsed_time(e1) / 200 * 1e3, 2)}
    print(json.dumps(res), flush=True)
