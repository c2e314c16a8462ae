"""PCIe copy rates on the box: H2D alone, D2H alone, both at once on two streams (pinned host
buffers of `MB` MiB, events), and the same with the copy split into `chunks` pieces."""
import json
import os
import sys

import torch

MB = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = torch.device("cuda", 0)
n = MB << 18
ha, hb = torch.empty(n, pin_memory=True), torch.empty(n, pin_memory=True)
da, db = torch.empty(n, device=dev), torch.empty(n, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    for s in (s1, s2):
        torch.cuda.current_stream().wait_stream(s)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def h2d():
    with torch.cuda.stream(s1):
        da.copy_(ha, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        hb.copy_(db, non_blocking=True)


def both():
    h2d()
    d2h()


gb = 4 * n / 1e9
out = {"MB": MB, "HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA")}
for name, fn, bytes_ in (("h2d", h2d, gb), ("d2h", d2h, gb), ("both", both, 2 * gb)):
    ms = timed(fn)
    out[name + "_ms"] = round(ms, 2)
    out[name + "_GBs"] = round(bytes_ / ms * 1e3, 1)
print(json.dumps(out), flush=True)
