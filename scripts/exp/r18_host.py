"""Is the ResNet-18 step (encode + decode, ~40 us of GPU work) bound by the host's launch path?
Times, per step over 200 steps: the host enqueue time (no synchronisation inside the loop), the
wall time to completion, and the GPU time between events — for the Python wrappers
(Plan.qsgd_encode / qsgd_decode) and for the bare ctypes calls with pre-built arguments."""
import ctypes
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402
from omnifed_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("resnet18")]
plan = codec.Plan.get(sizes, device=dev)
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
y = torch.empty(plan.arena_end, device=dev)
st = torch.cuda.current_stream(dev)
L = lib()
n = 200


def wrappers(i):
    plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=1.0, seed=7, offset=i)
    plan.qsgd_decode(q, 8, 8, nr, y_out=y)


h, sp = plan._h, ctypes.c_void_p(st.cuda_stream)
px, pq, pn, py = (ctypes.c_void_p(t.data_ptr()) for t in (x, q, nr, y))
null = ctypes.c_void_p(0)


def bare(i):
    L.omf_qsgd_encode_ex(h, px, 1.0, 3, 0, null, 7, i, null, pq, pn, sp)
    L.omf_qsgd_decode(h, pq, 8, 8, pn, py, 0, sp)


def measure(fn):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record(st)
    for i in range(n):
        fn(i)
    b.record(st)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"enqueue_us_per_step": round((t1 - t0) / n * 1e6, 2), "wall_us_per_step": round((t2 - t0) / n * 1e6, 2),
            "gpu_us_per_step": round(a.elapsed_time(b) / n * 1e3, 2)}


out = {"wrappers": measure(wrappers)}
try:
    out["bare_ctypes"] = measure(bare)
except Exception as e:  # the decode entry's signature differs: report the wrappers only
    out["bare_ctypes_error"] = repr(e)
plan.check()
print(json.dumps(out), flush=True)
