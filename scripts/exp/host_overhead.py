"""Host cost of one codec call (experiment): the Python wrapper against its parts, ResNet-18 arena
(GPU work per call is shorter than the host's, so the timings are host-bound)."""
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
plan = codec.Plan(sizes, device=dev)
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
y = torch.empty(plan.arena_end, device=dev)
L = lib()
st = torch.cuda.current_stream(dev).cuda_stream


def per_call(fn, n=2000):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return round((t1 - t0) / n * 1e6, 2)


args = (plan.handle, ctypes.c_void_p(q.data_ptr()), 8, 8, ctypes.c_void_p(nr.data_ptr()), ctypes.c_void_p(y.data_ptr()),
        0, ctypes.c_void_p(st))
res = {
    "torch.cuda.current_stream": per_call(lambda: torch.cuda.current_stream(dev).cuda_stream),
    "raw_stream": per_call(lambda: torch._C._cuda_getCurrentRawStream(0)),
    "decode_ctypes_only": per_call(lambda: L.omf_qsgd_decode(*args)),
    "decode_wrapper": per_call(lambda: plan.qsgd_decode(q, 8, 8, nr, y_out=y)),
    "encode_wrapper": per_call(lambda: plan.qsgd_encode(x, 3, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=0), 500),
    "torch_empty_like_launch": per_call(lambda: y.zero_()),
}
print(json.dumps(res), flush=True)
