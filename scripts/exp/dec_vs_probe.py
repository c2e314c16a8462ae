"""Production decoder vs the streaming probe's best decode shape, both in back-to-back loops of 10,
interleaved (experiment)."""
import ctypes
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnifed_amd import codec, shapes  # noqa: E402

so = "/tmp/dec_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/dec_probe.hip"],
               check=True)
L = ctypes.CDLL(so)
L.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(len(sizes), device=dev)
p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
y = torch.empty(p.arena_end, device=dev)
N = (p.arena_end // 16) * 16
st = torch.cuda.current_stream().cuda_stream
fns = {"production": lambda: p.qsgd_decode(q, 8, 16, nr, y_out=y),
       "probe U4 ntL ntS": lambda: L.probe_run(3, q.data_ptr(), y.data_ptr(), N, st),
       "probe U1 ntL ntS": lambda: L.probe_run(1, q.data_ptr(), y.data_ptr(), N, st),
       "probe vec16 ntL ntS": lambda: L.probe_run(5, q.data_ptr(), y.data_ptr(), N, st)}
res = {k: [] for k in fns}
for rnd in range(7):
    for k, fn in fns.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 10)
for k, v in res.items():
    v = sorted(v)
    print(f"{k:20s}: median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}", flush=True)
