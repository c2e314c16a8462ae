"""Windowed fill+scatter probe for the Top-K arena decode (experiment; see scatter_probe.hip)."""
import ctypes
import subprocess

import torch

so = "/tmp/scatter_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                "scripts/exp/scatter_probe.hip"], check=True)
L = ctypes.CDLL(so)
L.probe_run.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                        ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 400 * (1 << 20)
y = torch.empty(N, device=dev)
flush = torch.empty(1 << 29, device=dev)
st = torch.cuda.current_stream().cuda_stream


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


for mb in (16, 32, 64, 128, 200):
    W = mb * (1 << 18)  # elements (4 B each) per window: mb MB
    nwin = N // W
    # 1 % of each window, random positions, grouped by window
    per = W // 100
    idx = (torch.randint(0, W, (nwin, per), device=dev) + torch.arange(nwin, device=dev)[:, None] * W).reshape(-1)
    val = torch.randn(idx.numel(), device=dev)
    ws = torch.arange(0, nwin + 1, dtype=torch.int64) * per
    t0 = timed(lambda: L.probe_run(y.data_ptr(), N, idx.data_ptr(), val.data_ptr(), ws.data_ptr(), nwin, W, 0, st))
    t1 = timed(lambda: L.probe_run(y.data_ptr(), N, idx.data_ptr(), val.data_ptr(), ws.data_ptr(), nwin, W, 1, st))
    print(f"window {mb:4d} MB: fill then scatter {t0:.3f} ms | windowed {t1:.3f} ms ({nwin} launches)", flush=True)
