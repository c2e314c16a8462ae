"""Streaming floor of the Top-K error-feedback pass (experiment; see ef_probe.hip)."""
import ctypes
import subprocess

import torch

so = "/tmp/ef_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/ef_probe.hip"],
               check=True)
L = ctypes.CDLL(so)
L.ef_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 401122304
x = torch.randn(N, device=dev)
r = torch.zeros(N, device=dev)
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


alg = 12 * N
t = timed(lambda: r.add_(x))
print(f"torch r.add_(x): {t:.3f} ms {alg / t / 1e6:.0f} GB/s", flush=True)
names = ["stream U4", "stream U4 nt-store", "stream U4 nt-store nt-load", "stream U8", "stream U8 nt-store",
         "stream U2 nt-store", "items 16Ki", "items 16Ki nt-store",
         "flat U1 B256", "flat U2 B256", "flat U4 B256", "flat U1 B512", "flat U2 B512", "flat U4 B512",
         "flat U1 B1024", "flat U2 B256 nt", "flat U4 B256 nt"]
import sys
only = [int(a) for a in sys.argv[1:]]
for v, nm in enumerate(names):
    if only and v not in only:
        continue
    grids = (1024, 2048, 4096, 8192) if v < 6 else (0,)
    for g in grids:
        t = timed(lambda: L.ef_run(v, x.data_ptr(), r.data_ptr(), N, g, st))
        print(f"{nm:28s} grid {g:5d}: {t:.3f} ms {alg / t / 1e6:.0f} GB/s", flush=True)
