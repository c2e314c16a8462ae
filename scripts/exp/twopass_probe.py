"""Two-pass encoder traffic with cache policies (experiment; see twopass_probe.hip)."""
import ctypes
import subprocess

import torch

so = "/tmp/twopass_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                "scripts/exp/twopass_probe.hip"], check=True)
L = ctypes.CDLL(so)
L.twopass_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 400 * (1 << 20)
x = torch.randn(N, device=dev)
q = torch.empty(N // 4, dtype=torch.int32, device=dev)
part = torch.zeros(1024, device=dev)
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


alg = 5 * N
for pol in range(4):
    t = timed(lambda: L.twopass_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, N, pol, st))
    print(f"full passes pol {pol}: {t:.3f} ms ({alg / t / 1e6:.0f} GB/s alg)", flush=True)
for mb in (8, 16, 25, 40, 50, 100):
    W = mb * (1 << 20)
    for pol in range(4):
        t = timed(lambda: L.twopass_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, W, pol, st))
        print(f"window {4 * mb:4d} MB pol {pol}: {t:.3f} ms ({alg / t / 1e6:.0f} GB/s alg)", flush=True)
