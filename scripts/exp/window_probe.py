"""Windowed two-pass probe (experiment): does launch w's re-read of window w hit the Infinity Cache?

For each window size: launches alternate "read window w+1" and "f32->i8 window w"
(window_probe.hip).  Compare with one full read pass + one full convert pass (no reuse
possible) and with the single convert pass alone (floor).
"""
import ctypes
import subprocess

import torch

so = "/tmp/window_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/window_probe.hip"],
               check=True)
L = ctypes.CDLL(so)
L.window_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 400 * (1 << 20)  # elements (1.68 GB fp32), multiple of every window below
x = torch.randn(N, device=dev)
q = torch.empty(N // 4, dtype=torch.int32, device=dev)
part = torch.zeros(1024, device=dev)
flush = torch.empty(1 << 29, device=dev)
st = torch.cuda.current_stream().cuda_stream


def timed(fn, reps=5):
    best = 1e9
    for _ in range(reps):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


alg = 5 * N  # read 4N once + write 1N
# full passes: window = N means one read launch then one convert launch
t_full = timed(lambda: L.window_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, N, 0, 0, st))
print(f"two full passes      {t_full:.3f} ms  ({alg / t_full / 1e6:.0f} GB/s algorithmic)", flush=True)
t_conv = timed(lambda: L.window_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, N, 0, 2, st))
print(f"convert pass alone   {t_conv:.3f} ms  ({alg / t_conv / 1e6:.0f} GB/s algorithmic)", flush=True)
for mb_el in (4, 8, 16, 25, 40, 50, 80, 100):
    W = mb_el * (1 << 20)
    if N % W:
        continue
    for inter in (0, 1):
        t = timed(lambda: L.window_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, W, inter, 0, st))
        print(f"window {4 * mb_el:4d} MB inter={inter}  {t:.3f} ms  ({alg / t / 1e6:.0f} GB/s algorithmic)",
              flush=True)
