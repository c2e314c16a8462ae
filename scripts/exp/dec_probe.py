"""Decoder / encoder streaming-shape probe (experiment; see dec_probe.hip)."""
import ctypes
import subprocess

import torch

so = "/tmp/dec_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/dec_probe.hip"],
               check=True)
L = ctypes.CDLL(so)
L.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 401122304
q = torch.randint(-8, 8, (N // 4,), dtype=torch.int32, device=dev)
y = torch.randn(N, device=dev)
flush = torch.empty(1 << 29, device=dev)
st = torch.cuda.current_stream().cuda_stream


def timed(fn, reps=7):
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


names = {0: "dec U1 ntS", 1: "dec U1 ntL ntS", 2: "dec U4 ntS", 3: "dec U4 ntL ntS", 4: "dec vec16 ntS",
         5: "dec vec16 ntL ntS", 6: "dec U1 ntL", 7: "dec U1 plain",
         10: "enc U1 plain", 11: "enc U1 ntL", 12: "enc U1 ntL ntS", 13: "enc U4 ntL ntS", 14: "enc U2 ntL ntS",
         15: "enc U1 ntS"}
for v, nm in names.items():
    t = timed(lambda: L.probe_run(v, q.data_ptr(), y.data_ptr(), N, st))
    print(f"{nm:22s}: {t:.3f} ms  {5 * N / t / 1e6:.0f} GB/s (5 B/elem)", flush=True)
