"""Read-only streaming shapes (experiment; see read_probe.hip)."""
import ctypes
import subprocess

import torch

so = "/tmp/read_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/read_probe.hip"],
               check=True)
L = ctypes.CDLL(so)
L.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 401122304
x = torch.randn(N, device=dev)
part = torch.zeros(16, device=dev)
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


names = ["U1 B256", "U2 B256", "U4 B256", "U8 B256", "U16 B256", "U1 B256 nt", "U4 B256 nt", "U16 B256 nt",
         "U4 B512", "U4 B1024"]
for v, nm in enumerate(names):
    t = timed(lambda: L.probe_run(v, x.data_ptr(), part.data_ptr(), N, st))
    print(f"{nm:14s}: {t:.3f} ms  {4 * N / t / 1e6:.0f} GB/s", flush=True)
