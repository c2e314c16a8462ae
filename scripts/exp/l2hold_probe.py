"""L2-hold probe (experiment): re-reading each chunk H chunk-steps after its first read, from the
same workgroup (same XCD L2).  Compare with H = 0 (one read per chunk) — see l2hold_probe.hip."""
import ctypes
import subprocess

import torch

so = "/tmp/l2hold_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/l2hold_probe.hip"],
               check=True)
L = ctypes.CDLL(so)
L.hold_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 400 * (1 << 20)
x = torch.randn(N, device=dev)
q = torch.empty(N // 4, dtype=torch.int32, device=dev)
part = torch.zeros(16, device=dev)
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


alg = 5 * N
for per in (4, 2, 1):
    for grid in (256, 512):
        for H in (0, 1, 2, 4, 8):
            t = timed(lambda: L.hold_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, H, grid, per, st))
            print(f"chunk {16 * per:3d} KiB grid {grid:4d} H={H}  {t:.3f} ms  ({alg / t / 1e6:.0f} GB/s algorithmic 5N)",
                  flush=True)
