"""Cache-policy probe for a two-pass read (experiment; see policy_probe.hip)."""
import ctypes
import subprocess

import torch

so = "/tmp/policy_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/policy_probe.hip"],
               check=True)
L = ctypes.CDLL(so)
L.probe_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 400 * (1 << 20)
x = torch.randn(N, device=dev)
q = torch.empty(N // 4, dtype=torch.int32, device=dev)
part = torch.zeros(16, device=dev)
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


W = 32 * (1 << 20)  # 128 MB windows
for pa in (0, 1, 2, 3, 16):
    ta = timed(lambda: L.probe_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, N, pa, 0, 1, st))
    for pb in (0, 2):
        tw = timed(lambda: L.probe_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, W, pa, pb, 0, st))
        tf = timed(lambda: L.probe_run(x.data_ptr(), q.data_ptr(), part.data_ptr(), N, N, pa, pb, 0, st))
        print(f"A aux {pa:2d} alone {ta:.3f} | B aux {pb}: windowed 128MB {tw:.3f}  full passes {tf:.3f} ms", flush=True)
