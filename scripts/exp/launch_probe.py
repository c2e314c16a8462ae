"""Cost of a small dependent launch after a streaming pass (experiment; launch_probe.hip)."""
import ctypes
import subprocess

import torch

so = "/tmp/launch_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                "scripts/exp/launch_probe.hip"], check=True)
L = ctypes.CDLL(so)
L.probe_run.argtypes = [ctypes.c_int, ctypes.c_int64] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + [ctypes.c_void_p] * 4
dev = torch.device("cuda", 0)
N = 400 * (1 << 20)
x = torch.randn(N, device=dev)
q = torch.empty(N // 4, dtype=torch.int32, device=dev)
a = torch.randint(0, 1 << 20, (4 << 20,), dtype=torch.int32, device=dev)
b = torch.randint(0, 1 << 20, (1 << 20,), dtype=torch.int32, device=dev)
out = torch.zeros(4 << 20, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream


def run(mode, wgs):
    L.probe_run(mode, wgs, x.data_ptr(), q.data_ptr(), N // 4, a.data_ptr(), b.data_ptr(), out.data_ptr(), st)


cases = [(0, 0), (1, 1), (1, 1536), (1, 12288), (2, 1536), (2, 12288), (3, 1536), (3, 12288)]
res = {c: [] for c in cases}
for rnd in range(7):
    for c in cases:
        run(*c)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run(*c)
        e1.record()
        torch.cuda.synchronize()
        res[c].append(e0.elapsed_time(e1) / 20)
base = sorted(res[(0, 0)])[3]
for c in cases:
    v = sorted(res[c])[3]
    print(f"mode {c[0]} wgs {c[1]:6d}: {v:.4f} ms  (+{(v - base) * 1e3:.1f} us)", flush=True)
