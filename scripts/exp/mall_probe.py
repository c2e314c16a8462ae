"""Does the 256 MiB Infinity Cache serve a re-read? cold vs warm read passes over S bytes (experiment)."""
import ctypes
import sys

import torch

so = "/tmp/bw_probe.so"
import subprocess
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/bw_probe.hip"], check=True)
L = ctypes.CDLL(so)
L.probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
big = torch.randn(1 << 29, device=dev)  # 2 GiB flush buffer
out = torch.empty(16, device=dev)
st = torch.cuda.current_stream().cuda_stream


def read(t, grid=4096):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    L.probe(2, t.data_ptr(), out.data_ptr(), t.numel() // 4, grid, st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


for mb in (16, 64, 128, 192, 240, 320, 512):
    t = torch.randn(mb * (1 << 20) // 4, device=dev)
    res = []
    for rep in range(3):
        read(big)
        c = read(t)
        w1 = read(t)
        w2 = read(t)
        res.append((c, w1, w2))
    c, w1, w2 = [min(r[i] for r in res) for i in range(3)]
    B = t.numel() * 4
    print(f"{mb:4d} MB  cold {B / c / 1e6:7.0f} GB/s  warm {B / w1 / 1e6:7.0f} GB/s  warm2 {B / w2 / 1e6:7.0f} GB/s")
    del t
