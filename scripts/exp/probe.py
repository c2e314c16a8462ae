"""Run the bandwidth probes + codec phase breakdown on the L400 arena (experiment)."""
import ctypes
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
so = "/tmp/bw_probe.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, "scripts/exp/bw_probe.hip"], check=True)
L = ctypes.CDLL(so)
L.probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
N = 401122304
a = torch.randn(N, device=dev)
b = torch.empty(N, device=dev)
st = torch.cuda.current_stream().cuda_stream
names = {0: ("copy", 8), 1: ("copy nt", 8), 2: ("read", 4), 3: ("write", 4), 4: ("write nt", 4),
         5: ("f32->i8", 5), 6: ("f32->i8 nt", 5), 7: ("i8->f32", 5), 8: ("i8->f32 nt", 5)}


def tm(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for grid in (2048,) if "--bw" in sys.argv else ():
    for w, (nm, bpe) in names.items():
        n4 = N // 4
        ms = tm(lambda: L.probe(w, a.data_ptr(), b.data_ptr(), n4, grid, st))
        print(f"grid {grid:6d} {nm:12s} {ms:.4f} ms  {bpe * N / ms / 1e6:7.1f} GB/s")

L.alu_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
if "--alu" in sys.argv:
    iters, grid = 4096, 2048
    for op, nm, per in ((0, "mad_u64_u32+xor", 2), (1, "mul_hi_u32+add", 2), (2, "xor,lshr,xor", 3), (3, "fma_f32", 1)):
        ms = tm(lambda: L.alu_probe(op, b.data_ptr(), iters, grid, st), reps=3)
        lane_ops = iters * 8 * grid * 256
        print(f"alu {nm:18s} {ms:.3f} ms  {lane_ops / ms / 1e9:8.1f} G elem-ops/s  ({per} instr each)")

from omnifed_amd import codec, shapes  # noqa: E402
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
for chunk in (65536,):
    p = codec.Plan.get(sizes, device=dev, chunk=chunk)
    x = torch.randn(p.arena_end, device=dev) * 1e-3
    q = torch.empty(p.arena_end, dtype=torch.int8, device=dev)
    y = torch.empty(p.arena_end, device=dev)
    nr = torch.empty(p.nt, device=dev)
    u = torch.rand(p.arena_end, device=dev)
    p.qsgd_norms(x, norm_out=nr)
    nin = nr.clone()
    print("resident capacity", p.resident_capacity, "items", p.encode_items)

    def enc(strategy, **kw):
        p.set_encode_strategy(strategy)
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, **kw)
        p.set_encode_strategy("resident")

    rows = {
        "encode (resident, philox)": (lambda: enc("resident", seed=1), 5),
        "encode (resident, u in)": (lambda: enc("resident", u=u), 9),
        "encode (ordered, philox)": (lambda: enc("ordered", seed=1), 5),
        "encode (ordered, u in)": (lambda: enc("ordered", u=u), 9),
        "norms only": (lambda: p.qsgd_norms(x, norm_out=nr), 4),
        "quant flat (norm in, philox)": (lambda: p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, norm_in=nin), 5),
        "quant flat (norm in, u in)": (lambda: p.qsgd_encode(x, 4, q_out=q, norm_out=nr, u=u, norm_in=nin), 9),
        "decode": (lambda: p.qsgd_decode(q, 8, 16, nr, y_out=y), 5),
        "decode accumulate": (lambda: p.qsgd_decode(q, 8, 16, nr, y_out=y, accumulate=True), 9),
    }
    for nm, (fn, bpe) in rows.items():
        ms = tm(fn)
        print(f"chunk {chunk:6d} {nm:30s} {ms:.4f} ms  {bpe * N / ms / 1e6:7.1f} GB/s (counting {bpe} B/elem)")
    print("co-resident:", p.check())
    # Top-K (k = 1 %) with error feedback over the whole arena
    res = torch.zeros(p.arena_end, device=dev)
    p.topk_encode(x, 0.01, residual=res, residual_mode=2)
    ms = tm(lambda: p.topk_encode(x, 0.01, residual=res, residual_mode=1), reps=5)
    print(f"topk encode (ratio 0.01, EF)      {ms:.4f} ms  {16.24 * N / ms / 1e6:7.1f} GB/s (algorithmic 16N+24k)")
    ms = tm(lambda: p.topk_encode(x, 0.01), reps=5)
    print(f"topk encode (ratio 0.01, no EF)   {ms:.4f} ms  {8.24 * N / ms / 1e6:7.1f} GB/s (algorithmic 8N+24k)")
