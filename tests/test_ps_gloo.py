"""World-size-2 gloo tests (CPU) of the multi-GPU PS weighted sum orchestration (omnifed_amd/ps.py).

The collectives and their ordering are exercised with gloo on CPU; the device decode /
divide steps are supplied by the CPU oracle here (on the GPU box they are the HIP
kernels, covered by tests/test_gpu_*).  Expected results follow the reference PS:
sum of decoded client updates (arrival = rank order) divided by total samples
(global_grpc_server.py:147-171).
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from omnifed_amd.ps import weighted_sum_gather, weighted_sum_reduce


class OracleOps:
    def decode(self, q, width, levels, norms, y, accumulate):
        # one tensor arena: the whole buffer is tensor 0
        yy = oracle.qsgd_dequantize(q, float(norms[0]), levels, (q.numel(),))
        if accumulate:
            y += yy
        else:
            y.copy_(yy)
        return y

    def div_(self, y, d):
        y /= d
        return y


def _client(rank, n=1000, s=4):
    torch.manual_seed(100 + rank)
    x = torch.randn(n) * 1e-2 * (rank + 1)
    q, norm, width, levels = oracle.qsgd_quantize(x, s, u=torch.from_numpy(oracle.mt19937_uniforms(7 + rank, n)))
    return q, torch.tensor([norm], dtype=torch.float32), width, levels


def _worker(rank, world, port, mode, q_out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q, norm, width, levels = _client(rank)
        total = float(sum(range(1, world + 1)))
        ops = OracleOps()
        if mode == "reduce":
            y = oracle.qsgd_dequantize(q, float(norm[0]), levels, (q.numel(),)).clone()
            out = weighted_sum_reduce(y, total, ops)
        else:
            acc = torch.empty(q.numel())
            out = weighted_sum_gather(q, norm, width, levels, acc, total, ops)
        if rank == 0:
            q_out.put(out.numpy().tobytes())
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["reduce", "gather"])
def test_weighted_sum_world2(mode):
    world = 2
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, qq)) for r in range(world)]
    for p in procs:
        p.start()
    got = np.frombuffer(qq.get(timeout=120), dtype=np.float32)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dec = []
    for r in range(world):
        q, norm, width, levels = _client(r)
        dec.append(oracle.qsgd_dequantize(q, float(norm[0]), levels, (q.numel(),)))
    want = oracle.ps_aggregate(dec, sum(range(1, world + 1))).numpy()
    if mode == "gather":  # deterministic rank-order sum: bit-exact
        assert got.tobytes() == want.tobytes()
    else:  # reduce order belongs to the collective: fp32 sum of 2 terms is exact-order independent
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-9)
