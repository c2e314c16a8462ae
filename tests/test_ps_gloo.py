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
        if y is None:
            return yy.clone()
        if accumulate:
            y += yy
        else:
            y.copy_(yy)
        return y

    def div_(self, y, d):
        y /= d
        return y


def _assert_within_bound(got, terms, total):
    """|reduce/total - exact/total| <= ps.weighted_sum_error_bound (fp64 exact sum)."""
    from omnifed_amd.ps import weighted_sum_error_bound

    t64 = torch.stack([t.double() for t in terms])
    exact = t64.sum(0) / float(total)
    bound = weighted_sum_error_bound(t64.abs().sum(0), exact, len(terms), total)
    err = (torch.from_numpy(np.array(got, np.float32)).double() - exact).abs()
    assert bool((err <= bound).all()), float((err - bound).max())


def test_error_bound_covers_every_summation_order():
    """weighted_sum_error_bound holds for 8 fp32 terms summed in many orders (sequential in
    random permutations and pairwise trees), as an 8-rank RCCL reduce may sum them."""
    from omnifed_amd.ps import weighted_sum_error_bound

    g = torch.Generator().manual_seed(3)
    terms = [torch.randn(20000, generator=g) * (10.0 ** (i % 4 - 2)) for i in range(8)]
    terms[3][:100] = -terms[2][:100]  # cancellation
    t64 = torch.stack([t.double() for t in terms])
    total = 37.0
    exact = t64.sum(0) / total
    bound = weighted_sum_error_bound(t64.abs().sum(0), exact, 8, total)
    orders = [torch.randperm(8, generator=g).tolist() for _ in range(20)]
    for order in orders:
        acc = torch.zeros(20000)
        for i in order:
            acc = acc + terms[i]
        got = acc / np.float32(total)
        assert bool(((got.double() - exact).abs() <= bound).all())
    pair = list(terms)
    while len(pair) > 1:  # a tree (reduce-scatter style)
        pair = [pair[i] + pair[i + 1] for i in range(0, len(pair), 2)]
    assert bool(((pair[0] / np.float32(total)).double() - exact).abs().le(bound).all())


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


@pytest.mark.parametrize("world", [2, 4, 8])  # 8: the driver's largest node, rehearsed on gloo
@pytest.mark.parametrize("mode", ["reduce", "gather"])
def test_weighted_sum_world2(mode, world):
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
    else:  # the reduce order belongs to the collective: the any-order fp64 bound
        _assert_within_bound(got, dec, sum(range(1, world + 1)))


# ---------------------------------------------------------------- weighted round (alpha) and Top-K

class WeightedOracleOps(OracleOps):
    """Client encode with the weighting applied first (torch.mul(x, w), global_grpc.py:104) and
    the reference MT19937 stream: the oracle of GpuOps.encode's fused alpha."""

    def __init__(self, seed):
        self.seed = seed

    def encode(self, x, bit_width, alpha, call, q=None, norms=None):
        xw = torch.mul(x, alpha)
        u = torch.from_numpy(oracle.mt19937_uniforms(self.seed + call, x.numel()))
        q, norm, width, levels = oracle.qsgd_quantize(xw, bit_width, u=u)
        return q, torch.tensor([norm], dtype=torch.float32)


def _weighted_worker(rank, world, port, mode, q_out):
    from omnifed_amd.ps import qsgd_weighted_round, total_weight

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(200 + rank)
        x = torch.randn(3000) * 1e-2
        w = 10.0 * (rank + 1) + 7
        total = total_weight(w, "cpu")
        out = qsgd_weighted_round(x, w, total, WeightedOracleOps(50 + rank), 4, call=3, mode=mode)
        if rank == 0:
            q_out.put((out.numpy().tobytes(), total))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode", ["gather", "reduce"])
def test_weighted_round_world2(mode, world):
    """Σ_i decode(Q(w_i·x_i)) / Σ_i w_i over two, four and eight ranks, the weights applied before
    encoding: gather mode bit-exact in rank order, reduce mode within the any-order fp64 bound."""
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_weighted_worker, args=(r, world, port, mode, qq)) for r in range(world)]
    for p in procs:
        p.start()
    raw, total = qq.get(timeout=120)
    got = np.frombuffer(raw, dtype=np.float32)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ws = [10.0 * (r + 1) + 7 for r in range(world)]
    assert total == sum(ws)
    dec = []
    for r in range(world):
        torch.manual_seed(200 + r)
        x = torch.randn(3000) * 1e-2
        q, norm = WeightedOracleOps(50 + r).encode(x, 4, ws[r], 3)
        dec.append(oracle.qsgd_dequantize(q, float(norm[0]), 16, (3000,)))
    want = oracle.ps_aggregate(dec, sum(ws)).numpy()
    if mode == "gather":
        assert got.tobytes() == want.tobytes()
    else:
        _assert_within_bound(got, dec, sum(ws))


class TopKOracleOps(OracleOps):
    """Arena scatter-add of one client's packed selection (omf_topk_decode_arena's oracle)."""

    def __init__(self, sizes):
        from omnifed_amd.codec import arena_layout

        self.sizes = sizes
        self.offsets, self.end = arena_layout(sizes)

    def topk_decode(self, values, indices, ratio, y, mode):
        k0 = 0
        for o, n in zip(self.offsets, self.sizes):
            k = oracle.topk_k(n, ratio)
            seg = y[o:o + n]
            seg.data[indices[k0:k0 + k]] += values[k0:k0 + k]  # core.py:67
            k0 += k
        return y


def _lwd_case(cid):
    g2 = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_r2.npz"))
    import json

    with open(os.path.join(os.path.dirname(__file__), "golden", "golden_r2_index.json")) as f:
        case = json.load(f)["lwd"][cid]
    return g2, case


def _topk_worker(rank, world, port, dst, q_out):
    from omnifed_amd.ps import topk_sparse_aggregate

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g2, case = _lwd_case(0)
        nt = len(case["shapes"])
        sizes = [int(np.prod(s)) for s in case["shapes"]]
        vals = torch.from_numpy(np.concatenate([g2[f"lwd/0/vals/{rank}/{t}"] for t in range(nt)]))
        idx = torch.from_numpy(np.concatenate([g2[f"lwd/0/idx/{rank}/{t}"] for t in range(nt)]))
        ops = TopKOracleOps(sizes)
        acc = torch.empty(ops.end)
        out = topk_sparse_aggregate(vals, idx, case["ratio"], acc, ops, dst=dst)
        if dst is None or rank == dst:
            q_out.put((rank, out.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dst", [None, 0])
def test_topk_sparse_aggregate_world2(dst):
    """Multi-GPU Top-K (all-gather or gather to a root, rank-order scatter-add, / world) equals the
    reference's layerwise_decompress over the reference TopKCompression selections, bit for bit."""
    world = 2
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_topk_worker, args=(r, world, port, dst, qq)) for r in range(world)]
    for p in procs:
        p.start()
    results = [qq.get(timeout=120) for _ in range(world if dst is None else 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g2, case = _lwd_case(0)
    from omnifed_amd.codec import arena_layout

    sizes = [int(np.prod(s)) for s in case["shapes"]]
    offs, _ = arena_layout(sizes)
    for _, raw in results:
        got = np.frombuffer(raw, dtype=np.float32)
        for t, (o, n) in enumerate(zip(offs, sizes)):
            assert got[o:o + n].tobytes() == g2[f"lwd/0/out/{t}"].tobytes(), t
