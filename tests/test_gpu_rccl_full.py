"""The multi-GPU PS aggregates (omnifed_amd/ps.py) on the FULL Llama-400M arena over a real RCCL
group of world size 1 (round 4): the code bench.py's N > 1 leg runs — the RCCL gather of the
401 MB int8 payload, the RCCL reduce of the 1.6 GB fp32 arena, the all-gather / gather of the
48 MB Top-K selections — executed at the bench's size on the GPU, against the one-GPU
DeviceAggregator (bytes) and the oracle (global_grpc_server.py:147-171, torch_mpi.py:302-359,
core.py:62-71).  No scaling is claimed: the 8-GPU curve is the driver's."""

import numpy as np
import pytest
import torch

import oracle
from omnifed_amd import codec, shapes

pytestmark = pytest.mark.gpu

NAMED = shapes.model_shapes("llama400m")


@pytest.fixture(scope="module")
def l400(nccl1):
    gpu = nccl1
    sizes = [shapes.numel(s) for _, s in NAMED]
    plan = codec.Plan.get(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(1000)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    return gpu, plan, x


def _oracle_q(x_np, s, norm, u_np):
    q, *_ = oracle.qsgd_quantize(torch.from_numpy(np.ascontiguousarray(x_np)), s, norm=norm,
                                 u=torch.from_numpy(np.ascontiguousarray(u_np)))
    return q


@pytest.mark.parametrize("mode", ["gather", "reduce"])
def test_qsgd_weighted_round_full_llama400m(l400, mode):
    from omnifed_amd.ps import DeviceAggregator, GpuOps, qsgd_weighted_round, total_weight, weighted_sum_error_bound

    gpu, plan, x = l400
    ops = GpuOps(plan, seed=0x5EED)
    w = 3.0
    total = total_weight(w, gpu)
    s, call = 4, 9
    bufs = [(torch.empty(plan.payload_elems(8), dtype=torch.int8, device=gpu),
             torch.empty(plan.nt, dtype=torch.float32, device=gpu))]
    out = qsgd_weighted_round(x, w, total, ops, s, call, mode=mode, bufs=bufs)
    torch.cuda.synchronize()
    # the one-GPU drop-in aggregator with the same encode: bytes equal (gather: exact; reduce of
    # one rank: the same single term)
    q, norms = plan.qsgd_encode(x, s, alpha=w, seed=ops.key, offset=call)
    agg = DeviceAggregator(NAMED, device=gpu)
    assert agg.plan is plan
    plan.qsgd_decode(q, 8, 16, norms, y_out=agg.acc, accumulate=True)
    agg.total_samples = int(w)
    avg = agg.apply()
    oh = out.cpu().numpy()
    for (name, _), o, n in zip(NAMED, plan.offsets, plan.sizes):
        assert avg[name].cpu().numpy().reshape(-1).tobytes() == oh[o:o + n].tobytes(), name
    # oracle on sampled tensors (the vocabulary matrices included): levels, decode, / total
    xh, qh, nh = x.cpu().numpy(), q.cpu().numpy(), norms.cpu().numpy()
    for t in (0, 1, 91, len(NAMED) - 2, len(NAMED) - 1):
        o, n = plan.offsets[t], plan.sizes[t]
        xw = (xh[o:o + n] * np.float32(w)).astype(np.float32)
        want_q = _oracle_q(xw, s, float(nh[t]), oracle.philox_uniforms(ops.key, call, t, n))
        assert qh[o:o + n].tobytes() == want_q.numpy().tobytes(), t
        dec = oracle.qsgd_dequantize(want_q, float(nh[t]), 16, (n,))
        want = (dec / np.float32(total)).numpy()
        got = oh[o:o + n]
        if mode == "gather":
            assert got.tobytes() == want.tobytes(), t
        bound = weighted_sum_error_bound(dec.double().abs(), torch.from_numpy(want).double(), 1, total).numpy()
        assert np.all(np.abs(got.astype(np.float64) - want.astype(np.float64)) <= bound), t


@pytest.mark.parametrize("dst", [None, 0])
def test_topk_sparse_aggregate_full_llama400m(l400, dst):
    """All-gather (or gather to the root) of one client's whole L400 selection (k = 1 %,
    error feedback, weighting fused), scatter-add, / client count: every tensor equals the
    oracle's layerwise_decompress of that selection, bit for bit."""
    from omnifed_amd.ps import GpuOps, topk_sparse_aggregate

    gpu, plan, x = l400
    ratio = 0.01
    res = torch.zeros(plan.arena_end, device=gpu)
    vals, idx, ks = plan.topk_encode(x, ratio, residual=res, residual_mode=2, alpha=2.0)
    ops = GpuOps(plan)
    acc = torch.empty(plan.arena_end, device=gpu)
    out = topk_sparse_aggregate(vals, idx, ratio, acc, ops, client_count=1, dst=dst)
    torch.cuda.synchronize()
    vh, ih, oh = vals.cpu(), idx.cpu(), out.cpu()
    K = 0
    for t, (o, n, k) in enumerate(zip(plan.offsets, plan.sizes, ks)):
        want = oracle.layerwise_decompress([vh[K:K + k]], [ih[K:K + k]], (n,), 1)
        assert oh[o:o + n].numpy().tobytes() == want.reshape(-1).numpy().tobytes(), t
        K += k
