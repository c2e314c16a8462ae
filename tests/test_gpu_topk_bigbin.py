"""Top-K fine bins of more than kBucketHalf (2048) keys: a bucket of their own, no fallback.

The bucket sort orders a bucket of up to 4096 keys in LDS; buckets are the fine bins whose rank
starts fall in one 2048-wide window, so a fine bin of more than 2048 keys used to send the whole
call to the device-wide radix-sort fallback (the PS downlink's disjoint two-client
sparse average, one lm_head bin of 2 166 keys, took it on 4 of 10 calls).  Such a bin now gets a
bucket of its own (topk_scatter_planned); only a bin of more than 4096 keys — one magnitude shared
that widely, a cluster the fine bins cannot split — still takes the fallback.  Every case: the
bytes of the forced fallback (values, indices, residual), and with tie_order="torch" the oracle's
(torch.topk on the CPU)."""

import numpy as np
import pytest
import torch

import oracle
from omnifed_amd import codec, shapes

pytestmark = pytest.mark.gpu


def _both(plan, x, ratio, residual0=None, mode=0):
    outs = []
    for fb in (0, 1):
        res = residual0.clone() if residual0 is not None else None
        plan.set_topk(fallback=fb)
        plan.topk_stats(reset=True)
        try:
            v, i, ks = plan.topk_encode(x, ratio, residual=res, residual_mode=mode)
            torch.cuda.synchronize()
        finally:
            plan.set_topk(fallback=0)
        outs.append((v.clone(), i.clone(), res, plan.topk_stats(reset=True)))
    return outs, ks


def _clustered(n, cluster, value, distinct, seed):
    """N(0, 1) with `cluster` elements on (or within a few ulps of) `value`, both signs."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g)
    pos = torch.randperm(n, generator=g)[:cluster]
    v = torch.full((cluster,), value)
    if distinct:  # consecutive floats above value: one fine bin unless the sample saw the cluster
        v = (v.view(torch.int32) + torch.arange(cluster, dtype=torch.int32) % 97).view(torch.float32)
    sign = torch.where(torch.rand(cluster, generator=g) < 0.5, -1.0, 1.0)
    x[pos] = v * sign
    return x


@pytest.mark.parametrize("cluster,distinct,fallback", [(3000, False, 0), (3000, True, 0), (4000, False, 0),
                                                       (5000, False, 1)])
def test_big_fine_bin(gpu, cluster, distinct, fallback):
    sizes = [2 << 20, 70000, 1 << 20]
    plan = codec.Plan(sizes, device=gpu)
    xh = torch.zeros(plan.arena_end)
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        xh[o:o + n] = _clustered(n, cluster if t != 1 else 100, 3.0, distinct, 10 + t)
    x = xh.to(gpu)
    r0 = torch.randn(plan.arena_end, generator=torch.Generator().manual_seed(4)) * 0.1
    r0[(xh.abs() >= 3.0) & (xh.abs() < 3.001)] = 0.0  # t' = r0 + x keeps the clusters
    r0 = r0.to(gpu)
    (a, b), ks = _both(plan, x, 0.01, residual0=r0, mode=1)
    assert a[3]["fallback"] == fallback and a[3]["fast"] == 1 - fallback, a[3]
    assert b[3]["fallback"] == 1
    assert torch.equal(a[1], b[1]), "indices"
    assert a[0].cpu().numpy().tobytes() == b[0].cpu().numpy().tobytes(), "values"
    assert a[2].cpu().numpy().tobytes() == b[2].cpu().numpy().tobytes(), "residual"
    # the reference's bytes (ties: torch's CPU order)
    res = r0.clone()
    v, i, ks = plan.topk_encode(x, 0.01, residual=res, residual_mode=1, tie_order="torch")
    vh, ih, tp = v.cpu(), i.cpu(), (r0 + x).cpu()
    K = 0
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        k = ks[t]
        ov, oi = oracle.topk_sparse(tp[o:o + n], 0.01)
        assert ih[K:K + k].numpy().tobytes() == oi.numpy().tobytes(), t
        assert vh[K:K + k].numpy().tobytes() == ov.numpy().tobytes(), t
        K += k


def test_ps_disjoint_sparse_average_llama400m_no_fallback(gpu):
    """The PS downlink of the reference's Top-K round on Llama-400M (scheme topk, aggregate_payload
    params: global_grpc_server.py:147-171, 213-234): two clients with independent gradients and
    error feedback send their second call's selections, the PS sums the zero-filled decodes,
    halves them and re-encodes the sparse average with its own error feedback, ten requests: every
    call on the fast path (round 5: 4 of 10 fell back on a 2 166-key lm_head bin), and the first
    one byte-equal to the forced fallback."""
    named = shapes.model_shapes("llama400m")
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=gpu)
    ratio = 0.01
    g = torch.Generator(device=gpu).manual_seed(11)
    acc = torch.zeros(plan.arena_end, device=gpu)
    for c in range(2):
        res = torch.empty(plan.arena_end, device=gpu)
        for call in range(2):
            x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
            v, i, _ = plan.topk_encode(x, ratio, residual=res, residual_mode=2 if call == 0 else 1)
        plan.topk_decode_arena(v, i, ratio, y=acc, mode=2)
        del res, x
    avg = acc / 2.0
    del acc
    ps_res = torch.empty(plan.arena_end, device=gpu)
    (a, b), _ = _both(plan, avg, ratio, residual0=ps_res, mode=2)
    assert a[3]["fallback"] == 0, a[3]
    assert torch.equal(a[1], b[1]) and a[0].cpu().numpy().tobytes() == b[0].cpu().numpy().tobytes()
    assert a[2].cpu().numpy().tobytes() == b[2].cpu().numpy().tobytes()
    del b
    ps_res = a[2]
    plan.topk_stats(reset=True)
    for _ in range(10):
        plan.topk_encode(avg, ratio, residual=ps_res, residual_mode=1)
    st = plan.topk_stats(reset=True)
    assert st["calls"] == 10 and st["fallback"] == 0, st
