"""Top-K on exact-zero-heavy inputs: the zero-mode fast path (round 5).

The reference's default Top-K setup (``scheme: topk``, ``aggregate_payload: params``,
``/root/reference/conf/base.yaml:194-198``) has the PS re-encode, for every ``GetUpdatedModel``,
the average of the clients' zero-filled Top-K decodes (``global_grpc_server.py:147-171,
213-234``): at most C·k non-zeros per tensor.  With fewer than ~1.4 k non-zeros the sampled
threshold used to land in the zero bin and every element became a candidate (the radix-sort
fallback, ~25 ms on Llama-400M).  Zero mode takes every non-zero as a candidate and completes a
tensor with fewer than k of them by its lowest-index zeros (the exact tail's ``zero_fill_chunk``).  These tests
check that the fast path is taken (the plan's verdict counters) and that its bytes — values,
indices, error-feedback residual — equal the device-wide radix-sort fallback's, which the other
Top-K tests pin to ``torch.topk`` and the reference's goldens; and, on small cases, the oracle.
"""

import numpy as np
import pytest
import torch

import oracle
from omnifed_amd import codec

pytestmark = pytest.mark.gpu

SIZES = [3 << 20, 1000, 1_000_003, 70000, 5 << 20, 4096]


def _sparse_arena(plan, sizes, nnz_of_k, ratio, gen, neg_zero=True):
    """An arena whose tensor t holds round(nnz_of_k * k_t) non-zeros at random positions, the
    rest exact zeros (half of them -0.0 when neg_zero)."""
    x = torch.zeros(plan.arena_end, device="cuda")
    for o, n in zip(plan.offsets, sizes):
        k = oracle.topk_k(n, ratio)
        m = min(n, max(0, int(round(nnz_of_k * k))))
        seg = x[o:o + n]
        if neg_zero:
            neg = torch.rand(n, device="cuda", generator=gen) < 0.5
            seg[neg] = -0.0
        pos = torch.randperm(n, device="cuda", generator=gen)[:m]
        seg[pos] = torch.randn(m, device="cuda", generator=gen)
    return x


def _both(plan, x, ratio, residual0=None, mode=0, alpha=1.0):
    outs = []
    for fb in (0, 1):
        res = residual0.clone() if residual0 is not None else None
        plan.set_topk(fallback=fb)
        plan.topk_stats(reset=True)
        try:
            v, i, ks = plan.topk_encode(x, ratio, residual=res, residual_mode=mode, alpha=alpha)
            torch.cuda.synchronize()
        finally:
            plan.set_topk(fallback=0)
        outs.append((v, i, res, plan.topk_stats(reset=True)))
    return outs, ks


@pytest.mark.parametrize("nnz_of_k", [0.0, 0.5, 1.0, 1.2, 2.0])
@pytest.mark.parametrize("mode", [0, 1])
def test_zero_heavy_fast_path_equals_fallback(gpu, nnz_of_k, mode):
    """nnz ∈ {0, 0.5k, k, 1.2k, 2k} per tensor, ±0 zeros, alpha fused: no fallback, and values,
    indices and residual byte-equal to the forced radix-sort fallback."""
    ratio = 0.01
    plan = codec.Plan(SIZES, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(int(nnz_of_k * 10) + 100 * mode)
    x = _sparse_arena(plan, SIZES, nnz_of_k, ratio, g)
    r0 = _sparse_arena(plan, SIZES, nnz_of_k / 2, ratio, g) if mode == 1 else None
    (a, b), ks = _both(plan, x, ratio, residual0=r0, mode=mode, alpha=3.0)
    fast, slow = a[3], b[3]
    assert fast["calls"] == 1 and fast["fast"] == 1 and fast["fallback"] == 0, fast
    assert slow["fallback"] == 1, slow
    if nnz_of_k < 1.0:
        assert fast["zero_fill"] == 1, fast
    assert torch.equal(a[1], b[1]), "indices"
    assert a[0].cpu().numpy().tobytes() == b[0].cpu().numpy().tobytes(), "values (signed zeros included)"
    if mode:
        assert a[2].cpu().numpy().tobytes() == b[2].cpu().numpy().tobytes(), "residual"
    # the selection itself: every non-zero (or the largest k), then the lowest-index zeros
    K = 0
    for t, (o, n) in enumerate(zip(plan.offsets, SIZES)):
        k = ks[t]
        tp = x[o:o + n] * 3.0 + (r0[o:o + n] if mode else 0.0)
        want, _ = torch.topk(tp.abs(), k, sorted=True)
        assert torch.equal(a[0][K:K + k].abs(), want), t
        nz = int((tp != 0).sum())
        if nz < k:
            zi = a[1][K + nz:K + k].cpu().numpy()
            zeros = torch.nonzero(tp == 0).flatten()[: k - nz].cpu().numpy()
            assert np.array_equal(zi, zeros), t
        K += k


def test_zero_fill_matches_oracle_small(gpu):
    """Small tensors (the sample keeps every non-zero): the oracle's k largest magnitudes, values
    = t' at the indices (signed zeros), the residual = t' with the selection zeroed."""
    sizes = [5000, 300, 20000]
    plan = codec.Plan(sizes, device=gpu)
    xh = torch.zeros(plan.arena_end)
    rng = np.random.default_rng(7)
    for o, n in zip(plan.offsets, sizes):
        xh[o:o + n] = -0.0
        p = rng.choice(n, size=max(1, n // 400), replace=False)
        xh[o + p] = torch.from_numpy(rng.standard_normal(len(p)).astype(np.float32))
    res = torch.zeros(plan.arena_end, device=gpu)
    v, i, ks = plan.topk_encode(xh.to(gpu), 0.01, residual=res, residual_mode=2)
    st = plan.topk_stats()
    assert st["fallback"] == 0 and st["zero_fill"] >= 1, st
    K = 0
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        k = ks[t]
        tp = xh[o:o + n]
        ov, oi = oracle.topk_sparse(tp, 0.01)
        vh, ih = v[K:K + k].cpu(), i[K:K + k].cpu()
        assert torch.equal(torch.sort(vh.abs(), descending=True).values, torch.sort(ov.abs(), descending=True).values)
        assert vh.numpy().tobytes() == tp[ih].numpy().tobytes()  # -0.0 kept
        want_res = tp.clone()
        want_res[ih] = tp[ih] - tp[ih]
        assert res[o:o + n].cpu().numpy().tobytes() == want_res.numpy().tobytes()
        K += k


def test_ps_sparse_average_downlink(gpu):
    """The reference's steady state: two clients' error-feedback Top-K selections (overlapping and
    disjoint), zero-filled and summed on the PS, divided by the sample total, re-encoded by the
    PS's own Top-K compressor (mode 2, then mode 1 on the next round): fast path, and the bytes of
    the forced fallback."""
    sizes = [1 << 22, 65536, 3 << 20, 1000]
    plan = codec.Plan(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(3)
    ratio = 0.01
    base = torch.randn(plan.arena_end, device=gpu, generator=g)
    ps_res = torch.zeros(plan.arena_end, device=gpu)  # mode 2 writes it without reading it
    for rnd in range(2):
        acc = torch.zeros(plan.arena_end, device=gpu)
        for c in range(2):
            # overlap: client 1 sees client 0's gradient plus small noise (selections mostly agree)
            x = base + (0.05 * c) * torch.randn(plan.arena_end, device=gpu, generator=g)
            v, i, _ = plan.topk_encode(x, ratio)
            plan.topk_decode_arena(v, i, ratio, y=acc, mode=2)
        avg = acc / 2.0
        (a, b), ks = _both(plan, avg, ratio, residual0=ps_res, mode=2 if rnd == 0 else 1)
        nz = int((avg != 0).sum())
        assert nz < 2 * sum(ks), nz  # a sparse average (at most 2 k_t non-zeros per tensor)
        assert a[3]["fallback"] == 0 and a[3]["fast"] == 1, a[3]
        assert torch.equal(a[1], b[1]) and a[0].cpu().numpy().tobytes() == b[0].cpu().numpy().tobytes()
        assert a[2].cpu().numpy().tobytes() == b[2].cpu().numpy().tobytes()
        ps_res = a[2]
        base = torch.randn(plan.arena_end, device=gpu, generator=g)
