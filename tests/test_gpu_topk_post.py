"""The Top-K fast path's post-pass after round 5's LDS changes (*post-pass, round 5*).

``topk_bucket_scatter`` now stages the tensor's bucket table in LDS when every tensor of the launch
has <= 4096 bucket slots, and keeps each thread's first keys in registers between its two phases;
``topk_bucket_sort`` places a key's sub-bin by an LDS histogram of the bucket's own |t'| range
instead of the fine bins.  The order — and so the bytes — must not change: these tests drive
distributions that stress the new sub-bin rule (heavy tails, a lone outlier stretching the top
bucket's range, narrow spikes, subnormal magnitudes, long runs of equal magnitudes) and a k large
enough for the global-table scatter, and check the fast path (asserted by the plan's verdict
counters where it must be taken) against the device-wide radix-sort fallback and ``torch.topk``.
"""

import pytest
import torch

from omnifed_amd import codec

pytestmark = pytest.mark.gpu


def _both_paths(plan, x, ratio, residual0=None, mode=0, alpha=1.0):
    """(fast, fallback) outputs of one encode each on the same input, and the fast call's counters."""
    outs, stats = [], None
    for fb in (0, 1):
        res = residual0.clone() if residual0 is not None else None
        plan.set_topk(fallback=fb)
        plan.topk_stats(reset=True)
        try:
            v, i, ks = plan.topk_encode(x, ratio, residual=res, residual_mode=mode, alpha=alpha)
            torch.cuda.synchronize()
        finally:
            plan.set_topk(fallback=0)
        if fb == 0:
            stats = plan.topk_stats(reset=True)
        outs.append((v, i, res))
    return outs, ks, stats


def _check_against_torch(plan, sizes, tp, vals, idx, ks):
    K = 0
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        seg = tp[o:o + n]
        want, _ = torch.topk(seg.abs(), ks[t], sorted=True)
        got = vals[K:K + ks[t]]
        assert torch.equal(got.abs(), want), t
        assert torch.equal(got, seg[idx[K:K + ks[t]]]), t
        m = got.abs()
        same = m[:-1] == m[1:]
        ii = idx[K:K + ks[t]]
        assert bool(torch.all(ii[:-1][same] < ii[1:][same])), t  # ties: ascending index
        K += ks[t]


def _arena(plan, sizes, fill):
    x = torch.zeros(plan.arena_end, device="cuda")
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        x[o:o + n] = fill(t, n)
    return x


@pytest.mark.parametrize("dist", ["cauchy", "outlier", "spike", "subnormal", "runs"])
def test_post_pass_distributions_fast_equals_fallback(gpu, dist):
    sizes = [2 << 20, 1_000_003, 70000, 4096, 3 << 20]
    plan = codec.Plan(sizes, device=gpu)
    seed = {"cauchy": 1, "outlier": 2, "spike": 3, "subnormal": 4, "runs": 5}[dist]
    g = torch.Generator(device=gpu).manual_seed(seed)

    def fill(t, n):
        z = torch.randn(n, device=gpu, generator=g)
        if dist == "cauchy":  # heavy tail: each top bucket spans decades of |t'|
            return torch.tan((torch.rand(n, device=gpu, generator=g) - 0.5) * 3.14159)
        if dist == "outlier":  # one huge value: the top bucket's |t'| range is all outlier
            z[n // 3] = 3e30
            return z
        if dist == "spike":  # a narrow cluster of |t'| just around the k-th magnitude
            k = max(1, int(n * 0.01))
            kth = torch.topk(z.abs(), k).values[-1]
            pick = torch.rand(n, device=gpu, generator=g) < 0.004
            z[pick] = torch.sign(z[pick]) * kth * (1 + 1e-6 * torch.rand(int(pick.sum()), device=gpu, generator=g))
            return z
        if dist == "subnormal":  # every magnitude below 2^-126
            return z * 1e-39
        # runs: magnitudes repeated 40 times (ties within buckets, some sub-bins over the
        # insertion limit -> the bitonic path), random signs and positions
        lv = torch.rand(n // 40 + 1, device=gpu, generator=g) + 1.0
        v = lv.repeat_interleave(40)[:n]
        return v[torch.randperm(n, device=gpu, generator=g)] * torch.where(
            torch.rand(n, device=gpu, generator=g) < 0.5, -1.0, 1.0)

    x = _arena(plan, sizes, fill)
    r0 = torch.zeros(plan.arena_end, device=gpu)
    (a, b), ks, st = _both_paths(plan, x, 0.01, residual0=r0, mode=1)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2]), dist
    _check_against_torch(plan, sizes, x, a[0], a[1], ks)
    if dist in ("cauchy", "outlier", "subnormal"):
        assert st["fast"] == 1 and st["fallback"] == 0, st


def test_post_pass_large_k_global_bucket_table(gpu):
    """k over 8 Mi in one tensor (more than 4096 bucket slots): the scatter reads the plan's global
    bucket table (the LDS-staged one holds 4096), with error feedback; bytes equal the fallback's."""
    sizes = [12 << 20, 1 << 20]
    ratio = 0.75  # k = 9.4 M in the first tensor -> ~4600 bucket slots
    plan = codec.Plan(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(5)
    x = torch.randn(plan.arena_end, device=gpu, generator=g)
    r0 = torch.randn(plan.arena_end, device=gpu, generator=g) * 0.25
    (a, b), ks, st = _both_paths(plan, x, ratio, residual0=r0, mode=1, alpha=0.5)
    assert ks[0] > 8 << 20
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    assert st["fast"] == 1 and st["fallback"] == 0, st
    tp = r0 + x * 0.5
    _check_against_torch(plan, sizes, tp, a[0], a[1], ks)
