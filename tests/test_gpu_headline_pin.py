"""The bench's headline arenas pinned to the oracle directly, tensor by tensor (round 4).

bench.py encodes one client's Llama-400M update (N(0,1)·1e-3, generator seed 1000 + rank) at
s = 4 with on-device Philox draws and the client weighting fused as alpha, through the
bracketed single-read encoder.  Here EVERY tensor of that arena — and of Llama-400M at s = 3
with alpha = 3, and of Llama-150M at s = 4 — is compared with ``oracle.qsgd_quantize``
(qsgd.py:36-64 restated) given the GPU's norm and ``oracle.philox_uniforms``: payload bytes
equal, and the decode equal to ``oracle.qsgd_dequantize``.  The bracketed encoder's finish
pass (the undecided quads it lists and fixes) must have run: spec_stats()["listed"] > 0.

Round 5 adds the int32 wire (``bit_width: 8``, the reference's default, conf/base.yaml:200;
qsgd.py:18-21 stores levels > 127 as int32): on these plans an s = 8 encode takes the bracketed
encoder with its wide-level undecided list (asserted through the plan's record of the encoder it
launched; the fix pass must have run), Llama-400M (alpha 1) and Llama-150M (alpha 2), every tensor;
and test_wide_levels_bracket_equals_ring pins the wide path against the ring at s = 5-8.
"""

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

import oracle
from omnifed_amd import codec, shapes

pytestmark = pytest.mark.gpu


def _threads() -> int:
    import os

    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:  # pragma: no cover
        return 8


@pytest.mark.parametrize("cfg,s,alpha", [("llama400m", 4, 1.0), ("llama400m", 3, 3.0), ("llama150m", 4, 1.0),
                                         ("llama400m", 8, 1.0), ("llama150m", 8, 2.0)])
def test_headline_arena_every_tensor_equals_oracle(gpu, cfg, s, alpha):
    named = shapes.model_shapes(cfg)
    sizes = [shapes.numel(sh) for _, sh in named]
    plan = codec.Plan.get(sizes, device=gpu)
    assert plan.strategy == "bracket"  # the default encoder of these arenas (bench.py's)
    g = torch.Generator(device=gpu)
    g.manual_seed(1000)  # bench.py's rank-0 client
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    seed, off = 0x5EED, 7
    q, norms = plan.qsgd_encode(x, s, alpha=alpha, seed=seed, offset=off)
    width = codec.storage_width(2**s)
    assert plan.last_encoder == "bracket"
    stats = plan.spec_stats()
    assert stats["listed"] > 0, stats  # the finish pass fixed undecided quads
    assert stats["whole"] == 0, stats  # no tensor needed the whole-tensor requantisation
    if s >= 7:
        assert width == 32 and q.dtype == torch.int32  # the int32 wire
    plan.check()
    L = 2**s
    y = plan.qsgd_decode(q, width, L, norms)
    xh = x.cpu().numpy()
    qh = q.cpu().numpy()
    yh = y.cpu().numpy()
    nh = norms.cpu().numpy()
    xs_all = xh if alpha == 1.0 else (xh * np.float32(alpha)).astype(np.float32)  # torch.mul(param, batch_samples)

    def check(t):
        o, n = plan.offsets[t], sizes[t]
        xs = xs_all[o:o + n]
        ref = float(np.sqrt(np.sum(xs.astype(np.float64) ** 2)))
        if abs(float(nh[t]) - ref) > 2e-6 * ref:
            return f"tensor {t}: norm {nh[t]} vs fp64 {ref}"
        u = torch.from_numpy(oracle.philox_uniforms(seed, off, t, n))
        want, _, _, _ = oracle.qsgd_quantize(torch.from_numpy(xs), s, norm=float(nh[t]), u=u)
        if qh[o:o + n].tobytes() != want.numpy().tobytes():
            bad = np.flatnonzero(qh[o:o + n] != want.numpy())
            return f"tensor {t}: {bad.size} levels differ, first at {bad[:4].tolist()}"
        want_y = oracle.qsgd_dequantize(want, float(nh[t]), L, (n,)).numpy()
        if yh[o:o + n].tobytes() != want_y.tobytes():
            return f"tensor {t}: decode differs"
        return None

    with ThreadPoolExecutor(_threads()) as ex:
        errors = [e for e in ex.map(check, range(len(sizes))) if e]
    assert not errors, errors[:5]


@pytest.mark.parametrize("s", [5, 6, 7, 8])
def test_wide_levels_against_the_oracle(gpu, s):
    """Bit widths 5-8 through the bracketed encoder's wide-level list, weighted, and the fused PS
    step at the same widths: every tensor's levels equal the oracle's given the GPU norm and draws
    (the fix pass ran: listed > 0), and the average is numpy's fp32 division."""
    sizes = [5, 16384, 70001] + [1 << 20] * 4 + [4 << 20] * 4 + [3000, 2_000_000, 8 << 20]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy("bracket")  # 30 M elements: below the default crossover
    g = torch.Generator(device=gpu)
    g.manual_seed(77 + s)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    L = 2**s
    seed, off = 9, 4
    q, norms = plan.qsgd_encode(x, s, alpha=2.0, seed=seed, offset=off)
    assert plan.last_encoder == "bracket"
    stats = plan.spec_stats()
    # the fix pass ran; a mid-size tensor (70 001 elements) may overflow its wave lists at s = 8 and be
    # requantised whole (exact, and cheap at that size) — the large ones never are
    assert stats["listed"] > 0 and stats["whole"] <= 1, stats
    avg, qa, na = plan.ps_apply_encode(x, 3.0, s, seed=seed, offset=off + 1)
    assert plan.last_encoder == "bracket"
    plan.check()
    xh = x.cpu().numpy()
    xs_all = (xh * np.float32(2.0)).astype(np.float32)
    av_all = xh / np.float32(3.0)
    qh, nh, qah, nah, ah = q.cpu().numpy(), norms.cpu().numpy(), qa.cpu().numpy(), na.cpu().numpy(), avg.cpu().numpy()

    def check(t):
        o, n = plan.offsets[t], sizes[t]
        for src, qq, nn, off_ in ((xs_all, qh, nh, off), (av_all, qah, nah, off + 1)):
            xs = src[o:o + n]
            ref = float(np.sqrt(np.sum(xs.astype(np.float64) ** 2)))
            if abs(float(nn[t]) - ref) > 2e-6 * ref:
                return f"tensor {t}: norm {nn[t]} vs fp64 {ref}"
            u = torch.from_numpy(oracle.philox_uniforms(seed, off_, t, n))
            want, _, _, _ = oracle.qsgd_quantize(torch.from_numpy(xs), s, norm=float(nn[t]), u=u)
            if qq[o:o + n].tobytes() != want.numpy().tobytes():
                bad = np.flatnonzero(qq[o:o + n] != want.numpy())
                return f"tensor {t}: {bad.size} levels differ, first at {bad[:4].tolist()}"
        if ah[o:o + n].tobytes() != av_all[o:o + n].tobytes():
            return f"tensor {t}: average differs"
        return None

    assert L > 16
    with ThreadPoolExecutor(_threads()) as ex:
        errors = [e for e in ex.map(check, range(len(sizes))) if e]
    assert not errors, errors[:5]


@pytest.mark.parametrize("cfg", ["llama400m", "llama150m"])
def test_fused_bracket_equals_bracket_launch(gpu, cfg):
    """The bracket folded into the pass (omf_plan_set_fused_bracket: its first workgroups sample, the
    pass's blocks poll for their tensor's bracket) writes the payload, norms and — for the fused PS
    step — the average of the separate bracket launch, bit for bit (weighted, s = 3 and 4; and the
    wide levels' one-wave version, s = 6 (int8 wire) and 8 (int32 wire), whose sixteen parts sum the
    sample in another grouping: its bracket may list other quads, the payload is exact either way)."""
    named = shapes.model_shapes(cfg)
    sizes = [shapes.numel(sh) for _, sh in named]
    plan = codec.Plan(sizes, device=gpu)
    assert plan.strategy == "bracket"
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    for s in (3, 4, 6, 8):
        outs = []
        for fb in (False, True):
            plan.set_fused_bracket(fb)
            q, n = plan.qsgd_encode(x, s, alpha=2.0, seed=3, offset=s)
            st = plan.spec_stats()
            avg, qa, na = plan.ps_apply_encode(x, 7.0, s, seed=3, offset=10 + s)
            plan.check()
            outs.append((q, n, avg, qa, na, st))
        plan.set_fused_bracket(False)
        (q1, n1, a1, qa1, na1, st1), (q2, n2, a2, qa2, na2, st2) = outs
        assert st2["whole"] == 0 and st2["listed"] > 0, st2
        assert torch.equal(n1, n2) and torch.equal(na1, na2)
        for o, k in zip(plan.offsets, sizes):
            assert torch.equal(q1[o:o + k], q2[o:o + k]) and torch.equal(qa1[o:o + k], qa2[o:o + k])
            assert torch.equal(a1[o:o + k], a2[o:o + k])
