"""The bracketed single-read encoder on bf16 / fp16 tensors (round 4), pinned to the oracle tensor
by tensor.  The reference quantises in the tensor's dtype (qsgd.py:36-64: torch.mul(param,
batch_samples), v / norm and the norm itself rounded to bf16 / fp16; the fraction promoted to
fp32); the encoder decides every level that is the same for all norms of its bracket with the
format's rounding folded into the bracket's multipliers (and fp16's subnormal quotients into an
absolute slack), and fixes the rest exactly.  The arena mixes tensors read whole by the bracket
and sampled ones; at 1e-3 scale a quarter of the fp16 quotients are subnormal."""

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

import oracle
from omnifed_amd import codec

pytestmark = pytest.mark.gpu

SIZES = [3, 1000, 16384, 16385, 70001, 1 << 20, 4 << 20, 28 << 20]  # >= 2^25: the bracket's arenas


@pytest.mark.parametrize("fmt,s,alpha", [(1, 4, 1.0), (1, 3, 3.0), (2, 4, 1.0), (2, 2, 5.0)])
def test_bracketed_half_formats_equal_oracle(gpu, fmt, s, alpha):
    dt = torch.bfloat16 if fmt == 1 else torch.float16
    plan = codec.Plan(SIZES, device=gpu)
    assert plan.strategy == "bracket"
    g = torch.Generator(device=gpu).manual_seed(77 + fmt)
    x = (torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3).to(dt).float()  # the exact upcast
    seed, off = 0x5EED, 3
    q, norms = plan.qsgd_encode(x, s, alpha=alpha, seed=seed, offset=off, value_format=fmt)
    stats = plan.spec_stats()
    plan.check()
    assert stats["listed"] > 0, stats
    L = 2**s
    y = plan.qsgd_decode(q, 8, L, norms)
    xh, qh, yh, nh = x.cpu(), q.cpu().numpy(), y.cpu().numpy(), norms.cpu().numpy()

    def check(t):
        o, n = plan.offsets[t], SIZES[t]
        v = xh[o:o + n].to(dt)
        if alpha != 1.0:
            v = torch.mul(v, alpha)  # the client weighting in the tensor's dtype
        ref = float(torch.norm(v.float().double()))
        if not abs(float(nh[t]) - ref) <= 2 ** -7 * ref:  # the norm rounded to the format
            return f"tensor {t}: norm {nh[t]} vs {ref}"
        if float(torch.tensor(float(nh[t])).to(dt).float()) != float(nh[t]):
            return f"tensor {t}: norm {nh[t]} is not a {dt} value"
        u = torch.from_numpy(oracle.philox_uniforms(seed, off, t, n))
        want, _, _, _ = oracle.qsgd_quantize(v, s, norm=float(nh[t]), u=u)
        if qh[o:o + n].tobytes() != want.numpy().tobytes():
            bad = np.flatnonzero(qh[o:o + n] != want.numpy())
            return f"tensor {t}: {bad.size} levels differ, first at {bad[:4].tolist()}"
        want_y = oracle.qsgd_dequantize(want, float(nh[t]), L, (n,)).numpy()
        if yh[o:o + n].tobytes() != want_y.tobytes():
            return f"tensor {t}: decode differs"
        return None

    with ThreadPoolExecutor(8) as ex:
        errors = [e for e in ex.map(check, range(len(SIZES))) if e]
    assert not errors, errors[:5]


def test_bracketed_half_equals_two_pass_given_its_norms(gpu):
    """Same payload as the two-pass encoder fed the bracketed encoder's norms (norm_in), for both
    formats: the decided levels and the fixed ones alike."""
    plan = codec.Plan(SIZES, device=gpu)
    other = codec.Plan(SIZES, device=gpu)
    other.set_encode_strategy("ordered")
    for fmt, dt in ((1, torch.bfloat16), (2, torch.float16)):
        g = torch.Generator(device=gpu).manual_seed(5 + fmt)
        x = (torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-2).to(dt).float()
        q, norms = plan.qsgd_encode(x, 4, alpha=2.0, seed=9, offset=1, value_format=fmt)
        q2, _ = other.qsgd_encode(x, 4, alpha=2.0, seed=9, offset=1, value_format=fmt, norm_in=norms)
        plan.check()
        other.check()
        for o, n in zip(plan.offsets, SIZES):
            assert torch.equal(q[o:o + n], q2[o:o + n]), (fmt, o, n)


def test_bracketed_half_requantise_whole_path(gpu):
    """A norm outside its bracket sends the tensor to the exact whole-tensor requantisation (the
    finish workgroups, quant_sub with the format's rounding): brackets left from an arena 100x
    smaller (the bracket launch skipped: test hook spec bit 0) put every sampled tensor there.
    Payload equal to the oracle's given the GPU norms."""
    plan = codec.Plan(SIZES, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(31)
    x0 = (torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-4).bfloat16().float()
    plan.qsgd_encode(x0, 4, seed=1, offset=1, value_format=1)
    plan.check()
    x = (torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-2).bfloat16().float()
    try:
        plan.set_debug(spec=1)  # keep x0's brackets
        q, norms = plan.qsgd_encode(x, 4, alpha=3.0, seed=2, offset=5, value_format=1)
        stats = plan.spec_stats()
        plan.check()
    finally:
        plan.set_debug()
    assert stats["whole"] >= len(SIZES) - 1, stats
    qh, nh, xh = q.cpu().numpy(), norms.cpu().numpy(), x.cpu()
    for t, (o, n) in enumerate(zip(plan.offsets, SIZES)):
        v = torch.mul(xh[o:o + n].bfloat16(), 3.0)
        u = torch.from_numpy(oracle.philox_uniforms(2, 5, t, n))
        want, _, _, _ = oracle.qsgd_quantize(v, 4, norm=float(nh[t]), u=u)
        assert qh[o:o + n].tobytes() == want.numpy().tobytes(), t
