"""Bracketed single-read encoder (strategy 3, omf_qsgd.hip qsgd_spec_*) against the oracle.

Every payload is compared bit for bit with the oracle's QSGD quantiser given the encoder's own
norm (checked against fp64 at NORM_RTOL) and the Philox uniforms of oracle/philox.py — the bar
of every other strategy.  The inputs exercise each path of the encoder: levels decided for the
whole bracket, undecided quads fixed exactly, tensors whose norm falls outside the sampled
bracket (a few huge elements the sample misses), slot overflows (heavy tails), deferred tensors
(all zero, single non-zero, sub-normal scale) and non-finite tensors.
"""

import numpy as np
import pytest
import torch

import oracle
from inputs import exact_input
from omnifed_amd import codec, shapes

pytestmark = pytest.mark.gpu

NORM_RTOL = 2e-6


def _check_against_oracle(plan, x_host, q, norms, s, seed, offset, alpha=1.0, finite=True):
    qh, nh = q.cpu().numpy(), norms.cpu().numpy()
    for t, (o, n) in enumerate(zip(plan.offsets, plan.sizes)):
        p = x_host[o:o + n]
        if alpha != 1.0:
            p = (torch.from_numpy(p) * np.float32(alpha)).numpy()
        if finite:
            ref = float(np.sqrt(np.sum(p.astype(np.float64) ** 2)))
            if ref > 1e-18:  # smaller: fp32 squares underflow (every strategy's norm does)
                assert nh[t] == pytest.approx(ref, rel=NORM_RTOL), (t, n)
        if nh[t] == 0:  # zero norm: all-zero payload (the Python layer sends the tensor dense)
            assert not qh[o:o + n].any(), (t, n)
            continue
        u = oracle.philox_uniforms(seed, offset, t, n)
        want, *_ = oracle.qsgd_quantize(torch.from_numpy(np.ascontiguousarray(p)), s, norm=float(nh[t]),
                                        u=torch.from_numpy(u))
        assert qh[o:o + n].tobytes() == want.numpy().tobytes(), (t, n, s)


def _bracket_plan(gpu, sizes):
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy("bracket")
    return plan


@pytest.mark.parametrize("s", [1, 3, 4, 8])
def test_bracket_mixed_sizes(gpu, s):
    sizes = [1, 7, 1000, 4096, 4097, 16384, 16385, 40000, 65536, 65537, 100003, 262149, 1 << 20, 3 << 20]
    plan = _bracket_plan(gpu, sizes)
    x = np.zeros(plan.arena_end, np.float32)
    for i, (o, n) in enumerate(zip(plan.offsets, sizes)):
        x[o:o + n] = exact_input(100 + i, n, -9)
    xd = torch.from_numpy(x).to(gpu)
    q, norms = plan.qsgd_encode(xd, s, seed=21, offset=3)
    assert plan.check()
    if s <= 4:  # bracketed path (wider payloads take the two-pass encoder)
        st = plan.spec_stats()
        # at most the mid-size tensors (a wide sampled bracket) can overflow a slot and be redone
        assert st["deferred"] == 0 and st["whole"] <= sum(16384 < n < 300000 for n in sizes), st
        assert s > 1 or st["whole"] == 0, st
    _check_against_oracle(plan, x, q, norms, s, 21, 3)
    # deterministic, and the payload does not depend on what the buffer held before
    q2 = torch.full_like(q, 0x55)
    q2, n2 = plan.qsgd_encode(xd, s, q_out=q2, seed=21, offset=3)
    assert torch.equal(n2, norms)
    for o, n in zip(plan.offsets, plan.sizes):  # the gaps between tensors are padding, never written
        assert torch.equal(q2[o:o + n], q[o:o + n])


def test_bracket_weighted(gpu):
    sizes = [5000, 300000, 1 << 20]
    plan = _bracket_plan(gpu, sizes)
    g = torch.Generator().manual_seed(4)
    x = (torch.randn(plan.arena_end, generator=g) * 1e-3).numpy()
    q, norms = plan.qsgd_encode(torch.from_numpy(x).to(gpu), 4, alpha=3.0, seed=8)
    _check_against_oracle(plan, x, q, norms, 4, 8, 0, alpha=3.0)


def test_bracket_adversarial_distributions(gpu):
    """Inputs whose sampled bracket misses the norm or overflows the slots: exact anyway."""
    n = 1 << 20
    rng = np.random.default_rng(7)
    cases = []
    spikes = rng.standard_normal(n).astype(np.float32) * 1e-3
    spikes[rng.choice(n, 3, replace=False)] = 50.0           # norm dominated by 3 unsampled elements
    cases.append(spikes)
    cases.append(rng.standard_cauchy(n).astype(np.float32))  # heavy tails: wide bracket
    sparse = np.zeros(n, np.float32)
    sparse[rng.choice(n, 500, replace=False)] = rng.standard_normal(500).astype(np.float32)
    cases.append(sparse)                                        # 0.05 % non-zero
    cases.append(np.full(n, 0.125, np.float32))                 # every element the same level point
    cases.append(np.zeros(n, np.float32))                       # deferred: zero norm
    one = np.zeros(n, np.float32)
    one[n // 3] = -2.5
    cases.append(one)                                           # single non-zero
    cases.append((rng.standard_normal(n) * 1e-41).astype(np.float32))  # sub-normal scale
    cases.append((rng.standard_normal(n) * 1e15).astype(np.float32))   # large scale
    ramp = np.linspace(-1, 1, n, dtype=np.float32)
    cases.append(ramp)                                          # smooth structure (strata alias)
    sizes = [c.size for c in cases]
    plan = _bracket_plan(gpu, sizes)
    x = np.zeros(plan.arena_end, np.float32)
    for o, c in zip(plan.offsets, cases):
        x[o:o + c.size] = c
    for s in (2, 4, 8):
        q, norms = plan.qsgd_encode(torch.from_numpy(x).to(gpu), s, seed=s, offset=1)
        assert plan.check()
        if s <= 4:
            st = plan.spec_stats()
            # the spiked, zero and single-element tensors cannot keep their sampled bracket
            assert st["whole"] >= 3 and st["deferred"] >= 2, st
        _check_against_oracle(plan, x, q, norms, s, s, 1)


def test_bracket_non_finite_matches_two_pass(gpu):
    """NaN / inf tensors (norm NaN / inf): the same payload as the two-pass encoder."""
    n = 70000
    a = np.linspace(-1, 1, n, dtype=np.float32)
    b = a.copy()
    b[123] = np.nan
    c = a.copy()
    c[4567] = np.inf
    plan = _bracket_plan(gpu, [n, n, n])
    x = np.zeros(plan.arena_end, np.float32)
    for o, v in zip(plan.offsets, (a, b, c)):
        x[o:o + n] = v
    xd = torch.from_numpy(x).to(gpu)
    q3, n3 = plan.qsgd_encode(xd, 4, seed=2)
    plan.set_encode_strategy("ordered")
    q1, n1 = plan.qsgd_encode(xd, 4, seed=2)
    torch.testing.assert_close(n3[:1], n1[:1], rtol=2e-6, atol=0)
    assert torch.isnan(n3[1]) and torch.isinf(n3[2]) and torch.isnan(n1[1]) and torch.isinf(n1[2])
    for o in plan.offsets[1:]:
        assert torch.equal(q3[o:o + n], q1[o:o + n])


def test_bracket_resnet18_full_arena(gpu):
    """Every tensor of the ResNet-18 update (BASELINE config 1) at s = 3, 4 and 8."""
    sizes = [shapes.numel(sh) for _, sh in shapes.resnet18()]
    plan = _bracket_plan(gpu, sizes)
    g = torch.Generator().manual_seed(18)
    x = (torch.randn(plan.arena_end, generator=g) * 1e-3).numpy()
    xd = torch.from_numpy(x).to(gpu)
    for s in (3, 4, 8):
        q, norms = plan.qsgd_encode(xd, s, seed=77, offset=s)
        if s <= 4:
            assert plan.spec_stats()["listed"] > 0
        _check_against_oracle(plan, x, q, norms, s, 77, s)


def test_bracket_large_tensors_sampled(gpu):
    """Llama-sized tensors (16 Mi and 2^25 + 13 elements): whole-tensor parity."""
    sizes = [1 << 24, (1 << 25) + 13, 4096]
    plan = _bracket_plan(gpu, sizes)
    g = torch.Generator(device=gpu).manual_seed(3)
    xd = torch.randn(plan.arena_end, device=gpu, generator=g) * 2e-3
    q, norms = plan.qsgd_encode(xd, 4, seed=5, offset=9)
    st = plan.spec_stats()
    assert st["whole"] == 0 and st["listed"] > 0, st
    x = xd.cpu().numpy()
    _check_against_oracle(plan, x, q, norms, 4, 5, 9)


def test_bracket_llama400m_equals_quantiser_given_its_norms(gpu):
    """Full Llama-400M arena (183 tensors, 401 M elements), s = 4 and s = 3, client weight 3:
    the bracketed encoder's payload equals the flat quantiser's given the same norms (exact
    division, the same Philox draws: the element math of every strategy), and its norms agree
    with the two-pass encoder's to rounding."""
    sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes("llama400m")]
    plan = _bracket_plan(gpu, sizes)
    g = torch.Generator(device=gpu).manual_seed(400)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    for s in (4, 3):
        q, norms = plan.qsgd_encode(x, s, alpha=3.0, seed=17, offset=s)
        st = plan.spec_stats()
        assert st["whole"] == 0 and st["listed"] > 0, st
        q2, n2 = plan.qsgd_encode(x, s, alpha=3.0, seed=17, offset=s, norm_in=norms)
        assert torch.equal(n2, norms)
        for o, n in zip(plan.offsets, plan.sizes):
            assert torch.equal(q[o:o + n], q2[o:o + n]), (o, n, s)
        plan.set_encode_strategy("ordered")
        _, n3 = plan.qsgd_encode(x, s, alpha=3.0, seed=17, offset=s)
        plan.set_encode_strategy("bracket")
        torch.testing.assert_close(n3, norms, rtol=2e-6, atol=0)
        del q, q2


@pytest.mark.parametrize("s", [4, 8])
def test_arena_decoder_boundaries_and_padding(gpu, s):
    """qsgd_decode_arena on a layout with tiny tensors, odd sizes and caller-chosen gaps: every
    tensor element equals the oracle's decode (and the accumulate mode adds it), and padding
    between tensors is never written (a canary survives)."""
    rng = np.random.default_rng(11 + s)
    sizes = [1, 3, 5, 64, 1000, 4095, 4097, 10, 70001, 2, 16384, 9]
    offsets, cur = [], 0
    for n in sizes:
        cur = (cur + 3) // 4 * 4 + 4 * int(rng.integers(0, 600))  # starts: multiples of 4, random gaps
        offsets.append(cur)
        cur += n
    plan = codec.Plan(sizes, offsets=offsets, device=gpu)
    L = 2 ** s
    w = 8 if L <= 127 else 32
    qdt = np.int8 if w == 8 else np.int32
    q = np.zeros(plan.payload_elems(w), qdt)
    norms = rng.random(len(sizes)).astype(np.float32) + 0.5
    want = {}
    for t, (o, n) in enumerate(zip(offsets, sizes)):
        q[o:o + n] = rng.integers(-L, L + 1, n).astype(qdt)
        want[t] = oracle.qsgd_dequantize(torch.from_numpy(q[o:o + n].astype(np.int64)), float(norms[t]), L,
                                         (n,)).numpy()
    qd = torch.from_numpy(q).to(gpu)
    nd = torch.from_numpy(norms).to(gpu)
    canary = -12345.5
    y = torch.full((plan.arena_end,), canary, dtype=torch.float32, device=gpu)
    plan.qsgd_decode(qd, w, L, nd, y_out=y)
    yh = y.cpu().numpy()
    mask = np.ones(plan.arena_end, bool)
    for t, (o, n) in enumerate(zip(offsets, sizes)):
        assert yh[o:o + n].tobytes() == want[t].astype(np.float32).tobytes(), t
        mask[o:o + n] = False
    assert (yh[mask] == canary).all()  # padding untouched
    # accumulate: y += decode, padding still untouched
    plan.qsgd_decode(qd, w, L, nd, y_out=y, accumulate=True)
    yh2 = y.cpu().numpy()
    for t, (o, n) in enumerate(zip(offsets, sizes)):
        assert yh2[o:o + n].tobytes() == (want[t].astype(np.float32) + want[t].astype(np.float32)).tobytes(), t
    assert (yh2[mask] == canary).all()
