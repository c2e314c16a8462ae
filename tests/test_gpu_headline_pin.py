"""The bench's headline arenas pinned to the oracle directly, tensor by tensor (round 4).

bench.py encodes one client's Llama-400M update (N(0,1)·1e-3, generator seed 1000 + rank) at
s = 4 with on-device Philox draws and the client weighting fused as alpha, through the
bracketed single-read encoder.  Here EVERY tensor of that arena — and of Llama-400M at s = 3
with alpha = 3, and of Llama-150M at s = 4 — is compared with ``oracle.qsgd_quantize``
(qsgd.py:36-64 restated) given the GPU's norm and ``oracle.philox_uniforms``: payload bytes
equal, and the decode equal to ``oracle.qsgd_dequantize``.  The bracketed encoder's finish
pass (the undecided quads it lists and fixes) must have run: spec_stats()["listed"] > 0.
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


@pytest.mark.parametrize("cfg,s,alpha", [("llama400m", 4, 1.0), ("llama400m", 3, 3.0), ("llama150m", 4, 1.0)])
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
    stats = plan.spec_stats()
    plan.check()
    assert stats["listed"] > 0, stats  # the finish pass fixed undecided quads
    L = 2**s
    y = plan.qsgd_decode(q, 8, L, norms)
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


SPEC_LEGACY_FINISH = 512  # omf_plan_set_debug spec bit: the separate finish launch instead of the fused finish


@pytest.mark.parametrize("case", ["llama400m", "mixed", "degenerate", "ps_step"])
def test_fused_finish_equals_finish_launch(gpu, case):
    """The bracketed encoder's fused finish (each tensor folded and fixed by its last-arriving pass
    workgroup, blocks in the rotated order, the repair launch for bad tensors) writes the same payload
    and norms, bit for bit, as the separate finish launch — on the bench arena, on mixed sizes, on
    tensors whose sampled bracket is degenerate or misses the norm (requantised whole by the repair
    launch), and in the fused PS step (divide + encode)."""
    if case == "llama400m":
        sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes("llama400m")]
    else:
        sizes = [5, 16384, 70001, 1 << 20, 3000, 2_000_000, 1 << 25, 777_777, 4096 * 3 + 1]
    plan = codec.Plan(sizes, device=gpu)
    if plan.strategy != "bracket":
        plan.set_encode_strategy("bracket")
    g = torch.Generator(device=gpu).manual_seed(77)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    if case == "degenerate":  # a zero tensor, a single spike (degenerate samples), a spiky tensor (bracket misses)
        o1, o3, o5 = plan.offsets[1], plan.offsets[3], plan.offsets[5]
        x[o1:o1 + sizes[1]] = 0.0
        x[o3:o3 + sizes[3]] = 0.0
        x[o3 + 12345] = 5.0
        x[o5:o5 + sizes[5]:997] *= 4000.0
    outs = []
    for legacy in (False, True):
        plan.set_debug(spec=SPEC_LEGACY_FINISH if legacy else 0)
        try:
            if case == "ps_step":
                avg, q, n = plan.ps_apply_encode(x, 7.0, 4, seed=5, offset=2)
                outs.append((q.clone(), n.clone(), avg.clone()))
            else:
                q, n = plan.qsgd_encode(x, 4, alpha=3.0, seed=5, offset=2)
                outs.append((q.clone(), n.clone(), None))
            stats = plan.spec_stats()
            plan.check()
        finally:
            plan.set_debug()
        if case == "degenerate":
            assert stats["whole"] >= 2, stats  # the repair path ran
    (qa, na, aa), (qb, nb, ab) = outs
    assert torch.equal(na, nb)
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):  # tensor ranges (arena padding is never written)
        assert torch.equal(qa[o:o + n], qb[o:o + n]), t
        if aa is not None:
            assert torch.equal(aa[o:o + n], ab[o:o + n]), t
