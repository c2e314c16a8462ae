"""Round-3 GPU tests, all through the HIP C ABI:

* in-kernel timeouts surface as ``RuntimeError`` on every product entry point
  (``encode_updates_dict``, ``DeviceAggregator.accumulate_updates`` / ``apply_and_encode``,
  ``qsgd_weighted_round``), as the reference PS turns any codec exception into
  ``UpdateResponse(success=False)`` (global_grpc_server.py:138-145);
* the multi-GPU PS aggregates (omnifed_amd/ps.py) on a real RCCL group of world size 1
  (``nccl`` in-process, ``device_id`` bound): the weighted QSGD round in both modes and the
  Top-K sparse aggregate in both modes, against the oracle and the one-GPU aggregator;
* oracle pins of the fused PS step (f2) and of a stratified Llama-400M sample on the
  bracketed single-read encoder.
"""


import numpy as np
import pytest
import torch

import oracle
from omnifed_amd import codec, shapes
from omnifed_amd.hybrid.communicator.global_grpc_compression import encode_updates_dict
from omnifed_amd.hybrid.compression.qsgd import QSGDQuantCompression

pytestmark = pytest.mark.gpu

SPEC_NO_FOLD = 16  # omf_plan_set_debug spec bit: fold skipped, every fix wait expires
RING_NO_LOADED = 8  # omf_plan_set_debug ring bit: slots never marked loaded, hand-off waits expire


def _oracle_q(x_np, s, norm, u_np):
    q, *_ = oracle.qsgd_quantize(torch.from_numpy(np.ascontiguousarray(x_np)), s, norm=norm,
                                 u=torch.from_numpy(np.ascontiguousarray(u_np)))
    return q.numpy()


class _Forced:
    """Force the plan's next encodes to time out in-kernel (test hooks), restore on exit."""

    def __init__(self, plan, strategy):
        self.plan, self.strategy = plan, strategy

    def __enter__(self):
        self.prev = self.plan.strategy
        self.plan.set_encode_strategy(self.strategy)
        if self.strategy == "bracket":
            self.plan.set_debug(spec=SPEC_NO_FOLD)
            self.plan.set_resident_capacity(0, wait_us=50)  # the fix threads' norm-wait bound
        else:
            self.plan.set_debug(ring=RING_NO_LOADED, lds_wait_us=200)
        return self.plan

    def __exit__(self, *exc):
        torch.cuda.synchronize()
        self.plan.set_debug()
        self.plan.set_resident_capacity(0, wait_us=0)
        try:
            self.plan.check()  # drop whatever the forced launch left
        except codec.CodecError:
            pass
        self.plan.set_encode_strategy(self.prev)
        return False


NAMED = [("w1", (256, 1024)), ("b1", (1000,)), ("w2", (70001,)), ("n", (4096,))]


def _updates(gpu, seed=3):
    g = torch.Generator().manual_seed(seed)
    return {n: (torch.randn(s, generator=g) * 1e-2).to(gpu) for n, s in NAMED}


@pytest.mark.parametrize("strategy", ["bracket", "ring"])
def test_timeout_raises_on_the_drop_in(gpu, strategy):
    """A forced in-kernel timeout makes encode_updates_dict and the PS aggregator raise
    RuntimeError (never a silent invalid payload); the next encode is clean again."""
    from omnifed_amd.ps import DeviceAggregator

    upd = _updates(gpu)
    plan = codec.Plan.get([shapes.numel(s) for _, s in NAMED], device=gpu)  # the plan the drop-in uses
    comp = QSGDQuantCompression(bit_width=4, device=gpu)
    with _Forced(plan, strategy):
        with pytest.raises(RuntimeError, match="timeout|exceeded its bound"):
            encode_updates_dict(upd, comp)
    good = encode_updates_dict(upd, comp)  # no stale error, a valid payload
    assert [L.compression_type for L in good] == ["QSGDQuantCompression"] * len(NAMED)

    agg = DeviceAggregator(NAMED, device=gpu)
    assert agg.plan is plan
    with _Forced(plan, strategy):
        with pytest.raises(RuntimeError):
            agg.accumulate_updates(upd, comp, number_samples=5, weight=5)
    assert agg.update_count == 0 and agg.total_samples == 0  # the failed client was not counted
    assert not bool(agg.acc.any())  # and nothing reached the accumulator
    agg.accumulate_updates(upd, comp, number_samples=5, weight=5)
    agg.accumulate_updates(upd, comp, number_samples=7, weight=7)
    with _Forced(plan, strategy):
        with pytest.raises(RuntimeError):
            agg.apply_and_encode(comp)
    avg, layers = agg.apply_and_encode(comp)
    assert len(layers) == len(NAMED) and all(L.compression_type == "QSGDQuantCompression" for L in layers)
    # the accumulator keeps the sum; the average is acc / total (both branches alike)
    want = agg.acc.cpu().numpy() / np.float32(12)
    for i, (n, _) in enumerate(NAMED):
        o, k = agg.plan.offsets[i], agg.plan.sizes[i]
        assert avg[n].cpu().numpy().reshape(-1).tobytes() == want[o:o + k].tobytes(), n


# ---------------------------------------------------------------- RCCL, world size 1

def _r18_arena(gpu, seed):
    named = shapes.model_shapes("resnet18")
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(seed)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    return plan, x


@pytest.mark.parametrize("mode", ["gather", "reduce"])
def test_qsgd_weighted_round_rccl_world1(nccl1, mode):
    """qsgd_weighted_round over RCCL (world 1): Σ decode(Q(w·x)) / Σw equals the one-GPU path
    byte for byte, and per tensor the oracle's levels / decode given the GPU norm and draws."""
    from omnifed_amd.ps import DeviceAggregator, GpuOps, qsgd_weighted_round, total_weight, weighted_sum_error_bound

    gpu = nccl1
    plan, x = _r18_arena(gpu, 11)
    ops = GpuOps(plan, seed=77)
    assert ops.rank == 0
    w = 37.0
    total = total_weight(w, gpu)
    assert total == w
    s, call = 4, 5
    out = qsgd_weighted_round(x, w, total, ops, s, call, mode=mode)
    torch.cuda.synchronize()
    # one-GPU reference: the same encode, decode-accumulate into zeros, divide
    q, norms = plan.qsgd_encode(x, s, alpha=w, seed=ops.key, offset=call)
    acc = torch.zeros(plan.arena_end, device=gpu)
    plan.qsgd_decode(q, 8, 16, norms, y_out=acc, accumulate=True)
    codec.div_(acc, total)
    oh, ah, xh, qh, nh = (t.cpu().numpy() for t in (out, acc, x, q, norms))
    for o, n in zip(plan.offsets, plan.sizes):
        assert oh[o:o + n].tobytes() == ah[o:o + n].tobytes()
    # oracle: levels of fl32(w·x) given the GPU norm and the Philox draws, decode, / total
    for t in (0, 7, 20, len(plan.sizes) - 2, len(plan.sizes) - 1):
        o, n = plan.offsets[t], plan.sizes[t]
        xw = (xh[o:o + n] * np.float32(w)).astype(np.float32)
        want_q = _oracle_q(xw, s, float(nh[t]), oracle.philox_uniforms(ops.key, call, t, n))
        assert qh[o:o + n].tobytes() == want_q.tobytes(), t
        dec = oracle.qsgd_dequantize(torch.from_numpy(want_q), float(nh[t]), 16, (n,))
        want = (dec / np.float32(total)).numpy()
        got = oh[o:o + n]
        if mode == "gather":
            assert got.tobytes() == want.tobytes(), t
        bound = weighted_sum_error_bound(dec.double().abs(), torch.from_numpy(want).double(), 1, total).numpy()
        assert np.all(np.abs(got.astype(np.float64) - want.astype(np.float64)) <= bound), t
    # the drop-in aggregator (one GPU, same draws) gives the same average
    named = shapes.model_shapes("resnet18")
    agg = DeviceAggregator(named, device=gpu)
    assert agg.plan is plan
    agg.plan.qsgd_decode(q, 8, 16, norms, y_out=agg.acc, accumulate=True)
    agg.total_samples = int(w)
    avg = agg.apply()
    for (name, _), o, n in zip(named, plan.offsets, plan.sizes):
        assert avg[name].cpu().numpy().reshape(-1).tobytes() == oh[o:o + n].tobytes(), name


@pytest.mark.parametrize("dst", [None, 0])
def test_topk_sparse_aggregate_rccl_world1(nccl1, dst):
    """topk_sparse_aggregate over RCCL (all-gather, or gather to a root) of one client's
    selection: zeros, scatter-add in rank order, / client count — the reference's
    layerwise_decompress (core.py:62-71) restated by the oracle, bit for bit."""
    from omnifed_amd.ps import GpuOps, topk_sparse_aggregate

    gpu = nccl1
    sizes = [5000, 1 << 20, 70001, 300_000]
    plan = codec.Plan.get(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(21)
    x = torch.randn(plan.arena_end, device=gpu, generator=g)
    ratio = 0.01
    vals, idx, ks = plan.topk_encode(x, ratio)
    ops = GpuOps(plan)
    acc = torch.empty(plan.arena_end, device=gpu)
    out = topk_sparse_aggregate(vals, idx, ratio, acc, ops, client_count=1, dst=dst)
    torch.cuda.synchronize()
    vh, ih, oh = vals.cpu(), idx.cpu(), out.cpu()
    K = 0
    for o, n, k in zip(plan.offsets, sizes, ks):
        want = oracle.layerwise_decompress([vh[K:K + k]], [ih[K:K + k]], (n,), 1)
        assert oh[o:o + n].numpy().tobytes() == want.reshape(-1).numpy().tobytes()
        K += k


def test_weighted_round_timeout_raises_on_every_rank(nccl1):
    """A forced encoder timeout inside qsgd_weighted_round raises before any payload moves
    (the flags are agreed with an RCCL all-reduce), and the next round is clean."""
    from omnifed_amd.ps import GpuOps, qsgd_weighted_round

    gpu = nccl1
    sizes = [1 << 20, 5000, 3 << 20]
    plan = codec.Plan.get(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(5)
    x = torch.randn(plan.arena_end, device=gpu, generator=g)
    ops = GpuOps(plan, seed=3)
    for strategy in ("bracket", "ring"):
        with _Forced(plan, strategy):
            with pytest.raises(RuntimeError, match="in-kernel timeout"):
                qsgd_weighted_round(x, 2.0, 2.0, ops, 4, 0, mode="gather")
        out = qsgd_weighted_round(x, 2.0, 2.0, ops, 4, 1, mode="reduce")
        for o, n in zip(plan.offsets, plan.sizes):  # tensor ranges (the arena padding is never written)
            assert bool(torch.isfinite(out[o:o + n]).all())


# ---------------------------------------------------------------- oracle pins (f2, bracketed L400)

@pytest.mark.parametrize("strategy", ["bracket", "ring"])
def test_fused_ps_step_against_the_oracle(gpu, strategy):
    """omf_ps_apply_encode: avg = acc / total (numpy's fp32 division) and, per tensor, the payload
    equals the oracle's quantisation of that average given the GPU norm and Philox draws, and the
    norm is within 2e-6 of the fp64 norm (not a comparison with another GPU encoder call)."""
    sizes = [5, 16384, 70001, 1 << 20, 3000, 2_000_000]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy(strategy)
    g = torch.Generator(device=gpu).manual_seed(19)
    acc = torch.randn(plan.arena_end, device=gpu, generator=g) * 3.0
    total, s, seed, off = 7.0, 3, 1234, 2
    avg, q, norms = plan.ps_apply_encode(acc, total, s, seed=seed, offset=off)
    assert plan.check()
    avg_np = acc.cpu().numpy() / np.float32(total)
    ah, qh, nh = avg.cpu().numpy(), q.cpu().numpy(), norms.cpu().numpy()
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        a = avg_np[o:o + n]
        assert ah[o:o + n].tobytes() == a.tobytes(), t
        ref = float(np.sqrt(np.sum(a.astype(np.float64) ** 2)))
        assert abs(float(nh[t]) - ref) <= 2e-6 * ref, t
        want = _oracle_q(a, s, float(nh[t]), oracle.philox_uniforms(seed, off, t, n))
        assert qh[o:o + n].tobytes() == want.tobytes(), t


def test_llama400m_bracketed_sample_against_the_oracle(gpu):
    """Llama-400M at s = 3 on the default (bracketed single-read) encoder: a stratified sample of
    8 whole tensors — embed_tokens, lm_head, the final norm, attention / MLP matrices and RMSNorm
    vectors of early, middle and late layers — equals the oracle given the GPU norm and draws."""
    named = shapes.model_shapes("llama400m")
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=gpu)
    assert plan.strategy == "bracket"
    g = torch.Generator(device=gpu).manual_seed(31)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    s, seed, off = 3, 99, 6
    q, norms = plan.qsgd_encode(x, s, seed=seed, offset=off)
    assert plan.check()
    names = [n for n, _ in named]
    want_names = ["model.embed_tokens.weight", "lm_head.weight", "model.norm.weight"]
    for layer, part in ((0, "self_attn.q_proj.weight"), (7, "mlp.down_proj.weight"),
                        (10, "input_layernorm.weight"), (15, "self_attn.o_proj.weight"),
                        (19, "mlp.up_proj.weight")):
        want_names.append(f"model.layers.{layer}.{part}")
    sample = [names.index(n) for n in want_names]
    assert len(set(sample)) == 8
    nh = norms.cpu().numpy()
    for t in sample:
        o, n = plan.offsets[t], sizes[t]
        xh = x[o:o + n].cpu().numpy()
        want = _oracle_q(xh, s, float(nh[t]), oracle.philox_uniforms(seed, off, t, n))
        assert q[o:o + n].cpu().numpy().tobytes() == want.tobytes(), names[t]


# ---------------------------------------------------------------- tiled zero-fill Top-K decode

def _scatter_ref(plan, values, indices, ks):
    """zeros(arena) then y[begin_t + idx] = v per tensor (torch on the GPU), skipping -1 / out of range."""
    y = torch.zeros(plan.arena_end, device=values.device)
    K = 0
    for o, n, k in zip(plan.offsets, plan.sizes, ks):
        ix, v = indices[K:K + k], values[K:K + k]
        ok = (ix >= 0) & (ix < n)
        y[o + ix[ok]] = v[ok]
        K += k
    return y


def test_topk_tiled_decode_matches_scatter(gpu):
    """Mode 0 through the tiled decoder (bucket by 64 Ki super-tile, LDS sub-tiles) equals zeros +
    scatter over the whole arena, padding included: random selections, a tensor whose selection is
    clustered in one sub-tile, padding indices (-1) and out-of-range indices are skipped, and stale
    contents of y are overwritten everywhere."""
    sizes = [5, 70001, 1 << 20, 3000, 200_003, 65536, 131_071]
    plan = codec.Plan(sizes, device=gpu)
    ratio = 0.01
    ks = plan.topk_ks(ratio)
    assert ks[2] <= 16384
    g = torch.Generator(device=gpu).manual_seed(12)
    vals, idx = [], []
    for t, (n, k) in enumerate(zip(sizes, ks)):
        if t == 2:  # clustered: every selected index in one 16 Ki sub-tile of a super-tile
            ix = torch.randperm(16384, device=gpu, generator=g)[:k] + 3 * 16384
        else:
            ix = torch.randperm(n, device=gpu, generator=g)[:k]
        if t == 4:
            ix[::7] = -1        # padding
            ix[3::11] = n + 5   # out of range
        idx.append(ix.to(torch.int64))
        vals.append(torch.randn(k, device=gpu, generator=g))
    v, ix = torch.cat(vals), torch.cat(idx)
    y = torch.full((plan.arena_end,), 7.0, device=gpu)
    got = plan.topk_decode_arena(v, ix, ratio, y=y, mode=0)
    torch.cuda.synchronize()
    want = _scatter_ref(plan, v, ix, ks)
    assert torch.equal(got, want)
    # the same workspace again (counts left zeroed by the previous call), another selection
    v2 = torch.randn_like(v)
    got2 = plan.topk_decode_arena(v2, ix, ratio, y=y, mode=0)
    assert torch.equal(got2, _scatter_ref(plan, v2, ix, ks))


@pytest.mark.parametrize("ntiny", [40, 700])
def test_topk_tiled_decode_many_small_tensors(gpu, ntiny):
    """A place block of the tiled decoder that spans many tensors finds each value's tensor by a
    search of their first-value offsets — staged in LDS up to 512 tensors (40 tiny tensors), from
    global memory beyond (700): both equal zeros + scatter, padding and out-of-range skipped."""
    sizes = [100] * ntiny + [70001, 3, 250, 9000] + [100] * 5
    plan = codec.Plan(sizes, device=gpu)
    ratio = 0.01
    ks = plan.topk_ks(ratio)
    g = torch.Generator(device=gpu).manual_seed(31 + ntiny)
    vals, idx = [], []
    for t, (n, k) in enumerate(zip(sizes, ks)):
        ix = torch.randperm(n, device=gpu, generator=g)[:k].to(torch.int64)
        if t % 9 == 4:
            ix[0] = -1  # padding
        if t % 13 == 6:
            ix[0] = n  # out of range
        idx.append(ix)
        vals.append(torch.randn(k, device=gpu, generator=g))
    v, ix = torch.cat(vals), torch.cat(idx)
    y = torch.full((plan.arena_end,), -3.0, device=gpu)
    got = plan.topk_decode_arena(v, ix, ratio, y=y, mode=0)
    torch.cuda.synchronize()
    assert torch.equal(got, _scatter_ref(plan, v, ix, ks))


def test_llama400m_topk_encode_then_tiled_decode(gpu):
    """Llama-400M, k = 1 %: the encoder's selection decoded by the tiled decoder equals zeros +
    scatter of the same (values, indices), over the whole arena."""
    named = shapes.model_shapes("llama400m")
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(23)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    vals, idx, ks = plan.topk_encode(x, 0.01)
    y = plan.topk_decode_arena(vals, idx, 0.01, mode=0)
    torch.cuda.synchronize()
    assert torch.equal(y, _scatter_ref(plan, vals, idx, ks))


@pytest.mark.parametrize("groups", [2, 3, 4, 7])
def test_topk_group_pipeline_matches_one_group(gpu, monkeypatch, groups):
    """The sampled Top-K path run as a two-stream pipeline of tensor groups gives the same bytes
    (values, indices, residual) as one group on the caller's stream, over three error-feedback
    calls — and so does the forced fallback sort with the pipeline on."""
    sizes = [1_500_000] * 9 + [3_000_017, 4096, 777_777, 2_000_000, 65_536, 1 << 21]
    assert sum(sizes) >= 1 << 24  # the pipeline's minimum arena
    plan = codec.Plan(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(31)
    xs = [torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3 for _ in range(3)]

    def run(n_groups, fallback=False):
        plan.set_topk(groups=n_groups, fallback=1 if fallback else 0)
        res = torch.zeros(plan.arena_end, device=gpu)
        outs = []
        for i, x in enumerate(xs):
            v, ix, _ = plan.topk_encode(x, 0.01, residual=res, residual_mode=2 if i == 0 else 1, alpha=3.0)
            outs.append((v.clone(), ix.clone()))
        torch.cuda.synchronize()
        return outs, res

    ref_outs, ref_res = run(1)
    for fb in (False, True):
        outs, res = run(groups, fb)
        for (v0, i0), (v1, i1) in zip(ref_outs, outs):
            assert torch.equal(v0, v1) and torch.equal(i0, i1)
        assert torch.equal(ref_res, res)


@pytest.mark.parametrize("knob,value", [("sure", (0, 0)), ("sure", (0.5, 0)), ("sure", (6, 32)), ("sure", (40, 0)),
                                        ("sample_runs", 4096), ("sample_runs", 512)])
def test_topk_sure_margin_does_not_change_the_selection(gpu, knob, value):
    """The "sure" bin (keys whose residual the fused pass zeroes at once) is a performance knob:
    with no margin about half the tensors take more sure keys than k (the bucket kernels give
    those their t' back), with a huge one none is sure — values, indices and the residual over
    three error-feedback calls equal the default's.  So does the sample size: 4 Ki runs per tensor
    take two sample blocks that flush into the tensor's global histogram (the default 2 Ki is one
    block deriving the threshold from its own), 512 a coarser threshold."""
    sizes = [1_500_000, 4096, 3_000_017, 777_777, 65_536, 2_000_000, 300]
    plan = codec.Plan(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(37)
    xs = [torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3 for _ in range(3)]

    def run():
        res = torch.zeros(plan.arena_end, device=gpu)
        outs = []
        for i, x in enumerate(xs):
            v, ix, _ = plan.topk_encode(x, 0.01, residual=res, residual_mode=2 if i == 0 else 1, alpha=2.0)
            outs.append((v.clone(), ix.clone()))
        torch.cuda.synchronize()
        return outs, res

    plan.set_topk(sample_runs=0, sure=(1.5, 2.0))  # the defaults
    ref_outs, ref_res = run()
    plan.set_topk(**{knob: value})
    outs, res = run()
    for (v0, i0), (v1, i1) in zip(ref_outs, outs):
        assert torch.equal(v0, v1) and torch.equal(i0, i1)
    assert torch.equal(ref_res, res)


# ---------------------------------------------------------------- grid encoder (strategy 4)

def _oracle_check(plan, x, q, norms, s, seed, off, alpha=1.0, tensors=None):
    xh, qh, nh = x.cpu().numpy(), q.cpu().numpy(), norms.cpu().numpy()
    for t in (range(plan.nt) if tensors is None else tensors):
        o, n = plan.offsets[t], plan.sizes[t]
        xs = (xh[o:o + n] * np.float32(alpha)).astype(np.float32) if alpha != 1.0 else xh[o:o + n]
        ref = float(np.sqrt(np.sum(xs.astype(np.float64) ** 2)))
        assert abs(float(nh[t]) - ref) <= 2e-6 * ref, t
        want = _oracle_q(xs, s, float(nh[t]), oracle.philox_uniforms(seed, off, t, n))
        assert qh[o:o + n].tobytes() == want.tobytes(), t


@pytest.mark.parametrize("cfg,s,alpha", [("resnet18", 3, 1.0), ("resnet18", 4, 7.0), ("resnet18", 8, 1.0),
                                         ("mixed", 4, 3.0)])
def test_grid_encoder_against_the_oracle(gpu, cfg, s, alpha):
    """The one-launch grid encoder: every tensor's norm within 2e-6 of fp64 and its payload the
    oracle's given that norm and the Philox draws (int8 and int32 payloads, weighting fused);
    its norms equal the bracketed / ring encoders' up to their own fold order."""
    if cfg == "mixed":
        sizes = [1, 5, 63, 64, 4097, 16384, 16385, 70001, 1 << 20, 3, 250_000]
    else:
        sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes(cfg)]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy("grid")
    assert plan.encoder_kernel == "qsgd_encode_grid"
    g = torch.Generator(device=gpu).manual_seed(41)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    x[plan.offsets[-1]:plan.offsets[-1] + 7] = 0.0
    seed, off = 12345, 9
    q, norms = plan.qsgd_encode(x, s, alpha=alpha, seed=seed, offset=off)
    assert plan.check() is True  # no recomputation: the grid was co-resident
    _oracle_check(plan, x, q, norms, s, seed, off, alpha)
    # decode round trip stays the decoder's
    L = 2**s
    y = plan.qsgd_decode(q, 8 if L <= 127 else 32, L, norms)
    for o, n in zip(plan.offsets, plan.sizes):  # tensor ranges: the decoder never writes the arena padding
        assert bool(torch.isfinite(y[o:o + n]).all())


def test_grid_encoder_barrier_timeout_recovers_exactly(gpu):
    """Test hook: no workgroup arrives at the grid barrier, every wait expires, and each
    workgroup recomputes the partials it needs from x in the producers' order — the same
    norms and payload bit for bit, reported as a recomputation (check() returns False)."""
    sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes("resnet18")][:20]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy("grid")
    g = torch.Generator(device=gpu).manual_seed(42)
    x = torch.randn(plan.arena_end, device=gpu, generator=g)
    q0, n0 = plan.qsgd_encode(x, 4, seed=3, offset=1)
    assert plan.check() is True
    q0, n0 = q0.clone(), n0.clone()
    plan.set_debug(spec=32)
    plan.set_resident_capacity(0, wait_us=100)
    try:
        q1, n1 = plan.qsgd_encode(x, 4, seed=3, offset=1)
        assert plan.check() is False
    finally:
        plan.set_debug()
        plan.set_resident_capacity(0, wait_us=0)
    assert torch.equal(n0, n1)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(q0[o:o + n], q1[o:o + n])
    q2, n2 = plan.qsgd_encode(x, 4, seed=3, offset=1)  # the counter still lines up afterwards
    assert plan.check() is True and torch.equal(n2, n0)
