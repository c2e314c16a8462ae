"""QSGD parity on the GPU through the HIP C ABI (omf_qsgd_encode / omf_qsgd_decode).

Bar (BASELINE.json north_star): the integer payload is bit-exact vs the reference
CPU codec and decoded floats equal it (tolerance 0: we get bit equality) given the
same (norm, u).  The reference's norm is injected from the golden vectors; the
GPU's own norm is checked against an fp64 reference (rel 2e-6) and then injected
into the oracle, which must reproduce the GPU payload bit for bit.
"""

import hashlib

import numpy as np
import pytest
import torch

import oracle
from inputs import exact_input, sha
from omnifed_amd import codec, shapes

pytestmark = pytest.mark.gpu

NORM_RTOL = 2e-6  # GPU norm (fp32 squares, fp64 partials) vs fp64 numpy


def _dev(a, gpu, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(gpu)


def _oracle_q(x_np, s, norm, u_np):
    q, *_ = oracle.qsgd_quantize(torch.from_numpy(x_np), s, norm=norm, u=torch.from_numpy(u_np))
    return q.numpy()


def test_golden_cases_injected(gpu, golden, golden_index):
    for c in golden_index["qsgd"]:
        key = f"qsgd/{c['id']}"
        n, s = c["n"], c["s"]
        plan = codec.Plan.get([n], device=gpu)
        x = _dev(golden[key + "/x"], gpu)
        u = _dev(oracle.mt19937_uniforms(c["seed"], n), gpu)
        nin = torch.tensor([c["norm"]], dtype=torch.float32, device=gpu)
        q, norms = plan.qsgd_encode(x, s, u=u, norm_in=nin)
        assert q[:n].cpu().numpy().tobytes() == golden[key + "/q"].tobytes(), key
        y = plan.qsgd_decode(q, c["width"], c["level"], norms)
        assert y.cpu().numpy().tobytes() == golden[key + "/y"].tobytes(), key


def test_golden_hashed_cases(gpu, golden_index):
    for c in golden_index["qsgd_hashed"]:
        n, s = c["n"], c["s"]
        x_np = exact_input(c["seed"], n, c["scale_log2"])
        assert sha(x_np) == c["x_sha"]
        plan = codec.Plan.get([n], device=gpu)
        u = _dev(oracle.mt19937_uniforms(c["seed"], n), gpu)
        nin = torch.tensor([c["norm"]], dtype=torch.float32, device=gpu)
        q, norms = plan.qsgd_encode(_dev(x_np, gpu), s, u=u, norm_in=nin)
        assert hashlib.sha256(q[:n].cpu().numpy().tobytes()).hexdigest() == c["q_sha"], c
        y = plan.qsgd_decode(q, c["width"], 2**s, norms)
        assert sha(y.cpu().numpy()) == c["y_sha"], c


def test_golden_edge_cases(gpu, golden, golden_index):
    from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb

    for c in golden_index["qsgd_edge"]:
        key = f"edge/{c['name']}/{c['s']}"
        L = pb.LayerState()
        L.ParseFromString(golden[key + "/layer"].tobytes())
        x_np = golden[key + "/x"].reshape(-1)
        if L.compression_type != "QSGDQuantCompression":
            continue
        n = x_np.size
        plan = codec.Plan.get([n], device=gpu)
        norm = float(np.frombuffer(L.meta_tensor, np.float32)[0])
        u = _dev(oracle.mt19937_uniforms(c["seed"], n), gpu)
        q, norms = plan.qsgd_encode(_dev(x_np.astype(np.float32), gpu), c["s"], u=u,
                                    norm_in=torch.tensor([norm], device=gpu))
        assert q[:n].cpu().numpy().tobytes() == L.values_data, key
        y = plan.qsgd_decode(q, L.width, L.level, norms)
        assert y.cpu().numpy().tobytes() == golden[key + "/y"].tobytes(), key


MIXED_SIZES = [1, 7, 1000, 16384, 16385, 40000, 100003, 262149, 1 << 20]


def _mixed_arena(gpu, sizes, seed=3, scale=-9):
    plan = codec.Plan.get(sizes, device=gpu)
    x = torch.zeros(plan.arena_end, dtype=torch.float32)
    parts = []
    for i, (o, n) in enumerate(zip(plan.offsets, sizes)):
        p = exact_input(seed + i, n, scale)
        parts.append(p)
        x[o:o + n] = torch.from_numpy(p)
    return plan, x.to(gpu), parts


@pytest.mark.parametrize("strategy", ["ring", "resident", "ordered"])
def test_gpu_norm_accuracy_and_single_launch_parity(gpu, strategy):
    """Single-launch encode (in-kernel norm hand-off; every strategy) vs oracle given the GPU norm."""
    for s in (3, 4, 8):
        plan, x, parts = _mixed_arena(gpu, MIXED_SIZES, seed=10 * s)
        prev = plan.strategy
        plan.set_encode_strategy(strategy)
        u_host = np.zeros(plan.arena_end, np.float32)
        stream = oracle.MTStream(7 + s)
        for o, n in zip(plan.offsets, plan.sizes):
            u_host[o:o + n] = stream.draw(n)
        q, norms = plan.qsgd_encode(x, s, u=_dev(u_host, gpu))
        plan.check()
        norms_h = norms.cpu().numpy()
        qh = q.cpu().numpy()
        for i, (o, n, p) in enumerate(zip(plan.offsets, plan.sizes, parts)):
            ref = float(np.sqrt(np.sum(p.astype(np.float64) ** 2)))
            assert norms_h[i] == pytest.approx(ref, rel=NORM_RTOL), (s, n)
            want = _oracle_q(p, s, float(norms_h[i]), u_host[o:o + n])
            assert qh[o:o + n].tobytes() == want.tobytes(), (s, n)
        # norm-only entry point returns the identical norms
        n2 = plan.qsgd_norms(x)
        if strategy != "ring":  # the ring folds 64 KiB chunk partials, qsgd_norms 256 KiB items
            assert torch.equal(n2, norms)
        else:
            torch.testing.assert_close(n2, norms, rtol=2e-6, atol=0)
        plan.set_encode_strategy(prev)  # restore the default on the cached plan


def test_strategies_agree_and_fallback_exact(gpu):
    """Resident vs ordered encoders give identical bits; a non-co-resident grid (forced) falls back exactly."""
    sizes = [5, 1 << 24, 70000, (1 << 24) + 3, 1000]  # > capacity slabs: two-pass tensors inside resident
    plan = codec.Plan.get(sizes, device=gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    x = torch.randn(plan.arena_end, device=gpu, generator=g)
    prev = plan.strategy
    plan.set_encode_strategy("resident")
    q1, n1 = plan.qsgd_encode(x, 4, seed=3, offset=1)
    assert plan.check()
    plan.set_encode_strategy("ordered")
    q2, n2 = plan.qsgd_encode(x, 4, seed=3, offset=1)
    assert plan.check()
    # the strategies fold partials over different slab sizes: norms agree to rounding, and each
    # payload is exact for its own norm (checked against the oracle elsewhere)
    torch.testing.assert_close(n1, n2, rtol=2e-6, atol=0)
    plan.set_encode_strategy("ring")
    q3, n3 = plan.qsgd_encode(x, 4, seed=3, offset=1)
    assert plan.check()
    torch.testing.assert_close(n3, n2, rtol=2e-6, atol=0)
    plan.set_encode_strategy(prev)  # the default, on the cached plan
    for strategy in ("ring", "resident", "ordered"):
        small = codec.Plan([40000] * 8 + [1 << 20], device=gpu)
        small.set_encode_strategy(strategy)
        xs = torch.randn(small.arena_end, device=gpu, generator=g)
        qa, na = small.qsgd_encode(xs, 4, seed=9)
        assert small.check()
        small.set_resident_capacity(0, wait_us=1)  # 1 us norm waits: most items must recompute the norm
        qb, nb = small.qsgd_encode(xs, 4, seed=9)
        assert small.check() is False  # fallback taken, results exact
        assert torch.equal(na, nb)
        for o, n in zip(small.offsets, small.sizes):
            assert torch.equal(qa[o:o + n], qb[o:o + n])


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("hold", [0, 3])
def test_ring_configs_match_oracle(gpu, cfg, hold):
    """Every ring configuration, with large tensors held (hold=0) or taking two passes (hold=3
    chunks), gives the oracle's payload for its own norms, in both draw modes."""
    plan, x, parts = _mixed_arena(gpu, MIXED_SIZES + [300_000, 1 << 20], seed=31 + cfg)
    plan = codec.Plan(plan.sizes, device=gpu)
    plan.set_encode_strategy("ring")
    plan.set_ring(cfg=cfg, hold_max=hold)
    info = plan.ring_info
    assert info["cfg"] == cfg and (hold == 0 or info["two_pass_tensors"] >= 1)
    s = 4
    q, norms = plan.qsgd_encode(x, s, seed=11, offset=5)
    assert plan.check()
    qh, nh = q.cpu().numpy(), norms.cpu().numpy()
    for t, (o, n, p) in enumerate(zip(plan.offsets, plan.sizes, parts)):
        ref = float(np.sqrt(np.sum(p.astype(np.float64) ** 2)))
        assert nh[t] == pytest.approx(ref, rel=NORM_RTOL)
        want = _oracle_q(p, s, float(nh[t]), oracle.philox_uniforms(11, 5, t, n))
        assert qh[o:o + n].tobytes() == want.tobytes(), (t, n)
    u_host = np.random.default_rng(cfg).random(plan.arena_end, dtype=np.float32)
    q8, n8 = plan.qsgd_encode(x, 8, u=_dev(u_host, gpu))
    assert torch.equal(n8, norms)
    q8h = q8.cpu().numpy()
    for t, (o, n, p) in enumerate(zip(plan.offsets, plan.sizes, parts)):
        want = _oracle_q(p, 8, float(nh[t]), u_host[o:o + n])
        assert q8h[o:o + n].tobytes() == want.tobytes(), (t, n)


def test_philox_mode_matches_numpy_philox(gpu):
    s, seed, offset = 4, 0x1234_5678_9ABC, 17
    plan, x, parts = _mixed_arena(gpu, MIXED_SIZES, seed=77)
    q, norms = plan.qsgd_encode(x, s, seed=seed, offset=offset)
    plan.check()
    qh, nh = q.cpu().numpy(), norms.cpu().numpy()
    for t, (o, n, p) in enumerate(zip(plan.offsets, plan.sizes, parts)):
        u = oracle.philox_uniforms(seed, offset, t, n)
        want = _oracle_q(p, s, float(nh[t]), u)
        assert qh[o:o + n].tobytes() == want.tobytes(), n
    # deterministic, and the call offset changes the draws (padding between tensors is never written)
    q2, n2 = plan.qsgd_encode(x, s, seed=seed, offset=offset)
    assert torch.equal(norms, n2)
    q3, _ = plan.qsgd_encode(x, s, seed=seed, offset=offset + 1)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(q[o:o + n], q2[o:o + n])
    big = int(np.argmax(plan.sizes))
    o, n = plan.offsets[big], plan.sizes[big]
    assert not torch.equal(q[o:o + n], q3[o:o + n])


def test_alpha_fused_client_weighting(gpu):
    plan, x, parts = _mixed_arena(gpu, [5000, 70000], seed=5)
    alpha = 37.0
    q1, n1 = plan.qsgd_encode(x, 4, alpha=alpha, seed=9)
    q2, n2 = plan.qsgd_encode(x * alpha, 4, seed=9)
    assert torch.equal(n1, n2)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(q1[o:o + n], q2[o:o + n])


def test_decode_accumulate_and_levels(gpu):
    plan, x, _ = _mixed_arena(gpu, [333, 20000], seed=2)
    q, norms = plan.qsgd_encode(x, 3, seed=1)
    y = plan.qsgd_decode(q, 8, 8, norms)
    acc = torch.ones_like(y) * 0.5
    plan.qsgd_decode(q, 8, 8, norms, y_out=acc, accumulate=True)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(acc[o:o + n], y[o:o + n] + 0.5)
    # non power-of-two level on the wire: fl32(fl32(norm*q)/level)
    y10 = plan.qsgd_decode(q, 8, 10, norms).cpu()
    qc, nc = q.cpu(), norms.cpu()
    for t, (o, n) in enumerate(zip(plan.offsets, plan.sizes)):
        want = oracle.qsgd_dequantize(qc[o:o + n], float(nc[t]), 10, (n,))
        assert y10[o:o + n].numpy().tobytes() == want.numpy().tobytes()


def test_int32_payload_width(gpu):
    plan, x, parts = _mixed_arena(gpu, [4099, 50000], seed=8)
    q, norms = plan.qsgd_encode(x, 8, seed=3)
    assert q.dtype == torch.int32
    y = plan.qsgd_decode(q, 32, 256, norms)
    for o, n in zip(plan.offsets, plan.sizes):  # tensor ranges (the arena padding is never written)
        assert torch.isfinite(y[o:o + n]).all()


def test_div(gpu):
    y = torch.randn(12345, device=gpu)
    ref = (y.cpu() / 7.0).numpy()
    codec.div_(y, 7.0)
    assert y.cpu().numpy().tobytes() == ref.tobytes()


def test_bad_arguments_raise(gpu):
    plan = codec.Plan.get([100], device=gpu)
    with pytest.raises(ValueError):
        plan.qsgd_encode(torch.zeros(50, device=gpu), 4)  # shorter than the plan
    with pytest.raises(ValueError):
        plan.qsgd_encode(torch.zeros(100, device=gpu), 31)
    with pytest.raises(ValueError):
        plan.qsgd_decode(torch.zeros(100, dtype=torch.int8, device=gpu), 16, 4, torch.ones(1, device=gpu))


@pytest.mark.parametrize("cfg", ["resnet18"])
@pytest.mark.parametrize("bits", [3, 4, 8])
def test_full_config_parity_mt_stream(gpu, cfg, bits):
    """Whole R18 update arena (BASELINE config 2: "8-level" = s=3, the presets' s=4, the base
    default s=8 with an int32 wire), reference MT19937 stream, GPU norms: payload and decoded
    floats bit-exact vs the oracle per tensor."""
    named = shapes.model_shapes(cfg)
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=gpu)
    torch.manual_seed(0)
    x_host = torch.zeros(plan.arena_end)
    for o, n in zip(plan.offsets, sizes):
        x_host[o:o + n] = torch.randn(n) * 1e-3
    x = x_host.to(gpu)
    norms = plan.qsgd_norms(x)
    nh = norms.cpu().numpy()
    stream = oracle.MTStream(1234)
    u_host = np.zeros(plan.arena_end, np.float32)
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        if nh[t] != 0:
            u_host[o:o + n] = stream.draw(n)
    q, _ = plan.qsgd_encode(x, bits, u=_dev(u_host, gpu), norm_in=norms)
    L = 2**bits
    y = plan.qsgd_decode(q, 8 if L <= 127 else 32, L, norms)
    qh = q.cpu().numpy()
    yh = y.cpu().numpy()
    xh = x_host.numpy()
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        ref = float(np.sqrt(np.sum(xh[o:o + n].astype(np.float64) ** 2)))
        assert nh[t] == pytest.approx(ref, rel=NORM_RTOL)
        want = _oracle_q(xh[o:o + n], bits, float(nh[t]), u_host[o:o + n])
        assert qh[o:o + n].tobytes() == want.tobytes(), t
        want_y = oracle.qsgd_dequantize(torch.from_numpy(want), float(nh[t]), L, (n,)).numpy()
        assert yh[o:o + n].tobytes() == want_y.tobytes(), t


@pytest.mark.parametrize("cfg,s", [("llama400m", 4), ("llama150m", 4), ("llama150m", 8)])
def test_full_config_properties(gpu, cfg, s):
    """Full-size arenas: size-independent properties + exact oracle spot checks on 3 tensors.
    llama150m s=4 is the bench's other_configs arena; every encode here takes the bracketed
    encoder (s = 8, the int32 wire, through its wide-level variant: plan.last_encoder is asserted),
    and every tensor of each configuration is pinned to the oracle in test_gpu_headline_pin.py.
    The ring's int32-wire path is covered with wide levels off (test_full_config_ring_int32)."""
    named = shapes.model_shapes(cfg)
    sizes = [shapes.numel(sh) for _, sh in named]
    plan = codec.Plan.get(sizes, device=gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(0)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    seed, off = 42, 3
    q, norms = plan.qsgd_encode(x, s, seed=seed, offset=off)
    plan.check()
    assert plan.last_encoder == "bracket", (cfg, s)
    L = 2**s
    width = 8 if L <= 127 else 32
    y = plan.qsgd_decode(q, width, L, norms)
    nh = norms.cpu()
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        xs, qs, ys = x[o:o + n], q[o:o + n].to(torch.int64), y[o:o + n]
        ref = torch.linalg.vector_norm(xs.double()).item()
        assert nh[t].item() == pytest.approx(ref, rel=NORM_RTOL)
        lvl = xs.double().abs() / nh[t].double() * L
        mag = qs.abs().double()
        assert bool(((mag - lvl).abs() < 1.0 + 1e-4).all()), t           # q in {floor, floor+1}
        assert bool((torch.sign(qs) * torch.sign(xs).to(torch.int64) >= 0).all()), t
        step = nh[t].item() / L
        assert bool(((ys.double() - xs.double()).abs() <= step * (1 + 1e-5)).all()), t
        if n >= 1 << 20:  # unbiasedness: mean error in level units ~ N(0, <=0.5/sqrt(n))
            m = ((ys.double() - xs.double()) / step).mean().item()
            assert abs(m) < 8.0 / np.sqrt(n), (t, m)
    xh = x.cpu().numpy()
    qh = q.cpu().numpy()
    for t in (1, len(sizes) // 2, len(sizes) - 1):
        o, n = plan.offsets[t], sizes[t]
        u = oracle.philox_uniforms(seed, off, t, n)
        want = _oracle_q(xh[o:o + n], s, float(nh[t]), u)
        assert qh[o:o + n].tobytes() == want.tobytes(), t


def test_full_config_ring_int32(gpu):
    """The ring encoder's int32 wire on a bracketed plan (wide levels off: s = 8 goes to the ring):
    every tensor of Llama-150M equals the oracle given the norm."""
    named = shapes.model_shapes("llama150m")
    sizes = [shapes.numel(sh) for _, sh in named]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_wide_levels(False)
    g = torch.Generator(device=gpu).manual_seed(1)
    x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
    seed, off, s = 7, 2, 8
    q, norms = plan.qsgd_encode(x, s, seed=seed, offset=off)
    plan.check()
    assert plan.last_encoder == "ring"
    xh, qh, nh = x.cpu().numpy(), q.cpu().numpy(), norms.cpu()
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        u = oracle.philox_uniforms(seed, off, t, n)
        assert qh[o:o + n].tobytes() == _oracle_q(xh[o:o + n], s, float(nh[t]), u).tobytes(), t
