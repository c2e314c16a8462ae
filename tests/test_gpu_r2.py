"""Round-2 GPU tests: ring wait bounds and stream ordering, payload buffer bounds, bf16/fp16
encodes, the Top-K arena decode, and the configs BASELINE.json names (a full ResNet-18 PS
round pinned by the reference servicer, Llama-400M Top-K), all through the HIP C ABI.

Fixtures: tests/golden/golden_r2.npz + golden_r2_index.json (tests/golden/gen_golden_r2.py,
the real reference imported in the build container).
"""

import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

import oracle
from inputs import exact_input, sha
from omnifed_amd import codec, shapes
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    build_global_compressor,
    decode_layer_tensor,
    encode_layer_state,
    encode_updates_dict,
    qsgd_layer_from_payload,
)
from omnifed_amd.hybrid.compression.qsgd import QSGDQuantCompression

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16}


@pytest.fixture(scope="module")
def g2():
    return np.load(os.path.join(HERE, "golden", "golden_r2.npz"))


@pytest.fixture(scope="module")
def g2i():
    with open(os.path.join(HERE, "golden", "golden_r2_index.json")) as f:
        return json.load(f)


def _same_floats(a, b) -> bool:
    """Bit-equal fp32 arrays, except that a NaN matches any NaN (x86 makes inf * 0 the negative
    default NaN, the GPU the positive one)."""
    a, b = np.asarray(a, np.float32).reshape(-1), np.asarray(b, np.float32).reshape(-1)
    same = a.view(np.uint32) == b.view(np.uint32)
    return a.shape == b.shape and bool(np.all(same | (np.isnan(a) & np.isnan(b))))


def _layer(buf):
    L = pb.LayerState()
    L.ParseFromString(np.asarray(buf).tobytes())
    return L


# ---------------------------------------------------------------- ring robustness

@pytest.mark.parametrize("dbg", [2, 3])
def test_ring_debug_timing_modes_complete(gpu, dbg):
    """Ring debug switches 2 (quantisation off: the timing that hung before the ticket fix) and 3
    (norm waits off too) finish, report no timeout, and publish the same norms."""
    sizes = [7, 1000, 16384, 40000, 70001, 3, 1 << 20, 300_000]
    ref = codec.Plan(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(4)
    x = torch.randn(ref.arena_end, device=gpu, generator=g)
    _, n_ref = ref.qsgd_encode(x, 4, seed=1)
    assert ref.check()
    p = codec.Plan(sizes, device=gpu)
    p.set_debug(ring=dbg)  # test hook (omf_plan_set_debug); never read from the environment
    p.set_encode_strategy("ring")
    for hold in (0, 3):
        p.set_ring(hold_max=hold)
        _, nd = p.qsgd_encode(x, 4, seed=1)
        assert p.check()  # completed without OMF_ETIMEOUT
        if not dbg & 1:
            assert torch.equal(nd, n_ref) if hold == 0 else torch.allclose(nd, n_ref, rtol=2e-6, atol=0)


@pytest.mark.parametrize("strategy", ["ordered", "ring", "bracket", "grid"])
def test_encodes_on_two_streams_are_ordered(gpu, strategy):
    """One plan, launches alternating between two streams with no host synchronisation: each
    result equals the sequential one (the plan orders a launch after the previous stream's)."""
    sizes = [5000, 1 << 20, 70001, 3 << 20]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy(strategy)
    g = torch.Generator(device=gpu).manual_seed(8)
    xs = [torch.randn(plan.arena_end, device=gpu, generator=g) for _ in range(4)]
    want = []
    for i, x in enumerate(xs):
        q, n = plan.qsgd_encode(x, 4, seed=5, offset=i)
        want.append((q.clone(), n.clone()))
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)
    outs = []
    for i, x in enumerate(xs):
        st = s1 if i % 2 == 0 else s2
        st.wait_stream(torch.cuda.current_stream(gpu))
        with torch.cuda.stream(st):
            q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=gpu)
            n = torch.empty(plan.nt, dtype=torch.float32, device=gpu)
            plan.qsgd_encode(x, 4, q_out=q, norm_out=n, seed=5, offset=i, stream=st.cuda_stream)
            outs.append((q, n))
    torch.cuda.synchronize()
    assert plan.check()
    for (q, n), (qw, nw) in zip(outs, want):
        assert torch.equal(n, nw)
        for o, m in zip(plan.offsets, plan.sizes):
            assert torch.equal(q[o:o + m], qw[o:o + m])


def test_int8_payload_stays_inside_its_buffer(gpu):
    """An int8 payload is stored in whole dwords: the buffer must hold round_up(arena_end, 4)
    (a shorter one is refused), and nothing past that is written."""
    sizes = [5, 70001, 1003]  # the last tensor ends mid-dword
    plan = codec.Plan(sizes, device=gpu)
    assert plan.payload_elems(8) == (plan.arena_end + 3) // 4 * 4 > plan.arena_end
    x = torch.randn(plan.arena_end, device=gpu) + 1.0
    buf = torch.full((plan.payload_elems(8) + 64,), 0x5A, dtype=torch.int8, device=gpu)
    with pytest.raises(ValueError):
        plan.qsgd_encode(x, 4, q_out=buf[:plan.arena_end], seed=3)
    prev = plan.strategy
    for strategy in ("ring", "ordered", "grid"):
        plan.set_encode_strategy(strategy)
        buf.fill_(0x5A)
        q, norms = plan.qsgd_encode(x, 4, q_out=buf[:plan.payload_elems(8)], seed=3)
        assert plan.check()
        tail = buf[plan.payload_elems(8):].cpu().numpy()
        assert (tail == 0x5A).all(), strategy
        ref = oracle.philox_uniforms(3, 0, 2, sizes[2])
        o = plan.offsets[2]
        want, *_ = oracle.qsgd_quantize(x[o:o + sizes[2]].cpu(), 4, norm=float(norms[2]), u=torch.from_numpy(ref))
        assert q[o:o + sizes[2]].cpu().numpy().tobytes() == want.numpy().tobytes()
    plan.set_encode_strategy(prev)


# ---------------------------------------------------------------- bf16 / fp16 (golden_r2 half/*)

def test_half_goldens_given_the_reference_norm(gpu, g2, g2i):
    """bf16/fp16 tensors (weighted or not): the value-format encoder with the reference's norm
    and MT19937 draws reproduces the reference payload and decoded floats bit for bit."""
    for c in g2i["half"]:
        key = f"half/{c['id']}"
        L = _layer(g2[key + "/layer"])
        if L.compression_type != "QSGDQuantCompression":
            continue
        n, s = c["n"], c["s"]
        fmt = {"bf16": 1, "fp16": 2}[c["dtype"]]
        plan = codec.Plan.get([n], device=gpu)
        x = torch.from_numpy(g2[key + "/x"]).to(gpu)
        u = torch.from_numpy(oracle.mt19937_uniforms(c["seed"], n)).to(gpu)
        norm = np.frombuffer(L.meta_tensor, np.float32)[0]
        nin = torch.tensor([norm], dtype=torch.float32, device=gpu)
        alpha = 1.0 if c["weight"] is None else float(c["weight"])
        q, nout = plan.qsgd_encode(x, s, alpha=alpha, u=u, norm_in=nin, value_format=fmt)
        assert q[:n].cpu().numpy().tobytes() == L.values_data, key
        y = plan.qsgd_decode(q, L.width, L.level, nout)
        assert _same_floats(y[:n].cpu().numpy(), g2[key + "/y"]), key
        # the encoder's own norm is the reference's after the format's rounding
        nn = plan.qsgd_norms(x, alpha=alpha, value_format=fmt)
        ref64 = float(np.sqrt(np.sum(oracle_weighted(g2[key + "/x"], c).astype(np.float64) ** 2)))
        assert np.isinf(norm) or abs(float(nn[0]) - norm) <= 2 ** -7 * abs(norm), (key, float(nn[0]), norm, ref64)


def oracle_weighted(x32, c):
    t = torch.from_numpy(x32).to(DTYPES[c["dtype"]])
    if c["weight"] is not None:
        t = torch.mul(t, c["weight"])
    return t.float().numpy()


def test_half_drop_in_layers(gpu, g2, g2i):
    """The drop-in on a bf16/fp16 device tensor (rng=mt19937, weight=batch_samples): the LayerState
    is the reference's byte for byte whenever the GPU norm rounds to the reference's."""
    same = 0
    for c in g2i["half"]:
        key = f"half/{c['id']}"
        L = _layer(g2[key + "/layer"])
        x = torch.from_numpy(g2[key + "/x"]).to(DTYPES[c["dtype"]]).to(gpu)
        torch.manual_seed(c["seed"])
        comp = QSGDQuantCompression(bit_width=c["s"], rng="mt19937")
        got = encode_layer_state(L.layer_name, x, comp, weight=c["weight"])
        assert got.compression_type == L.compression_type
        if got.meta_tensor == L.meta_tensor:
            assert got.SerializeToString() == L.SerializeToString(), key
            same += 1
        dec = decode_layer_tensor(got)
        assert dec.dtype == torch.float32 and tuple(dec.shape) == tuple(L.original_shape)
    assert same >= len(g2i["half"]) - 3, same


def test_float64_qsgd_and_topk_are_refused(gpu):
    """fp64 is refused by both codecs (fp16 / bf16 Top-K: tests/test_gpu_topk_half.py)."""
    comp = QSGDQuantCompression(bit_width=4)
    with pytest.raises(ValueError, match="float64"):
        encode_layer_state("d", torch.randn(100, dtype=torch.float64, device=gpu), comp)
    tk = build_global_compressor(enabled=True, scheme="topk", compress_ratio=0.1)
    with pytest.raises(ValueError, match="float64"):
        encode_layer_state("h", torch.randn(100, device=gpu).double(), tk)


# ---------------------------------------------------------------- client weighting on the drop-in

def test_weight_equals_multiplying_first(gpu):
    """encode_updates_dict(upd, c, weight=w) == encode_updates_dict(torch.mul(upd, w), c):
    QSGD (one launch, alpha fused), Top-K (fused) and the dense passthrough."""
    g = torch.Generator().manual_seed(5)
    upd = {"a": torch.randn(33, 7, generator=g), "b": torch.randn(1000, generator=g), "z": torch.zeros(9),
           "i": torch.arange(4)}
    upd = {k: v.to(gpu) for k, v in upd.items()}
    w = 48
    for scheme in ("qsgd", "topk", None):
        outs = []
        for weighted in (False, True):
            torch.manual_seed(11)
            comp = None if scheme is None else build_global_compressor(enabled=True, scheme=scheme, bit_width=4,
                                                                       compress_ratio=0.1)
            if comp is not None and scheme == "qsgd":
                comp.rng = "mt19937"
            src = {k: torch.mul(v, w) for k, v in upd.items()} if not weighted else upd
            outs.append(encode_updates_dict(src, comp, weight=w if weighted else None))
        for a, b in zip(*outs):
            assert a.SerializeToString() == b.SerializeToString(), (scheme, a.layer_name)


# ---------------------------------------------------------------- Top-K arena decode (golden_r2 lwd/*)

def _lwd_packed(g2, cid, c, nshapes, gpu):
    vals = np.concatenate([g2[f"lwd/{cid}/vals/{c}/{t}"] for t in range(nshapes)])
    idx = np.concatenate([g2[f"lwd/{cid}/idx/{c}/{t}"] for t in range(nshapes)])
    return torch.from_numpy(vals).to(gpu), torch.from_numpy(idx).to(gpu)


def test_topk_arena_scatter_add_matches_layerwise_decompress(gpu, g2, g2i):
    """Every client's selection decoded into one arena (omf_topk_decode_arena mode 2, rank order)
    then / client_count == the reference's layerwise_decompress, per tensor, bit for bit; and the
    drop-in's layerwise_decompress gives the same."""
    from omnifed_amd.hybrid.compression.core import layerwise_decompress

    for case in g2i["lwd"]:
        cid, clients, ratio = case["id"], case["clients"], case["ratio"]
        shp = [tuple(s) for s in case["shapes"]]
        plan = codec.Plan([int(np.prod(s)) for s in shp], device=gpu)
        assert plan.topk_ks(ratio) == [g2[f"lwd/{cid}/vals/0/{t}"].size for t in range(len(shp))]
        acc = torch.zeros(plan.arena_end, device=gpu)
        for c in range(clients):
            v, ix = _lwd_packed(g2, cid, c, len(shp), gpu)
            plan.topk_decode_arena(v, ix, ratio, y=acc, mode=2)
        codec.div_(acc, float(clients))
        for t, (o, n) in enumerate(zip(plan.offsets, plan.sizes)):
            want = g2[f"lwd/{cid}/out/{t}"]
            assert acc[o:o + n].cpu().numpy().tobytes() == want.tobytes(), (cid, t)
            vals = [torch.from_numpy(g2[f"lwd/{cid}/vals/{c}/{t}"]).to(gpu) for c in range(clients)]
            ixs = [torch.from_numpy(g2[f"lwd/{cid}/idx/{c}/{t}"]).to(gpu) for c in range(clients)]
            got = layerwise_decompress(vals, ixs, shp[t], clients, gpu)
            assert got.reshape(-1).cpu().numpy().tobytes() == want.tobytes(), (cid, t)
        # zero-fill (mode 0) and overlay (mode 1) of one client
        v, ix = _lwd_packed(g2, cid, 0, len(shp), gpu)
        y0 = plan.topk_decode_arena(v, ix, ratio, mode=0)
        base = torch.randn(plan.arena_end, device=gpu)
        y1 = plan.topk_decode_arena(v, ix, ratio, y=base.clone(), mode=1)
        k0 = 0
        for t, (o, n, k) in enumerate(zip(plan.offsets, plan.sizes, plan.topk_ks(ratio))):
            z = torch.zeros(n, device=gpu)
            z[ix[k0:k0 + k]] = v[k0:k0 + k]
            assert torch.equal(y0[o:o + n], z)
            b = base[o:o + n].clone()
            b[ix[k0:k0 + k]] = v[k0:k0 + k]
            assert torch.equal(y1[o:o + n], b)
            k0 += k


# ---------------------------------------------------------------- ResNet-18 PS round (golden_r2 r18)

def test_resnet18_round_replay_pinned_by_reference_servicer(gpu, g2i):
    """BASELINE config 1 on the GPU: two clients weight their ResNet-18 update by batch_samples
    (alpha, fused), encode it with the reference's norms and MT19937 stream (every payload's
    SHA-256 equals the reference's), the PS decode-accumulates both and divides by the total
    (every averaged parameter's SHA-256 equals the reference CentralServerServicer's)."""
    from omnifed_amd.ps import DeviceAggregator

    sys.path.insert(0, os.path.join(HERE, "golden"))
    from gen_golden_r2 import r18_update

    r18 = g2i["r18"]
    named = shapes.model_shapes("resnet18")
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=gpu)
    agg = DeviceAggregator(named, device=gpu)
    for c, (ns, seed, rec) in enumerate(zip(r18["samples"], r18["seeds"], r18["clients"])):
        upd = r18_update(c, named)
        x = torch.zeros(plan.arena_end)
        for (name, _), o, n in zip(named, plan.offsets, sizes):
            x[o:o + n] = upd[name].reshape(-1)
        torch.manual_seed(seed)
        u = torch.zeros(plan.arena_end)
        for o, n in zip(plan.offsets, sizes):  # every tensor has a non-zero norm: draws in order
            u[o:o + n] = torch.rand(n)
        norms = torch.tensor([np.uint32(r["norm_bits"]).view(np.float32) for r in rec], dtype=torch.float32)
        q, nd = plan.qsgd_encode(x.to(gpu), r18["bit_width"], alpha=float(ns), u=u.to(gpu), norm_in=norms.to(gpu))
        qh = q.cpu().numpy()
        layers = []
        for t, ((name, shape), o, n, r) in enumerate(zip(named, plan.offsets, sizes, rec)):
            assert r["ctype"] == "QSGDQuantCompression"
            payload = qh[o:o + n].tobytes()
            assert hashlib.sha256(payload).hexdigest() == r["q_sha"], name
            L = qsgd_layer_from_payload(name, shape, payload, float(norms[t]), 8, 16)
            assert hashlib.sha256(L.SerializeToString()).hexdigest() == r["layer_sha"], name
            layers.append(L)
        agg.accumulate_layers(layers, number_samples=ns)
    avg = agg.apply()
    for name, _ in named:
        assert sha(avg[name].cpu().numpy()) == r18["out_sha"][name], name


def test_accumulate_updates_equals_wire_path(gpu):
    """DeviceAggregator.accumulate_updates (one weighted encode + one decode-accumulate on the
    device) == accumulate_layers(encode_updates_dict(..., weight)) for the same draws."""
    from omnifed_amd.ps import DeviceAggregator

    named = [("a", (33, 7)), ("b", (70001,)), ("c", (4, 4, 4))]
    g = torch.Generator().manual_seed(2)
    ups = [{n: torch.randn(s, generator=g).to(gpu) for n, s in named} for _ in range(2)]
    res = []
    for direct in (False, True):
        agg = DeviceAggregator(named, device=gpu)
        for c, u in enumerate(ups):
            torch.manual_seed(40 + c)
            comp = QSGDQuantCompression(bit_width=4, rng="mt19937")
            if direct:
                agg.accumulate_updates(u, comp, number_samples=10 + c, weight=10 + c)
            else:
                agg.accumulate_layers(encode_updates_dict(u, comp, weight=10 + c), number_samples=10 + c)
        res.append(agg.apply())
    for n, _ in named:
        assert torch.equal(res[0][n], res[1][n]), n


# ---------------------------------------------------------------- Llama-400M Top-K (BASELINE config 5)

def test_llama400m_topk_error_feedback_full_arena(gpu):
    """k = 1 % per tensor over the whole Llama-400M arena, two error-feedback calls: per tensor the
    selected magnitudes are torch.topk's, values are t' at the indices, and the residual is t'
    with the selected slots zeroed, byte for byte."""
    named = shapes.model_shapes("llama400m")
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=gpu)
    ratio = 0.01
    ks = plan.topk_ks(ratio)
    g = torch.Generator(device=gpu).manual_seed(17)
    res = torch.empty(plan.arena_end, device=gpu)
    for call in range(2):
        x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
        tprime = x.clone() if call == 0 else res + x
        vals, idx, _ = plan.topk_encode(x, ratio, residual=res, residual_mode=2 if call == 0 else 1)
        K = 0
        for t, (o, n, k) in enumerate(zip(plan.offsets, sizes, ks)):
            tp = tprime[o:o + n]
            v, ix = vals[K:K + k], idx[K:K + k]
            assert torch.equal(v, tp[ix]), (call, t)
            top = torch.topk(tp.abs(), k, sorted=True).values
            assert torch.equal(v.abs(), top), (call, t)  # descending |t'|: torch's magnitudes exactly
            want = tp.clone()
            want[ix] = 0.0
            assert torch.equal(res[o:o + n], want), (call, t)
            K += k
        del tprime


# ---------------------------------------------------------------- generated-module interop

def test_layer_states_belong_to_the_callers_pb2(gpu, monkeypatch):
    """With a generated global_grpc_pb2 registered under the reference's module name, every
    LayerState the codec builds is that module's, so the caller's ModelUpdate / ModelParameters
    accept them (global_grpc_client.py:75-80, global_grpc_server.py:226-230)."""
    name = pb.REFERENCE_MODULE
    stand_in = pb.schema_module(name)
    monkeypatch.setitem(sys.modules, name, stand_in)
    g = torch.Generator().manual_seed(1)
    upd = {"w": torch.randn(100, 10, generator=g).to(gpu), "z": torch.zeros(5, device=gpu)}
    for scheme in ("qsgd", "topk", None):
        comp = None if scheme is None else build_global_compressor(enabled=True, scheme=scheme, bit_width=4,
                                                                   compress_ratio=0.1)
        layers = encode_updates_dict(upd, comp, weight=3)
        assert all(type(L) is stand_in.LayerState for L in layers)
        msg = stand_in.ModelUpdate(client_id="c", round_number=1, layers=layers, number_samples=3)
        back = stand_in.ModelUpdate()
        back.ParseFromString(msg.SerializeToString())
        dec = {L.layer_name: decode_layer_tensor(L) for L in back.layers}
        assert set(dec) == {"w", "z"}
        stand_in.ModelParameters(round_number=1, layers=layers, is_ready=True)
        with pytest.raises(TypeError):  # the private schema's messages would be refused
            stand_in.ModelUpdate(layers=[pb.LayerState(layer_name="x")])


def test_default_encode_strategy_by_arena_size(gpu):
    """A new plan takes the bracketed single-read encoder for arenas of >= 2^25 elements and the
    single-read ring below."""
    small = codec.Plan([1 << 20, 5000], device=gpu)
    assert small.strategy == "ring"
    big = codec.Plan([1 << 24, 1 << 24, 1000], device=gpu)
    assert big.strategy == "bracket"
