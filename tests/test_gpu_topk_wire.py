"""Batched Top-K wire path (round 4): encode_updates_dict / decode_updates_dict /
decode_updates_into / DeviceAggregator.accumulate_layers over whole messages, against the
reference's golden outputs, the oracle and the per-layer path (global_grpc_compression.py:84-98,
140-160, 207-223; global_grpc_server.py:147-153; global_grpc_client.py:98-111)."""

import numpy as np
import pytest
import torch

import oracle
from omnifed_amd import codec
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    build_global_compressor,
    decode_layer_tensor,
    decode_updates_dict,
    decode_updates_into,
    encode_layer_state,
    encode_updates_dict,
    topk_layer_from_payload,
)
from omnifed_amd.hybrid.compression import TopKCompression

pytestmark = pytest.mark.gpu


def _layer(golden, key):
    L = pb.LayerState()
    L.ParseFromString(golden[key].tobytes())
    return L


def test_encode_updates_dict_topk_golden_error_feedback(gpu, golden, golden_index):
    """The reference's Top-K goldens driven through the batched dict encode: per ratio, every
    golden tensor of that ratio in ONE dict, 3 error-feedback calls.  Index sets equal the
    reference's, bytes equal where torch's order is defined, residuals byte-exact, and every
    LayerState byte-identical to the per-layer path's (a second compressor)."""
    by_ratio = {}
    for c in golden_index["topk"]:
        by_ratio.setdefault(c["ratio"], []).append(c)
    for ratio, cases in by_ratio.items():
        batched = TopKCompression(device=gpu, compress_ratio=ratio)
        single = TopKCompression(device=gpu, compress_ratio=ratio)
        for call in range(3):
            upd = {f"w{c['id']}": torch.from_numpy(golden[f"topk/{c['id']}/{call}/x"]).to(gpu).reshape(c["shape"])
                   for c in cases}
            layers = encode_updates_dict(upd, batched)
            per_layer = [encode_layer_state(n, t, single) for n, t in upd.items()]
            for L, P, c in zip(layers, per_layer, cases):
                key = f"topk/{c['id']}/{call}"
                assert L.SerializeToString() == P.SerializeToString(), key
                G = _layer(golden, key + "/layer")
                G.layer_name = L.layer_name  # the fixture encoded every case under the name "w"
                gidx = np.frombuffer(G.indices_data, np.int64)
                gval = np.frombuffer(G.values_data, np.float32)
                ih = np.frombuffer(L.indices_data, np.int64)
                vh = np.frombuffer(L.values_data, np.float32)
                assert set(ih.tolist()) == set(gidx.tolist()), key
                n, k = c["n"], len(gidx)
                if k * 64 <= n and len(np.unique(np.abs(gval))) == len(gval):
                    assert L.SerializeToString() == G.SerializeToString(), key
                else:
                    assert np.array_equal(vh[np.argsort(ih)], gval[np.argsort(gidx)]), key
                res = batched.residual.residuals[f"w{c['id']}"].cpu().numpy()
                assert res.tobytes() == golden[key + "/residual"].tobytes(), key
                assert res.tobytes() == single.residual.residuals[f"w{c['id']}"].cpu().numpy().tobytes(), key


def _model(gpu, seed, sizes=((64, 33), (4099,), (1,), (300, 301), (7,), (1 << 20,))):
    g = torch.Generator(device=gpu).manual_seed(seed)
    return {f"p{i}": torch.randn(*s, device=gpu, generator=g) * 1e-3 for i, s in enumerate(sizes)}


def test_topk_batched_equals_per_layer_weighted_mixed_state(gpu):
    """Weighted batched encode over 3 calls = the per-layer path byte for byte, including a dict
    where some names already have a residual and others are new (the -0.0 fill), a residual
    replaced by the caller (copied into the arena) and the per-layer path continuing from the
    batched path's residual views."""
    a = TopKCompression(device=gpu, compress_ratio=0.02)
    b = TopKCompression(device=gpu, compress_ratio=0.02)
    names = list(_model(gpu, 0))
    for call in range(4):
        upd = _model(gpu, call + 1)
        if call == 1:  # only some names seen before: mixed residual state
            upd = {n: upd[n] for n in names[:3]}
        if call == 2:
            upd["extra"] = torch.randn(5000, device=gpu)
            a.residual.residuals["p0"] = b.residual.residuals["p0"].clone()  # caller-replaced residual
        w = 3.0 if call % 2 else None
        got = encode_updates_dict(upd, a, weight=w)
        want = [encode_layer_state(n, t, b, weight=w) for n, t in upd.items()]
        for L, P in zip(got, want):
            assert L.SerializeToString() == P.SerializeToString(), (call, L.layer_name)
        for n in upd:
            assert torch.equal(a.residual.residuals[n].reshape(-1), b.residual.residuals[n].reshape(-1)), (call, n)
    # per-tensor compress on a name whose residual is a view of the batched arena
    x = torch.randn(64, 33, device=gpu)
    (va, ia), _ = a.compress(x, "p0")
    (vb, ib), _ = b.compress(x, "p0")
    assert torch.equal(va, vb) and torch.equal(ia, ib)
    assert torch.equal(a.residual.residuals["p0"], b.residual.residuals["p0"])


def test_topk_shared_arena_input_is_not_copied(gpu):
    """Tensors that are views of one arena in the plan's layout are encoded in place (the PS's
    average arena): same bytes as separate tensors."""
    sizes = [1000, 70000, 33]
    plan = codec.Plan.get(sizes, device=gpu)
    arena = torch.randn(plan.arena_end, device=gpu)
    views = {f"t{i}": arena[o:o + n] for i, (o, n) in enumerate(zip(plan.offsets, sizes))}
    copies = {k: v.clone() for k, v in views.items()}
    a = TopKCompression(device=gpu, compress_ratio=0.05)
    b = TopKCompression(device=gpu, compress_ratio=0.05)
    la = encode_updates_dict(views, a)
    lb = encode_updates_dict(copies, b)
    assert [L.SerializeToString() for L in la] == [L.SerializeToString() for L in lb]
    assert torch.equal(arena[plan.offsets[1]:plan.offsets[1] + sizes[1]], copies["t1"])  # input untouched


def _topk_message(gpu, seed=3, ratio=0.01):
    comp = TopKCompression(device=gpu, compress_ratio=ratio)
    upd = _model(gpu, seed)
    return upd, encode_updates_dict(upd, comp)


@pytest.mark.parametrize("placement", ["cuda", None])
def test_decode_updates_dict_topk_batched(gpu, placement):
    """One batched decode of a whole Top-K message = the reference's zero-filled dense decode
    (oracle.topk_desparse) per layer, bit for bit, on the requested placement; a mixed message
    (QSGD + Top-K + dense layers) decodes each layer as decode_layer_tensor does."""
    upd, layers = _topk_message(gpu)
    out = decode_updates_dict(layers, device=placement)
    for L in layers:
        v = torch.from_numpy(np.frombuffer(L.values_data, np.float32).copy())
        i = torch.from_numpy(np.frombuffer(L.indices_data, np.int64).copy())
        want = oracle.topk_desparse(v, i, int(np.prod(L.original_shape))).view(tuple(L.original_shape))
        got = out[L.layer_name]
        assert got.device.type == ("cuda" if placement else "cpu")
        assert got.cpu().numpy().tobytes() == want.numpy().tobytes(), L.layer_name
    q = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
    mixed = encode_updates_dict({"qa": torch.randn(5000, device=gpu)}, q) + layers[:3]
    dense = pb.layer_state(layer_name="d")
    dense.param_shape.extend([3])
    dense.param_update.extend([1.0, -2.0, 0.5])
    mixed.append(dense)
    out = decode_updates_dict(mixed, device="cuda")
    for L in mixed:
        assert torch.equal(out[L.layer_name].cpu(), decode_layer_tensor(L).cpu()), L.layer_name


def test_decode_topk_negative_and_out_of_range_indices(gpu):
    """numpy's indexing in the reference decoder: an index in [-n, 0) wraps (decoded at i + n), one
    outside [-n, n) raises IndexError — in the batched decoder, in the PS accumulate (before the
    accumulator is touched) and in the client downlink overlay (before any target is written)."""
    from omnifed_amd.ps import DeviceAggregator

    n1, n2 = 1000, 3000
    L1 = topk_layer_from_payload("a", (n1,), np.array([1.5, -2.0, 3.0], np.float32), np.array([-1, 5, -1000], np.int64))
    L2 = topk_layer_from_payload("b", (n2,), np.array([4.0], np.float32), np.array([2999], np.int64))
    out = decode_updates_dict([L1, L2], device="cuda")
    want = np.zeros(n1, np.float32)
    want[[-1, 5, -1000]] = [1.5, -2.0, 3.0]
    assert out["a"].cpu().numpy().tobytes() == want.tobytes()
    assert float(out["b"][2999]) == 4.0 and int(torch.count_nonzero(out["b"])) == 1
    bad = topk_layer_from_payload("b", (n2,), np.array([4.0, 1.0], np.float32), np.array([7, 3000], np.int64))
    with pytest.raises(IndexError):
        decode_updates_dict([L1, bad], device="cuda")
    agg = DeviceAggregator([("a", (n1,)), ("b", (n2,))], device=gpu)
    agg.accumulate_layers([L1, L2], 2)
    before = agg.acc.clone()
    with pytest.raises(IndexError):
        agg.accumulate_layers([L1, bad], 3)
    assert torch.equal(agg.acc, before) and agg.update_count == 1
    targets = {"a": torch.ones(n1, device=gpu), "b": torch.ones(n2, device=gpu)}
    with pytest.raises(IndexError):
        decode_updates_into([L1, bad], targets)
    assert bool(torch.all(targets["a"] == 1)) and bool(torch.all(targets["b"] == 1))


def test_ps_accumulate_topk_batched_equals_reference_servicer(gpu):
    """Three clients' Top-K updates accumulated by the PS (one scatter-add launch per client) then
    averaged = the reference servicer's `acc += decode` / total_samples (oracle, fp32 CPU), bit for
    bit — with one client's message missing a tensor and one sending its layers out of order."""
    from omnifed_amd.ps import DeviceAggregator

    shapes = [("p0", (64, 33)), ("p1", (4099,)), ("p2", (1,)), ("p3", (300, 301))]
    msgs, samples = [], [5, 11, 3]
    for c in range(3):
        comp = TopKCompression(device=gpu, compress_ratio=0.03)
        g = torch.Generator(device=gpu).manual_seed(40 + c)
        upd = {n: torch.randn(*s, device=gpu, generator=g) for n, s in shapes}
        if c == 1:
            upd.pop("p1")
        layers = encode_updates_dict(upd, comp)
        if c == 2:
            layers = layers[::-1]
        msgs.append(layers)
    agg = DeviceAggregator(shapes, device=gpu)
    for m, ns in zip(msgs, samples):
        agg.accumulate_layers(m, ns)
    out = agg.apply()
    for name, shape in shapes:
        acc = torch.zeros(int(np.prod(shape)))
        for m in msgs:
            for L in m:
                if L.layer_name == name:
                    v = torch.from_numpy(np.frombuffer(L.values_data, np.float32).copy())
                    i = torch.from_numpy(np.frombuffer(L.indices_data, np.int64).copy())
                    acc += oracle.topk_desparse(v, i, acc.numel())
        want = (acc / sum(samples)).reshape(shape)
        assert out[name].cpu().numpy().tobytes() == want.numpy().tobytes(), name


@pytest.mark.parametrize("shared", [False, True])
def test_decode_updates_into_topk_batched(gpu, shared):
    """Client downlink of a Top-K message: every target = the reference's overlay on param.data,
    byte for byte, for separate parameter tensors and for parameters that are views of one arena."""
    upd, layers = _topk_message(gpu, seed=9, ratio=0.05)
    names = list(upd)
    if shared:
        plan = codec.Plan.get([upd[n].numel() for n in names], device=gpu)
        arena = torch.randn(plan.arena_end, device=gpu)
        targets = {n: arena[o:o + upd[n].numel()].view(upd[n].shape) for n, o in zip(names, plan.offsets)}
    else:
        targets = {n: torch.randn(*upd[n].shape, device=gpu) for n in names}
    bases = {n: t.cpu().clone() for n, t in targets.items()}
    decode_updates_into(layers, targets)
    for L in layers:
        flat = bases[L.layer_name].numpy().reshape(-1).copy()
        flat[np.frombuffer(L.indices_data, np.int64)] = np.frombuffer(L.values_data, np.float32)
        assert targets[L.layer_name].cpu().numpy().reshape(-1).tobytes() == flat.tobytes(), L.layer_name


def test_topk_decode_counts_modes_and_absent_tensors(gpu):
    """omf_topk_decode_counts directly: zero counts (absent tensors) leave mode-0 output zero and
    modes 1/2 untouched; all three modes equal a per-tensor reference scatter."""
    sizes = [5000, 70000, 17, 200000]
    plan = codec.Plan.get(sizes, device=gpu)
    counts = [50, 0, 3, 2000]
    g = torch.Generator().manual_seed(2)
    vals, idxs = [], []
    for n, k in zip(sizes, counts):
        idxs.append(torch.randperm(n, generator=g)[:k])
        vals.append(torch.randn(k, generator=g))
    v = torch.cat(vals).to(gpu)
    ix = torch.cat(idxs).to(gpu)
    base = torch.randn(plan.arena_end, generator=g)
    for mode in (0, 1, 2):
        y = None if mode == 0 else base.to(gpu)
        y = plan.topk_decode_counts(counts, v, ix, y=y, mode=mode)
        want = torch.zeros(plan.arena_end) if mode == 0 else base.clone()
        for o, vv, ii in zip(plan.offsets, vals, idxs):
            if mode == 2:
                want[o + ii] = want[o + ii] + vv
            else:
                want[o + ii] = vv
        yh = y.cpu()
        for o, n in zip(plan.offsets, sizes):
            assert yh[o:o + n].numpy().tobytes() == want[o:o + n].numpy().tobytes(), mode
    with pytest.raises(ValueError):
        plan.topk_decode_counts([50, 0, 18, 2000], v, ix)  # 18 values for a 17-element tensor


def test_topk_wire_full_llama400m_equals_per_layer(gpu):
    """The bench's arena through the drop-in: the batched encode_updates_dict of the whole
    Llama-400M update (k = 1 %, weighting fused, two error-feedback calls) equals the per-layer
    encode_layer_state loop byte for byte, and the batched decode_updates_dict / PS accumulate of
    that message equal the per-layer decodes, bit for bit."""
    from omnifed_amd import shapes
    from omnifed_amd.ps import DeviceAggregator

    named = shapes.model_shapes("llama400m")
    g = torch.Generator(device=gpu).manual_seed(1000)
    a = TopKCompression(device=gpu, compress_ratio=0.01)
    b = TopKCompression(device=gpu, compress_ratio=0.01)
    for call in range(2):
        upd = {n: torch.randn(s, device=gpu, generator=g) * 1e-3 for n, s in named}
        got = encode_updates_dict(upd, a, weight=3.0)
        want = [encode_layer_state(n, t, b, weight=3.0) for n, t in upd.items()]
        for L, P in zip(got, want):
            assert L.SerializeToString() == P.SerializeToString(), (call, L.layer_name)
        del upd
    out = decode_updates_dict(got, device="cuda")
    agg = DeviceAggregator(named, device=gpu)
    agg.accumulate_layers(got, 3)
    for L in got:
        ref = decode_layer_tensor(L, device="cuda")
        assert torch.equal(out[L.layer_name], ref), L.layer_name
        assert torch.equal(agg._slice(L.layer_name), ref.reshape(-1)), L.layer_name
