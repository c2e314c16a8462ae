"""Top-K codec, PS aggregate-after-decode and the wire layer on the GPU, against the reference's golden outputs."""

import numpy as np
import pytest
import torch

import oracle
from inputs import exact_input
from omnifed_amd import codec
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    build_global_compressor,
    decode_layer_tensor,
    encode_layer_state,
    encode_updates_dict,
)
from omnifed_amd.hybrid.compression import TopKCompression, layerwise_decompress

pytestmark = pytest.mark.gpu


def _layer(golden, key):
    L = pb.LayerState()
    L.ParseFromString(golden[key].tobytes())
    return L


def test_topk_golden_error_feedback(gpu, golden, golden_index):
    """3 successive calls per name: residual, values_data and indices_data bit-exact (the
    reference's order, ties included: tie_order="torch")."""
    for c in golden_index["topk"]:
        comp = TopKCompression(device=gpu, compress_ratio=c["ratio"])
        n = c["n"]
        for call in c["calls"]:
            key = f"topk/{c['id']}/{call}"
            x = torch.from_numpy(golden[key + "/x"]).to(gpu)
            (vals, idx), ctx = comp.compress(x, "w")
            G = _layer(golden, key + "/layer")
            gidx = np.frombuffer(G.indices_data, np.int64)
            gval = np.frombuffer(G.values_data, np.float32)
            ih, vh = idx.cpu().numpy(), vals.cpu().numpy()
            assert ih.tobytes() == gidx.tobytes(), (key, n)
            assert vh.tobytes() == gval.tobytes(), (key, n)
            res = comp.residual.residuals["w"].cpu().numpy()
            assert res.tobytes() == golden[key + "/residual"].tobytes(), key
            dec = comp.decompress((vals, idx), ctx).cpu().numpy()
            assert dec.tobytes() == golden[key + "/dec_zero"].tobytes(), key
            # overlay decode (client downlink) through the wire layer
            base = torch.from_numpy(golden[key + "/base"])
            ov = decode_layer_tensor(G, base_tensor=base)
            assert ov.numpy().tobytes() == golden[key + "/dec_base"].tobytes(), key


def test_topk_multi_tensor_plan(gpu):
    sizes = [10, 5000, 16384, 16385, 300001, 1 << 20]
    plan = codec.Plan.get(sizes, device=gpu)
    xh = torch.zeros(plan.arena_end)
    for i, (o, n) in enumerate(zip(plan.offsets, sizes)):
        xh[o:o + n] = torch.from_numpy(exact_input(300 + i, n, -7))
    x = xh.to(gpu)
    res = torch.zeros(plan.arena_end, device=gpu)
    for call in range(2):
        values, indices, ks = plan.topk_encode(x, 0.01, residual=res, residual_mode=2 if call == 0 else 1)
        vh, ih = values.cpu().numpy(), indices.cpu().numpy()
        K = 0
        for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
            tp = xh[o:o + n] * (2 if call else 1)  # residual of selected = 0, else x: t' = x + res
            k = ks[t]
            _, ref_idx = torch.topk(tp.abs(), k, sorted=True)
            sel = ih[K:K + k]
            assert set(sel.tolist()) == set(ref_idx.tolist()), (call, t)
            mags = np.abs(vh[K:K + k])
            assert np.all(mags[:-1] >= mags[1:]), (call, t)
            K += k
        # t' for the next call: residual holds x with the selection zeroed; x + residual
        if call == 0:
            rh = res.cpu()
            for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
                kept = rh[o:o + n]
                assert int((kept == 0).sum()) >= ks[t]
            # make call 1's t' simple: residual := x everywhere
            res.copy_(x)


def test_topk_degenerate_ties(gpu):
    """All-equal magnitudes and mostly-zero tensors (k > nonzeros): the reference's bytes
    (torch.topk on the CPU: which zeros complete the selection, and the order), and, with
    tie_order="index", the device's own rule — the lowest-index zeros."""
    n = 70000
    x = torch.zeros(n)
    x[::1000] = 1.0
    plan = codec.Plan.get([n], device=gpu)
    ov, oi = oracle.topk_sparse(x, 0.01)
    values, indices, ks = plan.topk_encode(x.to(gpu), 0.01, tie_order="torch")
    assert indices.cpu().numpy().tobytes() == oi.numpy().tobytes()
    assert values.cpu().numpy().tobytes() == ov.numpy().tobytes()
    values, indices, ks = plan.topk_encode(x.to(gpu), 0.01, tie_order="index")
    ih = indices.cpu().numpy()
    k = ks[0]
    nz = np.arange(0, n, 1000)
    assert set(nz.tolist()) <= set(ih.tolist())
    rest = sorted(set(ih.tolist()) - set(nz.tolist()))
    assert rest == sorted(set(range(n)) - set(nz.tolist()))[: k - len(nz)]
    assert set(oi.tolist()) != set(ih.tolist())  # the two rules differ on this input


def _fmix32(h):
    h = h.astype(np.uint64)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    return h ^ (h >> np.uint64(16))


def _sample_positions(n, t, max_runs):
    """The elements omf_topk.hip's topk_sample reads for tensor t: one aligned run of 16 per
    max(256, ceil(n / max_runs)) elements, at a hashed position."""
    stride = max(256, -(-n // max_runs))
    lo = np.arange(0, n, stride, dtype=np.uint64)
    key = lo ^ np.uint64((t * 0x9E3779B9) & 0xFFFFFFFF)
    span = np.minimum(np.uint64(stride), np.uint64(n) - lo)
    runs = np.maximum(np.uint64(1), span // np.uint64(16))
    start = (lo + np.uint64(16) * (_fmix32(key) % runs)).astype(np.int64)
    pos = (start[:, None] + np.arange(16)[None, :]).reshape(-1)
    return pos[pos < n]


@pytest.mark.parametrize("alpha", [1.0, 3.0])
def test_topk_sampled_threshold_error_feedback(gpu, alpha):
    """Large tensors take the sampled-threshold single pass: over three error-feedback calls
    the selection has the magnitudes of torch.topk's (ties aside), the order is descending,
    and the residual is t' = residual + fl32(alpha x) with the selection zeroed, bit for bit."""
    sizes = [1 << 20, 3 << 20, 5000, 1_000_003, 4096]
    plan = codec.Plan(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(5)
    res = torch.zeros(plan.arena_end, device=gpu)
    ref_res = [torch.zeros(n, device=gpu) for n in sizes]
    for call in range(3):
        x = torch.randn(plan.arena_end, device=gpu, generator=g) * 1e-3
        values, indices, ks = plan.topk_encode(x, 0.01, residual=res, residual_mode=2 if call == 0 else 1,
                                               alpha=alpha)
        K = 0
        for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
            a = x[o:o + n] * torch.tensor(alpha, device=gpu)
            tp = a if call == 0 else ref_res[t] + a
            k = ks[t]
            v, i = values[K:K + k], indices[K:K + k]
            want, _ = torch.topk(tp.abs(), k, sorted=True)
            assert torch.equal(v.abs(), want), (call, t)
            assert torch.equal(v, tp[i]), (call, t)
            r = tp.clone()
            r[i] = 0.0
            assert torch.equal(res[o:o + n], r), (call, t)
            ref_res[t] = r
            K += k


def test_topk_sampled_threshold_redo(gpu):
    """A tensor whose sampled elements are exactly its largest: the sample puts the threshold
    above the k-th magnitude, the pass finds fewer than k candidates, and the tensor is redone
    exactly — the k largest, ties by ascending index."""
    runs = 16384  # the sample size the positions assume
    n = 1 << 25  # 16 Ki runs of 16 = 256 Ki samples < k = 335544
    x = np.ones(n, np.float32)
    sp = _sample_positions(n, 1, runs)
    x[sp] = 10.0
    sizes = [40000, n]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_topk(sample_runs=runs)
    xa = torch.zeros(plan.arena_end)
    xa[plan.offsets[1]:plan.offsets[1] + n] = torch.from_numpy(x)
    xa[:40000] = torch.arange(40000, dtype=torch.float32)
    values, indices, ks = plan.topk_encode(xa.to(gpu), 0.01)
    k = ks[1]
    assert k > len(sp)
    ih = indices[ks[0]:].cpu().numpy()
    vh = values[ks[0]:].cpu().numpy()
    rest = np.setdiff1d(np.arange(n), sp)[: k - len(sp)]
    assert ih.tolist() == sorted(sp.tolist()) + rest.tolist()
    assert np.all(vh[: len(sp)] == 10.0) and np.all(vh[len(sp):] == 1.0)
    assert indices[: ks[0]].cpu().tolist() == list(range(39999, 39999 - ks[0], -1))


def test_layerwise_decompress(gpu):
    n = 1000
    vals = [torch.randn(10), torch.randn(10)]
    ixs = [torch.randperm(n)[:10], torch.randperm(n)[:10]]
    out = layerwise_decompress(vals, ixs, (n,), 2, gpu)
    ref = oracle.layerwise_decompress(vals, ixs, (n,), 2)
    assert out.cpu().numpy().tobytes() == ref.numpy().tobytes()


def test_ps_device_aggregator_golden(gpu, golden, golden_index):
    from omnifed_amd.ps import DeviceAggregator

    for c in golden_index["ps"]:
        reqs = []
        for cl in range(3):
            r = pb.ModelUpdate()
            r.ParseFromString(golden[f"ps/{c['id']}/req/{cl}"].tobytes())
            reqs.append(r)
        named = [(L.layer_name, tuple(L.original_shape) or tuple(L.param_shape)) for L in reqs[0].layers]
        agg = DeviceAggregator(named, device=gpu)
        for r in reqs:
            agg.accumulate_layers(r.layers, r.number_samples)
        out = agg.apply()
        assert agg.total_samples == sum(c["samples"])
        for name in c["names"]:
            want = golden[f"ps/{c['id']}/out/{name}"]
            assert out[name].cpu().numpy().tobytes() == want.tobytes(), (c["scheme"], name)


def test_wire_roundtrip_and_reference_tests(gpu):
    """The reference's own codec tests (tests/test_hybrid_global_grpc_compression.py:16-69), re-expressed."""
    comp = TopKCompression(device="cpu", compress_ratio=0.25)
    x = torch.randn(32)
    (values, indices), ctx = comp.compress(x.clone(), name="layer0")
    assert values.numel() == max(1, int(32 * 0.25))
    assert comp.decompress((values, indices), ctx).shape == x.shape

    comp = TopKCompression(device="cpu", compress_ratio=0.1)
    base = torch.randn(4, 4)
    layer = encode_layer_state("conv.weight", base, comp)
    assert layer.compression_type == "TopKCompression" and len(layer.param_update) == 0
    dec = decode_layer_tensor(layer, base_tensor=base)
    mask = torch.ones(16, dtype=torch.bool)
    mask[torch.from_numpy(np.frombuffer(layer.indices_data, dtype=np.int64).copy())] = False
    assert torch.allclose(dec.reshape(-1)[mask], base.reshape(-1)[mask])

    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4)
    base = torch.randn(8)
    layer = encode_layer_state("fc.weight", base, comp)
    assert layer.compression_type == "QSGDQuantCompression"
    assert layer.values_data and layer.meta_tensor and layer.width == 8 and layer.level == 16
    assert decode_layer_tensor(layer).shape == base.shape


def test_encode_updates_dict_mt_matches_reference_when_norm_agrees(gpu, golden, golden_index):
    """Batched dict encode in parity RNG mode: payload identical to the reference wherever the GPU norm
    equals the reference's fp32 norm; otherwise identical to the oracle given the GPU norm."""
    for c in golden_index["dict"]:
        key = f"dict/{c['s']}"
        upd = {n: torch.from_numpy(golden[f"{key}/in/{n}"]) for n in c["names"]}
        comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=c["s"])
        comp.rng = "mt19937"
        torch.manual_seed(c["seed"])
        layers = encode_updates_dict(upd, comp)
        gpu_norms = [float(np.frombuffer(L.meta_tensor, np.float32)[0]) if L.meta_tensor else None for L in layers]
        want = oracle.qsgd_encode_dict(upd, c["s"], seed=c["seed"], norms=gpu_norms)
        for L, (name, q, norm, width, levels) in zip(layers, want):
            assert L.layer_name == name
            G = _layer(golden, f"{key}/layer/{name}")
            if q is None:
                assert L.compression_type == "" and G.compression_type == ""
                assert L.SerializeToString() == G.SerializeToString()
                continue
            assert L.values_data == q.numpy().tobytes(), name
            if L.meta_tensor == G.meta_tensor:
                assert L.SerializeToString() == G.SerializeToString(), name


def _encode_both_paths(plan, x, ratio, residual0=None, mode=0, alpha=1.0):
    """Top-K encode through the bucket-sort fast path and through the device-wide radix-sort
    fallback (omf_plan_set_topk force_fallback) on the same input."""
    outs = []
    for fb in (0, 1):
        res = residual0.clone() if residual0 is not None else None
        plan.set_topk(fallback=fb)
        try:
            v, i, ks = plan.topk_encode(x, ratio, residual=res, residual_mode=mode, alpha=alpha)
            torch.cuda.synchronize()
        finally:
            plan.set_topk(fallback=0)
        outs.append((v, i, res))
    return outs, ks


@pytest.mark.parametrize("ratio", [0.01, 0.1])
def test_topk_fast_path_equals_fallback_sort(gpu, ratio):
    """The bucket sort (fine-bin histogram, per-bucket LDS counting sort) and the device-wide
    radix sort give the same bytes: values, indices and the error-feedback residual."""
    sizes = [3 << 20, 1000, 1_000_003, 70000, 5 << 20]
    plan = codec.Plan(sizes, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(11)
    x = torch.randn(plan.arena_end, device=gpu, generator=g)
    x[plan.offsets[4]:plan.offsets[4] + sizes[4]] *= torch.rand(sizes[4], device=gpu, generator=g) ** 4  # heavy tail
    r0 = torch.randn(plan.arena_end, device=gpu, generator=g) * 0.1
    (a, b), ks = _encode_both_paths(plan, x, ratio, residual0=r0, mode=1, alpha=2.0)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    assert torch.equal(a[2], b[2])
    K = 0
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        tp = r0[o:o + n] + x[o:o + n] * 2.0
        want, _ = torch.topk(tp.abs(), ks[t], sorted=True)
        assert torch.equal(a[0][K:K + ks[t]].abs(), want), t
        K += ks[t]


def test_topk_clustered_magnitudes_bucket_merge(gpu):
    """Magnitudes repeated in runs of 50 (a sub-bin holds more keys than the counting sort's
    insertion limit, so those buckets are merge sorted): torch.topk's magnitudes, descending,
    ties by ascending index, and the same bytes as the fallback sort."""
    n = 1 << 20
    g = torch.Generator().manual_seed(3)
    levels = torch.rand(n // 50 + 1, generator=g) + 0.5
    xh = levels.repeat_interleave(50)[:n]
    xh = xh[torch.randperm(n, generator=g)] * torch.where(torch.rand(n, generator=g) < 0.5, -1.0, 1.0)
    plan = codec.Plan([n], device=gpu)
    (a, b), ks = _encode_both_paths(plan, xh.to(gpu), 0.01)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    k = ks[0]
    vh, ih = a[0].cpu(), a[1].cpu()
    want, _ = torch.topk(xh.abs(), k, sorted=True)
    assert torch.equal(vh.abs(), want)
    m = vh.abs()
    same = m[:-1] == m[1:]
    assert bool(torch.all(ih[:-1][same] < ih[1:][same]))
    assert torch.equal(vh, xh[ih])


def test_topk_exact_path_many_tensors_and_arena_decode(gpu):
    """A plan of more than 256 tensors takes the exact path (histogram of every t', segmented
    sort): selection = torch.topk's magnitudes in descending order, values = t' at the indices,
    the residual zeroed there; the whole-arena decode (k offsets over > 256 tensors) rebuilds it."""
    g = torch.Generator().manual_seed(21)
    sizes = [int(s) for s in torch.randint(50, 4000, (300,), generator=g)]
    plan = codec.Plan(sizes, device=gpu)
    x = torch.randn(plan.arena_end, generator=g).to(gpu)
    res = torch.zeros(plan.arena_end, device=gpu)
    values, indices, ks = plan.topk_encode(x, 0.05, residual=res, residual_mode=2)
    K = 0
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        k = ks[t]
        tp = x[o:o + n]
        v, i = values[K:K + k], indices[K:K + k]
        want, _ = torch.topk(tp.abs(), k, sorted=True)
        assert torch.equal(v.abs(), want), t
        assert torch.equal(v, tp[i]), t
        r = tp.clone()
        r[i] = 0.0
        assert torch.equal(res[o:o + n], r), t
        K += k
    y = plan.topk_decode_arena(values, indices, 0.05)
    for o, n in zip(plan.offsets, sizes):
        assert torch.equal(y[o:o + n] + res[o:o + n], x[o:o + n])


def test_encode_updates_dict_mt_is_the_reference_bit_for_bit(gpu, golden, golden_index):
    """Parity RNG mode computes each norm with the reference's own op on this host
    (torch.norm of the CPU copy), so every LayerState equals the reference's byte for byte -
    provided this host's torch.norm rounds like the fixture host's (ISA dependent, SURVEY §0.6;
    checked first, skipped otherwise)."""
    for c in golden_index["dict"]:
        key = f"dict/{c['s']}"
        upd = {n: torch.from_numpy(golden[f"{key}/in/{n}"]) for n in c["names"]}
        for n in c["names"]:
            G = _layer(golden, f"{key}/layer/{n}")
            if G.meta_tensor:
                ref = float(np.frombuffer(G.meta_tensor, np.float32)[0])
                if float(torch.norm(upd[n].reshape(-1)).item()) != ref:
                    pytest.skip("this host's torch.norm rounds differently from the fixture host's")
        comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=c["s"])
        comp.rng = "mt19937"
        torch.manual_seed(c["seed"])
        layers = encode_updates_dict(upd, comp)
        for L, n in zip(layers, c["names"]):
            G = _layer(golden, f"{key}/layer/{n}")
            assert L.SerializeToString() == G.SerializeToString(), n
