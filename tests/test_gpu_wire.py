"""Batched wire path on the GPU: decode_updates_dict / decode_updates_into vs the per-layer decoder."""

import numpy as np
import pytest
import torch

import oracle
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    build_global_compressor,
    decode_layer_tensor,
    decode_updates_dict,
    decode_updates_into,
    encode_updates_dict,
)

pytestmark = pytest.mark.gpu

SHAPES = [("w0", (64, 33)), ("b0", (33,)), ("zero", (7, 5)), ("w1", (1000, 17)), ("i", (4,)), ("e", (0,)),
          ("w2", (3, 5, 7, 11))]


def _updates(gpu, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in SHAPES:
        if name == "zero":
            out[name] = torch.zeros(shape)
        elif name == "i":
            out[name] = torch.arange(4, dtype=torch.int64)  # non-float: dense passthrough
        else:
            out[name] = torch.randn(shape, generator=g) * 1e-2
    return {k: v.to(gpu) for k, v in out.items()}


@pytest.mark.parametrize("bits", [4, 8])
def test_batched_decode_equals_per_layer(gpu, bits):
    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=bits, device=gpu)
    layers = encode_updates_dict(_updates(gpu), comp)
    kinds = {L.layer_name: L.compression_type for L in layers}
    assert kinds["w0"] == "QSGDQuantCompression" and kinds["zero"] == "" and kinds["i"] == ""
    ref = {L.layer_name: decode_layer_tensor(L) for L in layers}  # reference placement: CPU
    got = decode_updates_dict(layers)
    assert list(got) == [L.layer_name for L in layers]
    for name, t in got.items():
        assert t.device.type == "cpu" and t.shape == ref[name].shape
        assert t.dtype == ref[name].dtype
        assert np.array_equal(t.numpy().view(np.uint8), ref[name].numpy().view(np.uint8)), name
    got_d = decode_updates_dict(layers, device=gpu)
    for name, t in got_d.items():
        assert t.device == gpu or t.device.type == "cpu" and name == "i"
        assert torch.equal(t.cpu(), ref[name]), name
    # the decoded floats are the oracle's decompress_quantized of each payload
    for L in layers:
        if L.compression_type == "QSGDQuantCompression":
            q = torch.from_numpy(np.frombuffer(L.values_data, np.int8 if L.width == 8 else np.int32).copy())
            norm = float(np.frombuffer(L.meta_tensor, np.float32)[0])
            want = oracle.qsgd_dequantize(q, norm, L.level, tuple(L.original_shape))
            assert got[L.layer_name].numpy().tobytes() == want.numpy().tobytes()


def test_decode_into_targets_and_topk_overlay(gpu):
    upd = _updates(gpu, seed=3)
    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
    layers = encode_updates_dict(upd, comp)
    targets = {n: torch.full_like(t, 7.0) if t.is_floating_point() else torch.zeros_like(t) for n, t in upd.items()}
    decode_updates_into(layers, targets)
    for L in layers:
        want = decode_layer_tensor(L, base_tensor=targets[L.layer_name].clone())
        assert torch.equal(targets[L.layer_name].cpu(), want.cpu().to(targets[L.layer_name].dtype)), L.layer_name
    # Top-K downlink: overlay on the target in place (global_grpc_compression.py:153-156)
    tk = build_global_compressor(enabled=True, scheme="topk", compress_ratio=0.1, device=gpu)
    layers = encode_updates_dict({"w1": upd["w1"]}, tk)
    base = torch.randn_like(upd["w1"])
    want = decode_layer_tensor(layers[0], base_tensor=base.clone())
    decode_updates_into(layers, {"w1": base})
    assert torch.equal(base.cpu(), want.cpu())


def test_batched_decode_errors_in_message_order(gpu):
    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
    layers = encode_updates_dict(_updates(gpu), comp)
    bad = pb.LayerState()
    bad.CopyFrom(layers[0])
    bad.level = 0
    with pytest.raises(ValueError, match="invalid level"):
        decode_updates_dict([layers[1], bad])
    dense = pb.LayerState(layer_name="d")  # no param_shape: the reference raises for it first
    with pytest.raises(ValueError, match="missing param_shape"):
        decode_updates_dict([dense, bad])
    odd = pb.LayerState(layer_name="x", compression_type="Nope")
    with pytest.raises(ValueError, match="Unsupported compression_type"):
        decode_updates_dict([odd])


@pytest.mark.parametrize("strategy,hold", [("ring", 0), ("ring", 1), ("ordered", 0), ("bracket", 0)])
def test_fused_ps_apply_encode(gpu, strategy, hold):
    """avg = acc / total (numpy fp32 division, bit for bit) and its payload = encode(avg) with the
    same draws — in one launch (ring) or divide + encode (other strategies).  hold=1: every
    tensor of more than one ring chunk takes two passes (the second re-reads acc).  In place
    (avg_out is acc) the same average and payload come out of divide + encode."""
    from omnifed_amd import codec

    sizes = [5, 16384, 70001, 1 << 20, 3000]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy(strategy)
    if hold:
        plan.set_ring(hold_max=hold)
        assert plan.ring_info["two_pass_tensors"] >= 2
    g = torch.Generator(device=gpu).manual_seed(9)
    acc = torch.randn(plan.arena_end, device=gpu, generator=g) * 3.0
    total = 7
    avg, q, norms = plan.ps_apply_encode(acc, float(total), 4, seed=21, offset=4)
    assert plan.check()
    want = acc.cpu().numpy() / np.float32(total)
    got = avg.cpu().numpy()
    for o, n in zip(plan.offsets, plan.sizes):
        assert got[o:o + n].tobytes() == want[o:o + n].tobytes()
    q2, n2 = plan.qsgd_encode(torch.from_numpy(want).to(gpu), 4, seed=21, offset=4)
    assert torch.equal(norms, n2)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(q[o:o + n], q2[o:o + n])
    # in place (the PS's accumulator becomes the averaged model): same average, same payload
    acc2 = acc.clone()
    _, q3, n3 = plan.ps_apply_encode(acc2, float(total), 4, avg_out=acc2, seed=21, offset=4)
    assert plan.check()
    assert torch.equal(n3, n2)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(acc2[o:o + n], avg[o:o + n])
        assert torch.equal(q3[o:o + n], q2[o:o + n])
    # a partial overlap of avg_out and acc is refused
    big = torch.zeros(plan.arena_end + 64, device=gpu)
    with pytest.raises(ValueError, match="overlap"):
        plan.ps_apply_encode(big[:plan.arena_end], float(total), 4, avg_out=big[32:32 + plan.arena_end])


def test_device_aggregator_apply_and_encode(gpu):
    from omnifed_amd.ps import DeviceAggregator

    named = [("a", (33, 7)), ("b", (1000,)), ("c", (4, 4, 4))]
    agg = DeviceAggregator(named, device=gpu)
    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=8, device=gpu)
    for seed, ns in ((1, 10), (2, 30)):
        g = torch.Generator().manual_seed(seed)
        u = {n: torch.randn(s, generator=g) for n, s in named}
        agg.accumulate_layers(encode_updates_dict(u, comp), number_samples=ns)
    acc_before = agg.acc.clone()  # the PS sum of decoded updates, in arrival order
    avg, layers = agg.apply_and_encode(comp)
    assert agg.total_samples == 40
    want = acc_before.cpu().numpy() / np.float32(40)
    for (n, s), L in zip(named, layers):
        i = agg.index[n]
        o, k = agg.plan.offsets[i], agg.plan.sizes[i]
        assert avg[n].cpu().numpy().reshape(-1).tobytes() == want[o:o + k].tobytes()
        assert L.layer_name == n and L.compression_type == "QSGDQuantCompression"
        dec = decode_layer_tensor(L)
        norm = float(np.frombuffer(L.meta_tensor, np.float32)[0])
        assert float((dec - avg[n].cpu()).abs().max()) <= norm / L.level * (1 + 1e-6)
