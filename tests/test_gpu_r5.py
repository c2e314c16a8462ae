"""Round-5 robustness of the drop-in's Top-K decode paths.

* An integer base overlaid by ``decode_layer_tensor`` stays exact above 2^24, as the reference's
  numpy overlay does (``dense = base.numpy().copy(); dense[indices] = values``,
  global_grpc_compression.py:150-158 of the reference): only the assigned values are cast.
* A Top-K layer with more values than its tensor has elements (it must repeat indices) is decoded
  with numpy's last-wins rule by both ``decode_updates_dict`` and the PS's ``accumulate_layers``
  (global_grpc_server.py:108-111, 147-153), instead of raising in one and not the other.
"""

import numpy as np
import pytest
import torch

from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import decode_layer_tensor, decode_updates_dict
from omnifed_amd.ps import DeviceAggregator

pytestmark = pytest.mark.gpu


def _topk_layer(name, shape, values, indices):
    L = pb.LayerState()
    L.layer_name = name
    L.compression_type = "TopKCompression"
    L.values_data = np.asarray(values, np.float32).tobytes()
    L.values_dtype = "float32"
    L.indices_data = np.asarray(indices, np.int64).tobytes()
    L.indices_dtype = "int64"
    L.original_shape.extend(list(shape))
    return L


@pytest.mark.parametrize("dtype", [torch.int32, torch.int64])
def test_integer_base_overlay_is_exact(gpu, dtype):
    base = torch.tensor([2**24 + 1, 2**30 + 7, -(2**25) - 3, 5, 6], dtype=dtype)
    L = _topk_layer("w", (5,), [3.75, -2.5], [3, 1])
    out = decode_layer_tensor(L, base_tensor=base)
    want = base.numpy().copy()
    want[np.array([3, 1])] = np.array([3.75, -2.5], np.float32)  # numpy's cast on assignment
    assert out.dtype == dtype and np.array_equal(out.numpy(), want)


def test_topk_layer_with_repeated_indices_last_wins(gpu):
    n = 6
    vals, idx = [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0], [0, 2, 0, 5, 2, 1, 5, 3]  # k = 8 > n
    L = _topk_layer("w", (n,), vals, idx)
    want = np.zeros(n, np.float32)
    want[np.array(idx)] = np.array(vals, np.float32)  # numpy: the last value per index
    got = decode_updates_dict([L])["w"]
    assert np.array_equal(got.numpy(), want)
    agg = DeviceAggregator([("w", (n,)), ("v", (1000,))], device=gpu)
    M = _topk_layer("v", (1000,), [0.5, -1.5], [7, 999])
    agg.accumulate_layers([L, M], number_samples=2)
    acc = agg.acc.cpu().numpy()
    o_w, o_v = agg.plan.offsets
    assert np.array_equal(acc[o_w:o_w + n], want)
    assert acc[o_v + 7] == 0.5 and acc[o_v + 999] == -1.5


# ---------------------------------------------------------------- fused last client

def _oracle_q(x_np, s, norm, u_np):
    import oracle

    q, *_ = oracle.qsgd_quantize(torch.from_numpy(np.ascontiguousarray(x_np)), s, norm=norm,
                                 u=torch.from_numpy(np.ascontiguousarray(u_np)))
    return q.numpy()


@pytest.mark.parametrize("strategy", ["bracket", "ring"])
@pytest.mark.parametrize("width_in", [8, 32])
@pytest.mark.parametrize("keep", ["none", "acc", "other"])
def test_fused_last_client_against_the_oracle(gpu, strategy, width_in, keep):
    """omf_ps_accumulate_apply_encode: sum = acc + fl32(fl32(norm * q) / L) (numpy's fp32 ops), avg =
    sum / total, and per tensor the payload equals the oracle's quantisation of avg given the GPU
    norm and Philox draws; bytes equal to decode-accumulate followed by omf_ps_apply_encode; the sum
    stored where asked (acc_out), acc untouched otherwise."""
    import oracle
    from omnifed_amd import codec

    sizes = [5, 16384, 70001, 1 << 20, 3000, 2_000_000]
    plan = codec.Plan(sizes, device=gpu)
    plan.set_encode_strategy(strategy)
    g = torch.Generator(device=gpu).manual_seed(23 + width_in)
    acc = torch.randn(plan.arena_end, device=gpu, generator=g) * 3.0
    acc0 = acc.clone()
    L_in = 16 if width_in == 8 else 256
    qin = torch.randint(-L_in, L_in + 1, (plan.arena_end,), device=gpu, generator=g,
                        dtype=torch.int8 if width_in == 8 else torch.int32)
    nin = torch.rand(plan.nt, device=gpu, generator=g) * 40.0
    nin[4] = 0.0  # a tensor absent from the last client's message
    total, s, seed, off = 7.0, 3, 1234, 2
    acc_out = {"none": None, "acc": acc, "other": torch.empty_like(acc)}[keep]
    avg, q, norms = plan.ps_accumulate_apply_encode(acc, qin, width_in, L_in, nin, total, s, acc_out=acc_out,
                                                    seed=seed, offset=off)
    assert plan.check()
    assert plan.last_encoder == strategy
    # the two-call path on copies
    acc2 = acc0.clone()
    plan.qsgd_decode(qin, width_in, L_in, nin, y_out=acc2, accumulate=True)
    avg2, q2, n2 = plan.ps_apply_encode(acc2, total, s, seed=seed, offset=off)
    ah, qh, nh = avg.cpu().numpy(), q.cpu().numpy(), norms.cpu().numpy()
    a0, qi, ni = acc0.cpu().numpy(), qin.cpu().numpy(), nin.cpu().numpy()
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        y = (np.float32(ni[t]) * qi[o:o + n].astype(np.float32)) / np.float32(L_in)
        sm = (a0[o:o + n] + y).astype(np.float32)
        a = sm / np.float32(total)
        assert ah[o:o + n].tobytes() == a.tobytes(), t
        ref = float(np.sqrt(np.sum(a.astype(np.float64) ** 2)))
        assert abs(float(nh[t]) - ref) <= 2e-6 * ref, t
        want = _oracle_q(a, s, float(nh[t]), oracle.philox_uniforms(seed, off, t, n))
        assert qh[o:o + n].tobytes() == want.tobytes(), t
        if keep != "none":
            assert acc_out[o:o + n].cpu().numpy().tobytes() == sm.tobytes(), t
        else:
            assert acc[o:o + n].cpu().numpy().tobytes() == a0[o:o + n].tobytes(), t
    assert torch.equal(norms, n2)
    for o, n in zip(plan.offsets, sizes):  # tensor ranges (padding is never promised)
        assert torch.equal(avg[o:o + n], avg2[o:o + n]) and torch.equal(q[o:o + n], q2[o:o + n])


def test_aggregator_last_client_fused_equals_two_calls(gpu):
    """DeviceAggregator.accumulate_apply_encode (the last SendUpdate + the first GetUpdatedModel)
    returns the LayerStates and averages of accumulate_layers followed by apply_and_encode."""
    from omnifed_amd.hybrid.communicator.global_grpc_compression import build_global_compressor, encode_updates_dict

    named = [("a", (300, 1000)), ("b", (1000,)), ("c", (2048, 2048)), ("d", (7,)), ("e", (8192, 4096))]  # >= 2^25: bracketed
    g = torch.Generator(device=gpu).manual_seed(8)
    clients = [{n: torch.randn(s, device=gpu, generator=g) for n, s in named} for _ in range(3)]
    msgs = []
    for c, upd in enumerate(clients):
        comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
        comp.client_id = c
        msgs.append(encode_updates_dict(upd, comp, weight=float(c + 1)))
    A = DeviceAggregator(named, device=gpu)
    B = DeviceAggregator(named, device=gpu)
    assert A.plan.strategy == "bracket"
    srv_a = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
    srv_b = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
    srv_b._instance = srv_a._instance  # the same Philox key
    for m in msgs[:2]:
        A.accumulate_layers(m, number_samples=10)
        B.accumulate_layers(m, number_samples=10)
    avg_a, la = A.accumulate_apply_encode(msgs[2], 10, srv_a)
    assert A.plan.last_encoder == "bracket"
    B.accumulate_layers(msgs[2], number_samples=10)
    avg_b, lb = B.apply_and_encode(srv_b)
    assert A.total_samples == B.total_samples == 30
    assert [L.SerializeToString() for L in la] == [L.SerializeToString() for L in lb]
    for n, _ in named:
        assert torch.equal(avg_a[n], avg_b[n]), n


def test_aggregator_fused_without_sum_marks_the_accumulator_stale(gpu):
    """accumulate_apply_encode(keep_sum=False) leaves the accumulator without the last client's
    term: apply(), apply_and_encode() and a further accumulate raise until reset(); with the
    default keep_sum the accumulator holds the full sum, as accumulate_layers leaves it."""
    from omnifed_amd.hybrid.communicator.global_grpc_compression import build_global_compressor, encode_updates_dict

    named = [("a", (300, 1000)), ("e", (8192, 4096))]
    g = torch.Generator(device=gpu).manual_seed(9)
    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
    msgs = [encode_updates_dict({n: torch.randn(s, device=gpu, generator=g) for n, s in named}, comp)
            for _ in range(2)]
    srv = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=gpu)
    A, B = DeviceAggregator(named, device=gpu), DeviceAggregator(named, device=gpu)
    for agg in (A, B):
        agg.accumulate_layers(msgs[0], number_samples=5)
    A.accumulate_apply_encode(msgs[1], 5, srv)  # keep_sum (default)
    B.accumulate_layers(msgs[1], number_samples=5)
    assert torch.equal(A.acc, B.acc) and A.total_samples == B.total_samples == 10
    C = DeviceAggregator(named, device=gpu)
    C.accumulate_layers(msgs[0], number_samples=5)
    C.accumulate_apply_encode(msgs[1], 5, srv, keep_sum=False)
    for call in (C.apply, lambda: C.apply_and_encode(srv), lambda: C.accumulate_layers(msgs[0], 5)):
        with pytest.raises(RuntimeError, match="reset"):
            call()
    C.reset()
    C.accumulate_layers(msgs[0], number_samples=5)
    assert C.total_samples == 5
