"""Top-K on fp16 / bf16 tensors (round 4): the reference selects, compensates and keeps its residual
in the tensor's dtype (hybrid/compression/topk.py:33-42, core.py:26-37) and sends fp32 values
(global_grpc_compression.py:84-98: astype(float32); a bf16 tensor fails there in .numpy()); its
overlay decode returns the base's dtype (:151-156).  Checked against the reference's own torch op
sequence replayed on the CPU.  Half precision makes equal magnitudes common; the selection —
members at rank k and order — is torch's CPU topk's on the half tensor (tie_order="torch")."""

import numpy as np
import pytest
import torch

from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    decode_layer_tensor,
    decode_updates_into,
    encode_layer_state,
    encode_updates_dict,
    topk_layer_from_payload,
)
from omnifed_amd.hybrid.compression import TopKCompression

pytestmark = pytest.mark.gpu


def _bits(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().view(torch.int16).numpy()


def _rule_topk(t: torch.Tensor, k: int) -> np.ndarray:
    return torch.topk(t.abs(), k, sorted=False).indices.numpy()  # topk.py:13, on the CPU


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_topk_half_error_feedback_follows_the_reference_ops(gpu, dtype):
    comp = TopKCompression(device=gpu, compress_ratio=0.02)
    ref_res = {}
    g = torch.Generator().manual_seed(11)
    for call in range(3):
        w = 3.0 if call == 1 else 1.0
        for name, n in (("a", 3000), ("b", 70001), ("c", 5)):
            x = (torch.randn(n, generator=g) * 1e-2).to(dtype)
            (v, i), ctx = comp.compress_weighted(x.to(gpu), name, w)
            assert ctx == (n, x.size()) and v.dtype == dtype and i.dtype == torch.int64
            # the reference: update = param * batch_samples, then compensate, in the tensor's dtype
            t = torch.mul(x, w) if w != 1.0 else x
            if name in ref_res:
                t = 1.0 * ref_res[name] + 1.0 * t
            k = max(1, int(n * 0.02))
            got = i.cpu().numpy()
            assert got.tolist() == _rule_topk(t, k).tolist(), (call, name)
            assert np.array_equal(_bits(v), _bits(t[i.cpu()])), (call, name)
            mags = torch.sort(v.cpu().float().abs(), descending=True).values
            assert torch.equal(mags, torch.topk(t.float().abs(), k).values), (call, name)
            dec = torch.zeros(n, dtype=dtype)
            dec[i.cpu()] = v.cpu()
            ref_res[name] = t - dec  # core.py:32-37
            assert comp.residual.residuals[name].dtype == dtype
            assert np.array_equal(_bits(comp.residual.residuals[name].reshape(-1)), _bits(ref_res[name])), (call, name)
            assert np.array_equal(_bits(comp.decompress((v, i), ctx)), _bits(dec)), (call, name)


def test_topk_half_wire_encode_and_bf16_error(gpu):
    """fp16: the LayerState carries the fp16 values widened to fp32 (the reference's astype), through
    encode_layer_state and encode_updates_dict alike; bf16: the reference's TypeError (numpy has no
    bfloat16), raised after the residual was updated, as there."""
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(4099, generator=g) * 1e-2).half()
    a, b, per_tensor = (TopKCompression(device=gpu, compress_ratio=0.01) for _ in range(3))
    for call in range(2):
        L1 = encode_layer_state("w", x.to(gpu), a)
        L2, = encode_updates_dict({"w": x.to(gpu)}, b)
        (v, i), _ = per_tensor.compress(x.to(gpu), "w")  # pinned to the reference ops above
        want = topk_layer_from_payload("w", (4099,), v.float().cpu().numpy(), i.cpu().numpy())
        assert L1.SerializeToString() == want.SerializeToString() == L2.SerializeToString(), call
        assert L1.values_dtype == "torch.float32"
    c = TopKCompression(device=gpu, compress_ratio=0.01)
    with pytest.raises(TypeError, match="BFloat16"):
        encode_layer_state("w", x.to(gpu).bfloat16(), c)
    assert "w" in c.residual.residuals and c.residual.residuals["w"].dtype == torch.bfloat16


def test_topk_decode_onto_half_base_keeps_its_dtype(gpu):
    """global_grpc_compression.py:151-156: the overlay is a numpy copy of the base, so a fp16 base
    gives a fp16 result (the fp32 values rounded to nearest on assignment), an integer base an
    integer one, a fp64 base a fp64 one; a bf16 base raises as .numpy() does there.  The client
    downlink (decode_updates_into) writes the same into fp16 targets."""
    g = torch.Generator().manual_seed(5)
    n = 1000
    vals = (torch.randn(20, generator=g) * 1.2345).numpy().astype(np.float32)
    idx = np.random.default_rng(0).permutation(n)[:20].astype(np.int64)
    L = topk_layer_from_payload("w", (10, 100), vals, idx)
    for dt in (torch.float16, torch.float64, torch.int32, torch.float32):
        base = (torch.randn(10, 100, generator=g) * 50).to(dt)
        got = decode_layer_tensor(L, base_tensor=base.to(gpu))
        flat = base.numpy().reshape(-1).copy()
        flat[idx] = vals
        want = torch.from_numpy(flat.reshape(10, 100))
        assert got.dtype == want.dtype and got.device.type == "cuda", dt
        assert torch.equal(got.cpu(), want), dt
    with pytest.raises(TypeError, match="BFloat16"):
        decode_layer_tensor(L, base_tensor=torch.zeros(10, 100, dtype=torch.bfloat16, device=gpu))
    tgt = (torch.randn(10, 100, generator=g)).half()
    flat = tgt.numpy().reshape(-1).copy()
    flat[idx] = vals
    t_dev = tgt.to(gpu)
    decode_updates_into([L], {"w": t_dev})
    assert torch.equal(t_dev.cpu(), torch.from_numpy(flat.reshape(10, 100)))


def test_topk_fp16_dict_batched_equals_per_layer(gpu):
    """encode_updates_dict of an fp16 dict is ONE selection launch (the weighting and compensate as
    the reference's fp16 expressions over the dict's arena, residuals kept in fp16 views of one
    arena): byte-identical LayerStates and bit-identical residuals to the per-layer path over 3
    weighted error-feedback calls, with a name missing from one call and a residual replaced by
    the caller; a bf16 dict raises the reference's TypeError."""
    from omnifed_amd.hybrid.communicator.global_grpc_compression import _topk_batchable

    g = torch.Generator(device=gpu).manual_seed(21)
    shapes = {"a": (64, 33), "b": (4099,), "c": (1,), "d": (300, 301), "e": (1 << 18,)}
    a = TopKCompression(device=gpu, compress_ratio=0.02)
    b = TopKCompression(device=gpu, compress_ratio=0.02)
    for call in range(3):
        upd = {n: (torch.randn(*s, device=gpu, generator=g) * 1e-2).half() for n, s in shapes.items()}
        if call == 1:
            upd.pop("c")
        if call == 2:
            a.residual.residuals["a"] = b.residual.residuals["a"].clone()
        assert _topk_batchable(list(upd.values()))
        w = 3.0 if call != 1 else None
        got = encode_updates_dict(upd, a, weight=w)
        want = [encode_layer_state(n, t, b, weight=w) for n, t in upd.items()]
        for L, P in zip(got, want):
            assert L.SerializeToString() == P.SerializeToString(), (call, L.layer_name)
        for n in upd:
            ra, rb = a.residual.residuals[n], b.residual.residuals[n]
            assert ra.dtype == torch.float16 and np.array_equal(_bits(ra.reshape(-1)), _bits(rb.reshape(-1))), (call, n)
    with pytest.raises(TypeError, match="BFloat16"):
        encode_updates_dict({n: torch.randn(*s, device=gpu).bfloat16() for n, s in shapes.items()},
                            TopKCompression(device=gpu, compress_ratio=0.02))
