"""Top-K where magnitudes tie: the drop-in's bytes against the REAL reference's (golden_r6).

The reference selects with ``torch.topk(|t'|, k, sorted=False)`` on the CPU (topk.py:13): where
magnitudes tie, which of them are selected at rank k and their order are torch's CPU algorithm's.
The plugin layer's default ``tie_order="torch"`` reproduces them (``omf_topk_torch_order``);
these tests hold it to fixtures the reference itself produced (tests/golden/gen_golden_r6.py):
``values_data`` / ``indices_data``, the error-feedback residual and the overlay decode, byte for
byte — fewer non-zeros than k (the zero fill), a k-th magnitude shared across rank k, many equal
magnitudes inside the selection, k * 64 > n (nth_element's order) and a dict through
``encode_updates_dict``.
"""

import hashlib
import json
import os

import numpy as np
import pytest
import torch

import oracle
from inputs import exact_input, ints, sparse_input, tied_kth
from omnifed_amd import codec
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    _decode_topk_layer,
    _encode_topk_layer,
    encode_updates_dict,
)
from omnifed_amd.hybrid.compression import TopKCompression

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def g6():
    return np.load(os.path.join(GOLDEN, "golden_r6.npz"))


@pytest.fixture(scope="module")
def g6_index():
    with open(os.path.join(GOLDEN, "golden_r6_index.json")) as f:
        return json.load(f)


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _check_layer(L, g6, g6_index, key):
    assert L.compression_type == "TopKCompression", key
    assert L.values_data == g6[key + "/values"].tobytes(), key
    assert L.indices_data == g6[key + "/indices"].tobytes(), key
    assert _sha(np.frombuffer(L.SerializeToString(), np.uint8)) == g6_index["layer_sha"][key], key


def test_zero_fill_two_calls_and_overlay_equal_reference(gpu, g6, g6_index):
    """nnz in {0, 0.3 k, k - 1} at n in {70 000, 1 000 003}: both error-feedback calls' layers,
    the residual and the client's overlay decode (global_grpc_compression.py:153-156)."""
    for c in g6_index["zero"]:
        n, nnz = c["n"], c["nnz"]
        s1, s2, s3 = c["seeds"]
        comp = TopKCompression(device=gpu, compress_ratio=c["ratio"])
        key = f"zero/{c['id']}"
        L1 = _encode_topk_layer("w", torch.from_numpy(sparse_input(s1, n, nnz)).to(gpu), comp)
        _check_layer(L1, g6, g6_index, key + "/call0")
        L2 = _encode_topk_layer("w", torch.from_numpy(sparse_input(s2, n, nnz)).to(gpu), comp)
        _check_layer(L2, g6, g6_index, key + "/call1")
        res = comp.residual.residuals["w"].cpu().numpy().reshape(-1)
        assert _sha(res) == c["residual_sha"], key
        base = torch.from_numpy(exact_input(s3, n, -3))
        over = _decode_topk_layer(L1, base_tensor=base).numpy().reshape(-1)
        assert _sha(over) == c["overlay0_sha"], key
        if key + "/overlay0" in g6:
            assert over.tobytes() == g6[key + "/overlay0"].tobytes()


def test_ties_across_and_inside_the_selection_equal_reference(gpu, g6, g6_index):
    for c in g6_index["tied"]:
        n, k, kind = c["n"], c["k"], c["kind"]
        tid = c["id"]
        x = tied_kth(tid, n, k) if kind == "kth" else ints(tid, n, 3000) if kind == "ints" else exact_input(
            500 + tid, n, -7)
        assert _sha(x) == c["x_sha"]
        comp = TopKCompression(device=gpu, compress_ratio=c["ratio"])
        L = _encode_topk_layer("w", torch.from_numpy(x).to(gpu), comp)
        _check_layer(L, g6, g6_index, f"tied/{tid}")
        assert _sha(comp.residual.residuals["w"].cpu().numpy().reshape(-1)) == c["residual_sha"]


def test_nth_element_regime_equals_reference(gpu, g6, g6_index):
    """k * 64 > n: torch leaves nth_element's partition order (the reference's own test uses
    ratio 0.25, tests/test_hybrid_global_grpc_compression.py:17)."""
    for c in g6_index["nth"]:
        n = c["n"]
        x = exact_input(600 + c["id"], n, -1) if c["kind"] == "exact" else ints(600 + c["id"], n, 7)
        comp = TopKCompression(device=gpu, compress_ratio=c["ratio"])
        L = _encode_topk_layer("w", torch.from_numpy(x).to(gpu), comp)
        _check_layer(L, g6, g6_index, f"nth/{c['id']}")


def test_dict_two_calls_equal_reference(gpu, g6, g6_index):
    """encode_updates_dict (the batched one-launch path) through two error-feedback calls."""
    shapes = [(n, tuple(s)) for n, s in g6_index["dict"]["shapes"]]
    comp = TopKCompression(device=gpu, compress_ratio=g6_index["dict"]["ratio"])
    for call in range(2):
        upd = {}
        for t, (name, shape) in enumerate(shapes):
            n = int(np.prod(shape))
            seed = 700 + 10 * call + t
            x = sparse_input(seed, n, 100) if name == "z" else ints(seed, n, 200) if name == "w" else exact_input(
                seed, n, -5)
            upd[name] = torch.from_numpy(x).reshape(shape).to(gpu)
        for L in encode_updates_dict(upd, comp):
            _check_layer(L, g6, g6_index, f"dict/out/{call}/{L.layer_name}")
    for name, _ in shapes:
        got = comp.residual.residuals[name].cpu().numpy().reshape(-1)
        assert got.tobytes() == g6[f"dict/residual/{name}"].tobytes(), name


def test_torch_order_rewrites_tied_tensors_of_an_arena(gpu):
    """One tie-heavy arena encoded with the device order alone ("index") and with torch's
    ("torch"): the census rewrites the tied tensors, and the torch bytes — values, indices and the
    residual — equal the oracle's (torch.topk on the CPU) for every tensor."""
    sizes = [70000, 1 << 20, 4099, 37, 300001]
    plan = codec.Plan(sizes, device=gpu)
    xh = torch.zeros(plan.arena_end)
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        xh[o:o + n] = torch.from_numpy(ints(900 + t, n, 50 if t % 2 else 4000))
    xh[plan.offsets[0]:plan.offsets[0] + 70000:3] = 0.0
    x = xh.to(gpu)
    out = {}
    for order in ("index", "torch"):
        res = torch.empty(plan.arena_end, device=gpu)
        v, i, ks = plan.topk_encode(x, 0.01, residual=res, residual_mode=2, tie_order=order)
        out[order] = (v.cpu(), i.cpu(), res.cpu(), list(ks))
    assert plan.topk_reordered >= 3
    vt, it, rt, ks = out["torch"]
    K = 0
    for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
        k = ks[t]
        ov, oi = oracle.topk_sparse(xh[o:o + n], 0.01)
        assert it[K:K + k].numpy().tobytes() == oi.numpy().tobytes(), t
        assert vt[K:K + k].numpy().tobytes() == ov.numpy().tobytes(), t
        want = xh[o:o + n].clone()
        want[oi] = 0.0
        assert rt[o:o + n].numpy().tobytes() == want.numpy().tobytes(), t
        K += k


def test_ef_arena_torch_order_equals_oracle(gpu):
    """Three error-feedback calls over a multi-tensor arena of Gaussian gradients (equal
    magnitudes inside every large tensor's selection; ties at rank k on some calls), weighted
    (alpha): values, indices and residuals equal the oracle's TopKCompression byte for byte."""
    sizes = [1 << 22, 3 << 20, 5000, 1_000_003, 4096, 640]
    plan = codec.Plan(sizes, device=gpu)
    g = torch.Generator().manual_seed(61)
    res = torch.empty(plan.arena_end, device=gpu)
    refs = [oracle.TopKOracle(0.01) for _ in sizes]
    alpha = 3.0
    for call in range(3):
        xh = torch.randn(plan.arena_end, generator=g) * 1e-3
        v, i, ks = plan.topk_encode(xh.to(gpu), 0.01, residual=res, residual_mode=2 if call == 0 else 1,
                                    alpha=alpha, tie_order="torch")
        vh, ih, rh = v.cpu(), i.cpu(), res.cpu()
        K = 0
        for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
            k = ks[t]
            a = torch.mul(xh[o:o + n], alpha)
            (ov, oi), _ = refs[t].compress(a, "w")
            assert ih[K:K + k].numpy().tobytes() == oi.numpy().tobytes(), (call, t)
            assert vh[K:K + k].numpy().tobytes() == ov.numpy().tobytes(), (call, t)
            assert rh[o:o + n].numpy().tobytes() == refs[t].residuals["w"].numpy().tobytes(), (call, t)
            K += k
