"""CPU: the oracle and the library's host selection against the reference's Top-K tie fixtures.

``tests/golden/golden_r6.npz`` holds what the REAL reference codec produced where magnitudes tie
(tests/golden/gen_golden_r6.py).  The oracle (torch.topk on the CPU, oracle/topk.py) must give
the same bytes — that pins it — and so must ``omf_topk_select_host`` (the library's restatement
of torch's CPU algorithm, which ``omf_topk_torch_order`` runs on the GPU path's tied tensors).
"""

import ctypes
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from inputs import exact_input, ints, sparse_input, tied_kth
from omnifed_amd import _lib
from oracle import topk as otk

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


def _host_indices(t: np.ndarray, k: int) -> np.ndarray:
    t = np.ascontiguousarray(t, np.float32)
    out = np.empty(k, np.int64)
    _lib.check(_lib.lib().omf_topk_select_host(t.ctypes.data_as(ctypes.c_void_p), t.size, k,
                                               out.ctypes.data_as(ctypes.c_void_p)), "omf_topk_select_host")
    return out


def _check(vals, idx, g6, key):
    assert idx.tobytes() == g6[key + "/indices"].tobytes(), key
    assert vals.tobytes() == g6[key + "/values"].tobytes(), key


def test_zero_fill_cases(g6, g6_index):
    for c in g6_index["zero"]:
        n, nnz, k = c["n"], c["nnz"], c["k"]
        s1, s2, s3 = c["seeds"]
        orc = otk.TopKOracle(c["ratio"])
        key = f"zero/{c['id']}"
        x1 = sparse_input(s1, n, nnz)
        (v, i), _ = orc.compress(torch.from_numpy(x1.copy()), "w")
        _check(v.numpy(), i.numpy(), g6, key + "/call0")
        hi = _host_indices(x1, k)
        _check(x1[hi], hi, g6, key + "/call0")
        tp = orc.residuals["w"].numpy().reshape(-1) + sparse_input(s2, n, nnz)  # the second call's t'
        (v, i), _ = orc.compress(torch.from_numpy(sparse_input(s2, n, nnz)), "w")
        _check(v.numpy(), i.numpy(), g6, key + "/call1")
        hi = _host_indices(tp, k)
        _check(tp[hi], hi, g6, key + "/call1")
        assert _sha(orc.residuals["w"].numpy().reshape(-1)) == c["residual_sha"], key
        base = exact_input(s3, n, -3)
        over = base.copy()
        over[g6[key + "/call0/indices"]] = g6[key + "/call0/values"]
        assert _sha(over) == c["overlay0_sha"], key


def test_tied_cases(g6, g6_index):
    for c in g6_index["tied"]:
        n, k, kind, tid = c["n"], c["k"], c["kind"], c["id"]
        x = tied_kth(tid, n, k) if kind == "kth" else ints(tid, n, 3000) if kind == "ints" else exact_input(
            500 + tid, n, -7)
        assert _sha(x) == c["x_sha"]
        v, i = otk.topk_sparse(torch.from_numpy(x.copy()), c["ratio"])
        _check(v.numpy(), i.numpy(), g6, f"tied/{tid}")
        hi = _host_indices(x, k)
        _check(x[hi], hi, g6, f"tied/{tid}")
        a = np.abs(x)
        kth = np.sort(a)[::-1][k - 1]
        if kind == "kth":  # the fixture does tie across rank k
            assert (a == kth).sum() > (a[hi] == kth).sum()
        else:  # equal magnitudes inside the selection
            assert len(np.unique(a[hi])) < k


def test_nth_cases(g6, g6_index):
    for c in g6_index["nth"]:
        n, k = c["n"], c["k"]
        x = exact_input(600 + c["id"], n, -1) if c["kind"] == "exact" else ints(600 + c["id"], n, 7)
        assert k * 64 > n
        v, i = otk.topk_sparse(torch.from_numpy(x.copy()), c["ratio"])
        _check(v.numpy(), i.numpy(), g6, f"nth/{c['id']}")
        hi = _host_indices(x, k)
        _check(x[hi], hi, g6, f"nth/{c['id']}")
