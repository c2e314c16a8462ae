"""omf_topk_select_host (CPU, no GPU): the reference's Top-K selection, ties and order included.

The reference selects with ``torch.topk(t.abs(), k, sorted=False)`` on the CPU
(``src/omnifed/hybrid/compression/topk.py:13``).  Where magnitudes tie, which of them are taken at
rank k and their order inside the selection are fixed by torch's CPU algorithm (libstdc++
partial_sort for k*64 <= n, nth_element otherwise).  The library restates it on the host; these
tests pin the restatement to torch itself (the oracle's ``topk_sparse``) on tie-heavy inputs.
"""

import ctypes

import numpy as np
import pytest
import torch

from omnifed_amd import _lib
from oracle import topk as otk


def select_host(t: np.ndarray, k: int) -> np.ndarray:
    t = np.ascontiguousarray(t, dtype=np.float32)
    out = np.empty(k, dtype=np.int64)
    rc = _lib.lib().omf_topk_select_host(t.ctypes.data_as(ctypes.c_void_p), t.size, k,
                                         out.ctypes.data_as(ctypes.c_void_p))
    _lib.check(rc, "omf_topk_select_host")
    return out


def torch_indices(t: torch.Tensor, k: int) -> np.ndarray:
    return torch.topk(t.abs(), k, sorted=False).indices.numpy()


def _cases():
    g = torch.Generator().manual_seed(7)
    yield "gauss_1m", torch.randn(1 << 20, generator=g) * 1e-3, 10485
    yield "ints_100k", torch.randint(-20, 21, (100003,), generator=g).float(), 1000
    yield "two_values", torch.randint(0, 2, (65536,), generator=g).float(), 1024
    for n in (70000, 1000003):
        k = otk.topk_k(n, 0.01)
        for nnz in (0, int(0.3 * k), k - 1):
            x = torch.zeros(n)
            pos = torch.randperm(n, generator=g)[:nnz]
            x[pos] = torch.randn(nnz, generator=g)
            x[torch.randperm(n, generator=g)[: n // 3]] *= -1.0  # signed zeros: one magnitude
            yield f"zeros_n{n}_nnz{nnz}", x, k
    x = torch.randn(70000, generator=g)
    x[torch.randint(0, 70000, (40,), generator=g)] = float("nan")
    x[torch.randint(0, 70000, (40,), generator=g)] = float("inf")
    x[torch.randint(0, 70000, (40,), generator=g)] = -float("inf")
    yield "nan_inf", x, 700
    x = torch.randn(70000, generator=g)
    x[::7] = 0.5  # the k-th magnitude tied across rank k
    yield "tied_kth", x, 700


@pytest.mark.parametrize("name,x,k", list(_cases()), ids=lambda v: v if isinstance(v, str) else "")
def test_select_host_equals_torch_heap_regime(name, x, k):
    assert k * 64 <= x.numel()
    assert np.array_equal(select_host(x.numpy(), k), torch_indices(x, k)), name


def test_select_host_equals_torch_nth_element_regime():
    """k*64 > n: torch leaves nth_element's partition order (sorted=False)."""
    g = torch.Generator().manual_seed(3)
    for trial in range(200):
        n = int(torch.randint(1, 6000, (1,), generator=g))
        k = int(torch.randint(max(1, n // 64 + 1) if n >= 64 else 1, n + 1, (1,), generator=g))
        x = torch.randint(-4, 5, (n,), generator=g).float() if trial % 2 else torch.randn(n, generator=g)
        if trial % 5 == 0:
            x[torch.randint(0, n, (3,), generator=g)] = float("nan")
        assert np.array_equal(select_host(x.numpy(), k), torch_indices(x, k)), (trial, n, k)


def test_select_host_random_ratios_and_sizes():
    g = torch.Generator().manual_seed(11)
    for trial in range(120):
        n = int(torch.randint(1, 300000, (1,), generator=g))
        ratio = float(torch.empty(1).uniform_(0.0005, 0.3, generator=g))
        k = otk.topk_k(n, ratio)
        if k > n:
            continue
        levels = int(torch.randint(2, 5000, (1,), generator=g))
        x = (torch.randint(-levels, levels + 1, (n,), generator=g).float() if trial % 3
             else torch.randn(n, generator=g))
        assert np.array_equal(select_host(x.numpy(), k), torch_indices(x, k)), (trial, n, k)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_select_host_half_tensors_on_widened_values(dt):
    """torch's CPU topk of a half tensor compares the widened magnitudes: the same as ours on the
    exactly widened fp32 values."""
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(200003, generator=g) * 3).to(dt)
    k = otk.topk_k(x.numel(), 0.01)
    assert np.array_equal(select_host(x.float().numpy(), k), torch_indices(x, k))


def test_select_host_argument_errors():
    L = _lib.lib()
    t = np.zeros(8, np.float32)
    out = np.zeros(8, np.int64)
    p, o = t.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p)
    assert L.omf_topk_select_host(p, 8, 0, o) == _lib.OMF_EINVAL
    assert L.omf_topk_select_host(p, 8, 9, o) == _lib.OMF_EINVAL
    assert L.omf_topk_select_host(None, 8, 1, o) == _lib.OMF_EINVAL
    assert L.omf_topk_select_host(p, 8, 8, o) == _lib.OMF_OK
