"""Exact synthetic inputs shared by the golden generator and the tests (data recipe, no reference code)."""

import hashlib

import numpy as np


def exact_input(seed: int, n: int, scale_log2: int) -> np.ndarray:
    """fp32 input that is exact by construction: 24-bit signed integers times a power of two."""
    rs = np.random.RandomState(10_000 + seed)
    k = rs.randint(-(2**23), 2**23, n).astype(np.float64)
    return (k * 2.0 ** (scale_log2 - 23)).astype(np.float32)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def sparse_input(seed: int, n: int, nnz: int) -> np.ndarray:
    """``nnz`` exact non-zeros at random positions, zeros elsewhere (a third of them -0.0)."""
    rs = np.random.RandomState(20_000 + seed)
    x = np.zeros(n, np.float32)
    x[rs.permutation(n)[:nnz]] = exact_input(seed, nnz, -4)
    neg = rs.permutation(n)[: n // 3]
    x[neg] = -x[neg]  # zeros become -0.0, non-zeros flip sign
    return x


def tied_kth(seed: int, n: int, k: int) -> np.ndarray:
    """Exact random magnitudes with 10 random elements moved onto the k-th largest magnitude m
    (both signs): m is then shared across rank k."""
    rs = np.random.RandomState(30_000 + seed)
    x = exact_input(seed, n, -2)
    m = np.float32(np.sort(np.abs(x))[::-1][k - 1])
    pos = rs.permutation(n)[:10]
    x[pos] = np.where(rs.rand(10) < 0.5, m, -m).astype(np.float32)
    return x


def ints(seed: int, n: int, levels: int) -> np.ndarray:
    """Multiples of 1/8 in [-levels/8, levels/8]: many equal magnitudes."""
    rs = np.random.RandomState(40_000 + seed)
    return rs.randint(-levels, levels + 1, n).astype(np.float32) * np.float32(0.125)
