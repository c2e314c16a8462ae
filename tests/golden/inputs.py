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
