"""Philox4x32-10 in numpy — TEST INFRASTRUCTURE ONLY.

The perf-mode RNG of the HIP encoder (MT19937 is serial, so
on-device draws come from a counter-based generator).  The algorithm is the
published Philox4x32-10 of Salmon et al., "Parallel random numbers: as easy as
1, 2, 3" (SC'11); ``tests/test_oracle_golden.py`` pins it on the Random123
known-answer vectors.

Stream layout used by ``omf_qsgd_encode`` (include/omf_codec.h):
for element ``i`` of tensor ``t`` (tensor-local index) in a call with
``seed`` and ``offset``::

    ctr = (i >> 2 & 0xffffffff, i >> 34, t, offset & 0xffffffff)
    key = (seed & 0xffffffff, seed >> 32)
    u_i = (philox(ctr, key)[i & 3] & 0xFFFFFF) * 2**-24

i.e. the same 24-bit uniform rule as torch's CPU generator.
"""

from __future__ import annotations

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds; all inputs uint32 arrays/scalars."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for r in range(10):
            if r > 0:
                k0 = np.uint32(k0 + _W0)
                k1 = np.uint32(k1 + _W1)
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & _MASK).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & _MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def philox_uniforms(seed: int, offset: int, tensor_index: int, n: int) -> np.ndarray:
    """The perf-mode uniforms ``u_0..u_{n-1}`` for one tensor (layout above)."""
    nq = (n + 3) // 4
    j = np.arange(nq, dtype=np.uint64)
    c0 = (j & _MASK).astype(np.uint32)
    c1 = (j >> np.uint64(32)).astype(np.uint32)
    c2 = np.full(nq, tensor_index & 0xFFFFFFFF, dtype=np.uint32)
    c3 = np.full(nq, offset & 0xFFFFFFFF, dtype=np.uint32)
    o = philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    w = np.stack(o, axis=1).reshape(-1)[:n]
    return ((w & np.uint32(0xFFFFFF)).astype(np.float64) * 2.0**-24).astype(np.float32)
