"""Philox4x32-10 in numpy — TEST INFRASTRUCTURE ONLY.

The perf-mode RNG of the HIP encoder (MT19937 is serial, so
on-device draws come from a counter-based generator).  The algorithm is the
published Philox4x32-10 of Salmon et al., "Parallel random numbers: as easy as
1, 2, 3" (SC'11); ``tests/test_oracle_golden.py`` pins it on the Random123
known-answer vectors.

Stream layout used by ``omf_qsgd_encode`` (include/omf_codec.h) for element ``i``
(tensor-local index) of tensor ``t`` in a call with ``seed`` and ``offset``::

    j = i >> 2 ; m = j >> 8 ; G = ((m >> 2) << 8) | (j & 255)     # 16-element group
    W = philox(ctr(3G)) ++ philox(ctr(3G+1)) ++ philox(ctr(3G+2))  # 12 words = 384 bits
    ctr(c) = (c & 0xffffffff, c >> 32, t, offset & 0xffffffff), key = (seed & 0xffffffff, seed >> 32)
    f = 4 * (m & 3) + (i & 3)                                      # 24-bit field of W
    u_i = (bits [24 f, 24 f + 24) of W, little-endian) * 2**-24

i.e. the same 24-bit uniform rule as torch's CPU generator, three Philox calls per
16 elements.  A group is what one GPU thread quantises from four of its rows
(rows are 256 float4 = 1024 elements apart), so the kernel derives it from its
thread id without any cross-lane exchange.
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
    """The perf-mode uniforms ``u_0..u_{n-1}`` for one tensor (layout above).

    The groups of a tensor are (nearly) the dense range 0..max(G), so every group below max(G) + 1
    is generated and indexed by G directly (a few unused groups at a partial tail cost nothing);
    the whole tensor is processed in slices of 2^22 elements to bound the temporaries."""
    out = np.empty(n, dtype=np.float32)
    step = 1 << 22  # a multiple of 1024 * 4: a slice starts on a group-row boundary
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for a in range(0, n, step):
        i = np.arange(a, min(n, a + step), dtype=np.int64)
        j = i >> 2
        m = j >> 8
        G = ((m >> 2) << 8) | (j & 255)
        f = 4 * (m & 3) + (i & 3)
        g0 = int(G.min())
        groups = np.arange(g0, int(G.max()) + 1, dtype=np.uint64)
        gpos = G - g0
        words = np.empty((groups.size, 12), dtype=np.uint32)
        for c in range(3):
            ctr = 3 * groups + np.uint64(c)
            o = philox4x32_10((ctr & _MASK).astype(np.uint32), (ctr >> np.uint64(32)).astype(np.uint32),
                              np.full(groups.size, tensor_index & 0xFFFFFFFF, dtype=np.uint32),
                              np.full(groups.size, offset & 0xFFFFFFFF, dtype=np.uint32), k0, k1)
            for w in range(4):
                words[:, 4 * c + w] = o[w]
        bit = 24 * f
        wi = bit >> 5
        sh = (bit & 31).astype(np.uint64)
        lo = words[gpos, wi].astype(np.uint64)
        hi = words[gpos, np.minimum(wi + 1, 11)].astype(np.uint64)
        val = ((lo | (hi << np.uint64(32))) >> sh) & np.uint64(0xFFFFFF)
        out[a:a + len(i)] = (val.astype(np.float64) * 2.0**-24).astype(np.float32)
    return out
