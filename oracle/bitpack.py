"""Bit-packed QSGD wire (opt-in) restated in numpy — TEST INFRASTRUCTURE ONLY.

Not part of the reference (a new ``compression_type``, "QSGDBitPackedCompression"); the
layout it restates is the one ``include/omf_codec.h`` specifies for ``omf_qsgd_pack``:
level q in [-L, L] -> code q + L in b = ceil(log2(2L + 1)) bits, element i of a tensor
at bits [i*b, (i+1)*b) of the tensor's byte stream, least significant bit first.  The
round trip must give back the same integers as the reference's int8/int32 payload
(``global_grpc_compression.py:111-123``), so decoding a packed layer equals decoding the
reference layer.
"""

from __future__ import annotations

import numpy as np


def packed_bits(levels: int) -> int:
    return (2 * int(levels)).bit_length()


def pack(levels_q: np.ndarray, L: int) -> bytes:
    """Signed levels -> the tensor's packed bytes (ceil(n * b / 8) of them)."""
    b = packed_bits(L)
    q = np.asarray(levels_q, dtype=np.int64).reshape(-1)
    if q.size and (q.min() < -L or q.max() > L):
        raise ValueError("level outside [-L, L]")
    codes = (q + L).astype(np.uint64)
    bits = ((codes[:, None] >> np.arange(b, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(np.uint8)
    return np.packbits(bits.reshape(-1), bitorder="little").tobytes()


def unpack(data: bytes, n: int, L: int) -> np.ndarray:
    """The tensor's packed bytes -> its n signed levels (int64)."""
    b = packed_bits(L)
    bits = np.unpackbits(np.frombuffer(data, dtype=np.uint8), bitorder="little")[: n * b]
    if bits.size != n * b:
        raise ValueError("packed payload too short")
    w = (np.uint64(1) << np.arange(b, dtype=np.uint64))
    codes = (bits.reshape(n, b).astype(np.uint64) * w[None, :]).sum(axis=1)
    return codes.astype(np.int64) - int(L)
