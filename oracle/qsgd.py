"""QSGD oracle: the reference's torch-CPU op sequence, restated — TEST INFRASTRUCTURE ONLY.

Follows ``/root/reference/src/omnifed/hybrid/compression/qsgd.py``:

* ``storage_width``      ↔ ``choose_qsgd_storage_width`` (qsgd.py:18-21)
* ``qsgd_quantize``      ↔ ``QSGDQuantCompression.quantize_vector`` (qsgd.py:36-64)
* ``qsgd_dequantize``    ↔ ``QSGDQuantCompression.decompress_quantized`` (qsgd.py:84-96)
* ``qsgd_encode_dict``   ↔ ``encode_updates_dict`` + ``_encode_qsgd_layer``
  (global_grpc_compression.py:101-123, 207-211): one RNG stream consumed
  tensor by tensor; zero-norm / non-float / empty tensors consume no draws.

The op order is kept one-to-one (norm → div → sign/abs → ×L → floor.long →
sub → rand → compare → clamp → ×sign → cast) so that this module doubles as the
"reference-equivalent CPU codec" that ``bench.py`` times as ``cpu_baseline``
(kind ``"port"``).  ``norm`` and ``u`` may be injected: the reference's fp32
``torch.norm`` is ISA dependent, and MT19937 is serial, so bit-exact parity of
the payload is defined given ``(norm, u)``.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch


def storage_width(levels: int) -> Tuple[int, torch.dtype]:
    """qsgd.py:18-21 — int8 while levels <= 127, else int32."""
    if levels <= 127:
        return 8, torch.int8
    return 32, torch.int32


def mt19937_uniforms(seed: int, n: int) -> np.ndarray:
    """The first ``n`` draws of ``torch.manual_seed(seed); torch.rand(n)``.

    torch's CPU generator is MT19937; each fp32 uniform is
    ``(next32() & 0xFFFFFF) * 2**-24`` (verified bit-for-bit).
    """
    return MTStream(seed).draw(n)


class MTStream:
    """A continuing MT19937 uniform stream (numpy RandomState == torch CPU generator)."""

    def __init__(self, seed: int):
        self._rs = np.random.RandomState(seed)

    def draw(self, n: int) -> np.ndarray:
        if n == 0:
            return np.zeros(0, dtype=np.float32)
        w = self._rs.randint(0, 2**32, n, dtype=np.uint64)
        return ((w & 0xFFFFFF).astype(np.float64) * 2.0**-24).astype(np.float32)


def qsgd_quantize(
    v: torch.Tensor,
    s: int,
    norm: Optional[float] = None,
    u: Optional[torch.Tensor] = None,
):
    """qsgd.py:36-64 on a flat fp32 CPU tensor.

    Returns ``(q, norm, width, levels)``; ``(v, -1, -1, -1)`` for empty input and
    ``(zeros, -1, -1, -1)`` when the norm is zero (no RNG draw consumed).
    ``u`` (same numel as ``v``) replaces ``torch.rand_like`` when given.
    """
    if v.numel() == 0:
        return v, -1, -1, -1
    norm_v = torch.norm(v).item() if norm is None else float(norm)
    if norm_v == 0:
        return torch.zeros_like(v), -1, -1, -1
    v_normalized = v / norm_v
    signs = torch.sign(v_normalized)
    abs_v = torch.abs(v_normalized)
    levels = 2 ** int(s)
    scaled_abs = abs_v * levels
    lower = torch.floor(scaled_abs).long()
    prob_round_up = scaled_abs - lower.float()
    draws = torch.rand_like(prob_round_up) if u is None else u.reshape(prob_round_up.shape)
    round_up = (draws < prob_round_up).long()
    quantized_levels = torch.clamp(lower + round_up, 0, levels)
    signed_levels = signs.long() * quantized_levels
    width, dtype = storage_width(levels)
    return signed_levels.to(dtype), norm_v, width, levels


def qsgd_dequantize(q: torch.Tensor, norm: float, levels: int, shape) -> torch.Tensor:
    """qsgd.py:84-96: ``y = fl32(fl32(norm * q) / levels)``."""
    if levels <= 0 or norm is None or norm == -1:
        return q
    flat = q.float().reshape(-1)
    restored = float(norm) * flat / float(levels)
    return restored.reshape(shape)


def qsgd_encode_dict(
    updates: Dict[str, torch.Tensor],
    s: int,
    seed: Optional[int] = None,
    norms: Optional[List[Optional[float]]] = None,
):
    """encode_updates_dict for QSGD with one continuing MT19937 stream.

    ``seed`` None → torch's global generator (caller seeds it); else the numpy
    MT stream with that seed is injected.  ``norms[i]`` (optional) overrides the
    norm of tensor i.  Returns a list of ``(name, q|None, norm, width, levels)``
    with ``q`` None for dense passthrough tensors.
    """
    stream = MTStream(seed) if seed is not None else None
    out = []
    for i, (name, t) in enumerate(updates.items()):
        t = t.detach().cpu()
        if not (t.is_floating_point() and t.numel() > 0):
            out.append((name, None, -1, -1, -1))
            continue
        flat = t.flatten()
        nrm = None if norms is None else norms[i]
        u = None
        if stream is not None:
            n_eff = torch.norm(flat).item() if nrm is None else nrm
            if n_eff != 0:
                u = torch.from_numpy(stream.draw(flat.numel()))
        q, norm_v, width, levels = qsgd_quantize(flat, s, norm=nrm, u=u)
        if width == -1:
            out.append((name, None, -1, -1, -1))
        else:
            out.append((name, q.reshape(t.shape), norm_v, width, levels))
    return out
