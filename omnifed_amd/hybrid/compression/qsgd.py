"""QSGD quantisation on MI355X (mirror of ``src/omnifed/hybrid/compression/qsgd.py``).

Same public names, signatures, return conventions and error behaviour as the
reference (qsgd.py:11-107); the arithmetic runs in the HIP encoder/decoder of
``libomf_codec.so`` (``omf_qsgd_encode`` / ``omf_qsgd_decode``).  Input and
output tensors stay where the caller has them (a CPU tensor is encoded on the
GPU and its payload returned on the CPU, as ``_do_compress`` returns it on
``tensor.device``, qsgd.py:69).

Random draws (``rng``):
  * ``"philox"`` (default): on-device Philox4x32-10 keyed by a 63-bit seed drawn
    from torch's default CPU generator per call — so ``torch.manual_seed`` makes
    runs reproducible, as in the reference — plus a per-compressor call counter.
    Statistically the reference's ``rand_like`` (24-bit uniforms), not the same bits.
  * ``"mt19937"``: the reference's own stream: ``torch.rand`` on the default CPU
    generator, consumed tensor by tensor and skipped for zero-norm tensors
    (qsgd.py:47-48, 58), handed to the kernel as an input buffer.  Bit-identical
    payloads follow whenever the norm equals the reference's (its fp32
    ``torch.norm`` is ISA dependent).
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from ... import codec
from .core import Compression, compute_device, to_arena

QSGD_COMPRESSION_NAME = "QSGDQuantCompression"
# Opt-in bit-packed wire (not reference-compatible): codes q + L in
# ceil(log2(2L+1)) bits instead of int8/int32 levels (include/omf_codec.h omf_qsgd_pack).
QSGD_PACKED_COMPRESSION_NAME = "QSGDBitPackedCompression"


def should_compress_tensor(x: torch.Tensor) -> bool:
    """qsgd.py:14-15."""
    return isinstance(x, torch.Tensor) and x.is_floating_point() and x.numel() > 0


def choose_qsgd_storage_width(levels: int) -> tuple:
    """qsgd.py:18-21."""
    if levels <= torch.iinfo(torch.int8).max:
        return 8, torch.int8
    return 32, torch.int32


def encode_many(flats: Sequence[torch.Tensor], bit_width: int, dev: torch.device, rng: str = "philox",
                call_index: int = 0, alpha: float = 1.0, chunk: int = 0):
    """Encode several flat tensors in ONE launch.

    Returns ``(plan, q_arena, norms_dev)``: tensor i's levels are
    ``q_arena[plan.offsets[i] : plan.offsets[i] + plan.sizes[i]]``.
    """
    sizes = [int(f.numel()) for f in flats]
    plan = codec.Plan.get(sizes, device=dev, chunk=chunk)
    if len(flats) == 1:
        x = to_arena(flats[0], dev, plan)
    else:
        x = torch.empty(plan.arena_end, dtype=torch.float32, device=dev)
        for f, o, n in zip(flats, plan.offsets, sizes):
            x[o:o + n].copy_(f.detach().reshape(-1))
    s = int(bit_width)
    if rng == "mt19937":
        norms = plan.qsgd_norms(x, alpha=alpha)
        host_norms = norms.cpu().tolist()
        u_host = torch.zeros(plan.arena_end, dtype=torch.float32)
        for o, n, nv in zip(plan.offsets, sizes, host_norms):
            if nv != 0:
                u_host[o:o + n] = torch.rand(n)
        u = u_host.to(dev)
        q, norms = plan.qsgd_encode(x, s, alpha=alpha, u=u, norm_in=norms)
    elif rng == "philox":
        seed = int(torch.randint(0, 2**62, (1,)).item())
        q, norms = plan.qsgd_encode(x, s, alpha=alpha, seed=seed, offset=call_index)
    else:
        raise ValueError(f"unknown rng={rng!r}; expected 'philox' or 'mt19937'")
    return plan, q, norms


class QSGDQuantCompression(Compression):
    """QSGD (Alistarh et al., 2017), Algorithm 1 — on the GPU."""

    def __init__(self, bit_width: int = 8, device="cpu", rng: str = "philox", packed_wire: bool = False):
        super().__init__()
        self.s = int(bit_width)
        self.packed_wire = bool(packed_wire)  # encode_updates_dict / encode_layer_state emit packed layers
        self.device = torch.device(device)
        if rng not in ("philox", "mt19937"):
            raise ValueError(f"unknown rng={rng!r}; expected 'philox' or 'mt19937'")
        self.rng = rng
        self._calls = 0

    def _next_call(self) -> int:
        c = self._calls
        self._calls += 1
        return c

    def quantize_vector(self, v: torch.Tensor):
        """Q_s(v) for a flat tensor; returns ``(signed_levels, norm, width, levels)`` (qsgd.py:36-64)."""
        if v.numel() == 0:
            return v, -1, -1, -1
        out = self.encode_flat([v])
        q, norm, width, levels = out[0]
        if width == -1:
            return torch.zeros_like(v), -1, -1, -1
        return q.to(v.device), norm, width, levels

    def encode_flat(self, flats: List[torch.Tensor]) -> List[Tuple]:
        """Batched ``quantize_vector``: one launch for every tensor (all must be non-empty floats).

        Returns a ``(q_device_view, norm, width, levels)`` per tensor, or
        ``(None, -1, -1, -1)`` for a zero norm.
        """
        if not (0 <= self.s <= 30):
            # levels = 2**s must fit LayerState.level (int32); the reference fails there too.
            raise ValueError(f"QSGD bit_width={self.s} out of range [0, 30]")
        dev = compute_device(flats[0], self.device)
        plan, q, norms = encode_many(flats, self.s, dev, self.rng, self._next_call())
        levels = 2**self.s
        width, _ = choose_qsgd_storage_width(levels)
        host_norms = norms.cpu().tolist()
        out = []
        for o, n, nv in zip(plan.offsets, plan.sizes, host_norms):
            if nv == 0:
                out.append((None, -1, -1, -1))
            else:
                out.append((q[o:o + n], float(nv), width, levels))
        return out

    def _do_compress(self, tensor: torch.Tensor):
        flat = tensor.flatten()
        signed_levels, norm, width, levels = self.quantize_vector(flat)
        signed_levels = signed_levels.reshape(tensor.shape).to(tensor.device)
        return signed_levels, norm, width, levels

    def compress(self, tensor: torch.Tensor, name: str = ""):
        """qsgd.py:72-82: ``(signed_levels, norm, width, levels)``; -1s for dense passthrough."""
        del name
        if not should_compress_tensor(tensor):
            return tensor, -1, -1, -1
        return self._do_compress(tensor)

    @staticmethod
    def decompress_quantized(signed_levels: torch.Tensor, norm: float, levels: int, shape) -> torch.Tensor:
        """qsgd.py:84-96: ``norm * signed_level / levels`` (fp32), on the GPU."""
        if levels <= 0 or norm is None or norm == -1:
            return signed_levels
        out_dev = signed_levels.device
        dev = compute_device(signed_levels, torch.device("cpu"))
        flat = signed_levels.reshape(-1)
        if flat.dtype == torch.int8:
            width = 8
        else:
            width = 32
            if flat.dtype != torch.int32:
                flat = flat.to(torch.int32)
        n = flat.numel()
        if n == 0:
            return torch.zeros(0, dtype=torch.float32, device=out_dev).reshape(shape)
        plan = codec.Plan.get([n], device=dev)
        qbuf = flat
        if qbuf.device != dev or not qbuf.is_contiguous() or qbuf.data_ptr() % 16:
            qbuf = torch.empty(n, dtype=flat.dtype, device=dev)  # fresh allocations are 256-B aligned
            qbuf.copy_(flat)
        nrm = torch.tensor([float(norm)], dtype=torch.float32, device=dev)
        y = plan.qsgd_decode(qbuf, width, int(levels), nrm)
        return y[:n].reshape(shape).to(out_dev)

    def decompress(self, tensors, ctx):
        """qsgd.py:98-107; ``ctx = (norm, width, levels, shape)``."""
        norm, _width, levels, shape = ctx
        signed_levels = tensors[0] if isinstance(tensors, (tuple, list)) else tensors
        return self.decompress_quantized(signed_levels, norm, levels, shape)
