"""QSGD quantisation on MI355X (mirror of ``src/omnifed/hybrid/compression/qsgd.py``).

Same public names, signatures, return conventions and error behaviour as the
reference (qsgd.py:11-107); the arithmetic runs in the HIP encoder/decoder of
``libomf_codec.so`` (``omf_qsgd_encode`` / ``omf_qsgd_decode``).  Input and
output tensors stay where the caller has them (a CPU tensor is encoded on the
GPU and its payload returned on the CPU, as ``_do_compress`` returns it on
``tensor.device``, qsgd.py:69).

Random draws (``rng``):
  * ``"philox"`` (default): on-device Philox4x32-10 keyed by (``torch.initial_seed()``,
    the compressor's creation index, the client identity — the process's rank, or
    ``client_id`` when set) with the per-compressor call counter as the
    stream offset — so ``torch.manual_seed`` makes runs reproducible, as in the
    reference, and the caller's CPU generator is never advanced (the reference's
    ``rand_like`` consumes n of its draws per tensor; this codec consumes none, so
    data shuffling or CPU dropout after a swap sees a different generator state).
    Statistically the reference's ``rand_like`` (24-bit uniforms), not the same bits.
  * ``"mt19937"``: the reference's own stream: ``torch.rand`` on the default CPU
    generator, consumed tensor by tensor and skipped for zero-norm tensors
    (qsgd.py:47-48, 58), handed to the kernel as an input buffer, and the reference's own
    norm: ``torch.norm`` of the tensor's CPU copy (ISA dependent, SURVEY.md §0.6, so it is
    computed by the same op on the same host).  Payloads are then bit-identical to the
    reference's on that host.  A parity / debugging mode: the draws and norms run on the CPU.

Dtypes: the reference quantises in the tensor's own dtype.  float32, bfloat16 and
float16 tensors are encoded with that dtype's rounding (``omf_qsgd_encode_ex``
value formats); float64 tensors raise ``ValueError`` (no fp64 encoder).
"""

from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ... import codec
from .core import Compression, compute_device, gather_arena

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


_VALUE_FORMATS = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def value_format(dtype: torch.dtype) -> int:
    """The encoder's value format for a tensor dtype (omf_qsgd_encode_ex): 0 fp32, 1 bf16, 2 fp16."""
    fmt = _VALUE_FORMATS.get(dtype)
    if fmt is None:
        raise ValueError(f"QSGD on the MI355X codec encodes float32, bfloat16 and float16 tensors, not {dtype}")
    return fmt


def _arena(flats: Sequence[torch.Tensor], dev: torch.device, plan) -> torch.Tensor:
    return gather_arena(flats, dev, plan)  # bf16/fp16 -> fp32 is exact


def encode_groups(flats: Sequence[torch.Tensor], bit_width: int, dev: torch.device, rng: str = "philox",
                  call_index: int = 0, alpha: float = 1.0, chunk: int = 0, key: int = 0):
    """Encode flat tensors, ONE launch per dtype present (normally one).

    Returns ``[(plan, q_arena, norms_dev, members)]`` in order of first appearance:
    ``members[k]`` is the index into ``flats`` of the plan's tensor k (levels at
    ``q_arena[plan.offsets[k] : + plan.sizes[k]]``).  ``mt19937``: the uniforms are drawn
    tensor by tensor in ``flats`` order across the groups, skipping zero norms.
    ``philox``: key = ``key`` (+ the group's index), stream offset = ``call_index``.
    """
    if rng not in ("philox", "mt19937"):
        raise ValueError(f"unknown rng={rng!r}; expected 'philox' or 'mt19937'")
    members: Dict[torch.dtype, List[int]] = {}
    for i, f in enumerate(flats):
        value_format(f.dtype)
        members.setdefault(f.dtype, []).append(i)
    groups = []
    for dt, idx in members.items():
        plan = codec.Plan.get([int(flats[i].numel()) for i in idx], device=dev, chunk=chunk)
        groups.append((plan, _arena([flats[i] for i in idx], dev, plan), value_format(dt), idx))
    s = int(bit_width)
    out = []
    if rng == "mt19937":
        # Parity mode: each norm is the reference's own op on the host, torch.norm of the
        # (weighted) tensor's CPU copy in its dtype (qsgd.py:46 after global_grpc.py:101-123's
        # torch.mul) - so the payload is the reference's bit for bit on the same host, not only
        # when the GPU's fp32 norm happens to round alike.
        host = []
        for plan, x, fmt, idx in groups:
            hn = []
            for i in idx:
                v = flats[i].detach().reshape(-1)
                if alpha != 1.0:
                    v = torch.mul(v, alpha)
                hn.append(float(torch.norm(v.cpu()).item()))
            host.append(hn)
        norms = [torch.tensor(hn, dtype=torch.float32).to(dev) for hn in host]
        where = {i: (g, k) for g, (_, _, _, idx) in enumerate(groups) for k, i in enumerate(idx)}
        u_host = [torch.zeros(plan.arena_end, dtype=torch.float32) for plan, _, _, _ in groups]
        for i in range(len(flats)):  # the reference's draw order: tensor by tensor
            g, k = where[i]
            plan = groups[g][0]
            if host[g][k] != 0:
                o, n = plan.offsets[k], plan.sizes[k]
                u_host[g][o:o + n] = torch.rand(n)
        for (plan, x, fmt, idx), nd, uh in zip(groups, norms, u_host):
            q, nd = plan.qsgd_encode(x, s, alpha=alpha, u=uh.to(dev), norm_in=nd, value_format=fmt)
            out.append((plan, q, nd, idx))
    else:
        for g, (plan, x, fmt, idx) in enumerate(groups):
            q, nd = plan.qsgd_encode(x, s, alpha=alpha, seed=(int(key) + g) & (2**64 - 1), offset=call_index,
                                     value_format=fmt)
            out.append((plan, q, nd, idx))
    return out


def encode_many(flats: Sequence[torch.Tensor], bit_width: int, dev: torch.device, rng: str = "philox",
                call_index: int = 0, alpha: float = 1.0, chunk: int = 0, key: int = 0):
    """Encode flat tensors of ONE dtype in one launch: ``(plan, q_arena, norms_dev)``."""
    groups = encode_groups(flats, bit_width, dev, rng, call_index, alpha, chunk, key)
    if len(groups) != 1:
        raise ValueError("encode_many: the tensors must share one dtype (use encode_groups)")
    plan, q, norms, _ = groups[0]
    return plan, q, norms


_INSTANCES = itertools.count()


def client_identity() -> int:
    """This process's client identity: its rank in the default process group when one is
    initialised, else the launcher's ``RANK`` environment variable, else 0."""
    import os

    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return int(dist.get_rank())
    try:
        return int(os.environ.get("RANK", "0"))
    except ValueError:
        return 0


def philox_key(instance: int, client: int = 0) -> int:
    """64-bit Philox key of a compressor: splitmix64 of (torch.initial_seed(), creation index,
    client identity).  The identity keeps clients that share a seed (every process calling the
    reference's ``set_seed(1234)``, omnifed/data/utils.py:22) from drawing the same uniforms at
    every arena position, which would correlate their rounding errors and void the 1/N variance
    reduction of averaging N clients."""
    z = (int(torch.initial_seed()) * 0x9E3779B97F4A7C15 + int(instance) * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB
         + int(client) * 0xD1B54A32D192ED03)
    z &= 2**64 - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
    return z ^ (z >> 31)


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
        self._instance = next(_INSTANCES)
        self.client_id: Optional[int] = None  # None: client_identity() (the process's rank)

    def philox_key(self) -> int:
        """The Philox key of this compressor (see the module docstring)."""
        cid = client_identity() if self.client_id is None else int(self.client_id)
        return philox_key(self._instance, cid)

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

    def encode_flat(self, flats: List[torch.Tensor], alpha: float = 1.0) -> List[Tuple]:
        """Batched ``quantize_vector``: one launch for every tensor (all must be non-empty floats).

        ``alpha``: the client weighting ``param * batch_samples`` of GrpcCommunicator.aggregate
        (global_grpc.py:101-123), fused into the encoder: the levels are those of fl32(alpha * x).
        Returns a ``(q_device_view, norm, width, levels)`` per tensor, or
        ``(None, -1, -1, -1)`` for a zero norm.
        """
        if not (0 <= self.s <= 30):
            # levels = 2**s must fit LayerState.level (int32); the reference fails there too.
            raise ValueError(f"QSGD bit_width={self.s} out of range [0, 30]")
        dev = compute_device(flats[0], self.device)
        groups = encode_groups(flats, self.s, dev, self.rng, self._next_call(), alpha=alpha, key=self.philox_key())
        levels = 2**self.s
        width, _ = choose_qsgd_storage_width(levels)
        out: List[Tuple] = [None] * len(flats)
        for plan, q, norms, idx in groups:
            host_norms = norms.cpu().tolist()  # synchronises the stream
            plan.check()  # an in-kernel timeout raises (the payload would be invalid)
            for i, o, n, nv in zip(idx, plan.offsets, plan.sizes, host_norms):
                out[i] = (None, -1, -1, -1) if nv == 0 else (q[o:o + n], float(nv), width, levels)
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
