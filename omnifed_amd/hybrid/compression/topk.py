"""Top-K sparsification with error feedback on MI355X (mirror of ``src/omnifed/hybrid/compression/topk.py``).

``TopKCompression.compress`` = compensate (t' = residual + x) → select the
k = max(1, int(n·ratio)) largest |t'| → residual := t' − desparse(selection)
(topk.py:33-42, core.py:26-37), all in ``omf_topk_encode``; the per-name
residual lives on the GPU in ``self.residual.residuals[name]`` (flat fp32).  ``encode_arena``
(the batched wire path, ``encode_updates_dict``) encodes a whole update dict in one call; its
residuals live in one compressor-owned arena per dict layout and ``residuals[name]`` are views
of it, so the per-tensor and the batched paths share the same error-feedback state.
Selection (``tie_order``, default "torch"): the reference's bytes — where magnitudes tie, which of
them are selected at rank k and their order are those of torch's CPU ``topk`` (libstdc++
partial_sort / nth_element; ``omf_topk_torch_order``, host work on the tied tensors only).
"index": the device selection alone, (|t'| descending, index ascending), asynchronous; identical
bytes whenever k*64 <= n and no two of the k+1 largest |t'| of a tensor tie (decoded tensors also
agree when ties stay inside the selection, and in the nth_element regime k*64 > n without ties).
"""

from __future__ import annotations

import torch

from ... import codec
from .core import Compression, ResidualUpdates, compute_device, gather_arena, to_arena

TOPK_COMPRESSION_NAME = "TopKCompression"


def topk_sparse(tensor: torch.Tensor, compress_ratio: float, tie_order: str = "torch"):
    """topk.py:10-15 without error feedback: ``(values, indices)`` of the flat tensor."""
    dev = compute_device(tensor, torch.device("cpu"))
    n = tensor.numel()
    plan = codec.Plan.get([n], device=dev)
    x = to_arena(tensor, dev, plan)
    values, indices, _ = plan.topk_encode(x, compress_ratio, tie_order=tie_order)
    vdt = tensor.dtype if tensor.dtype in (torch.float16, torch.bfloat16) else values.dtype
    return values.to(tensor.device, vdt), indices.to(tensor.device)


def topk_desparse(values: torch.Tensor, indices: torch.Tensor, numel: int, device):
    """topk.py:18-21: zeros of ``numel`` with ``values`` scattered at ``indices``."""
    out_dev = torch.device(device)
    dev = compute_device(values, out_dev)
    y = torch.empty(max(int(numel), 4), dtype=values.dtype if values.dtype == torch.float32 else torch.float32,
                    device=dev)
    codec.topk_decode(values.to(dev, torch.float32), indices.to(dev, torch.int64), int(numel), y=y, mode=0)
    out = y[: int(numel)]
    if values.dtype in (torch.float16, torch.bfloat16):  # zeros of values.dtype (exact narrowing)
        out = out.to(values.dtype)
    return out.to(out_dev)


def topk_index_offset(K: int) -> int:
    """Byte offset of the indices in a combined (values, indices) buffer of K selected values."""
    return (4 * int(K) + 255) // 256 * 256


class TopKCompression(Compression):
    """Top-k sparsification with error feedback (largest-magnitude elements)."""

    def __init__(self, device="cpu", compress_ratio: float = 0.01, tie_order: str = "torch"):
        super().__init__()
        self.residual = ResidualUpdates()
        self.device = torch.device(device)
        self.compress_ratio = float(compress_ratio)
        if tie_order not in ("torch", "index"):
            raise ValueError(f"tie_order must be 'torch' or 'index', not {tie_order!r}")
        self.tie_order = tie_order  # module docstring
        self._arenas = {}  # residual arenas of the batched path, per dict layout

    def compress(self, tensor: torch.Tensor, name: str):
        """topk.py:33-42: ``((values, indices), (numel, shape))``; mutates the residual of ``name``."""
        return self.compress_weighted(tensor, name, 1.0)

    def _unit_residual_weights(self) -> None:
        """The error-feedback kernels compute t' = residual + x: ResidualUpdates' beta = gamma = 1,
        the only values the reference's TopKCompression constructs (topk.py:29)."""
        if self.residual.beta != 1.0 or self.residual.gamma != 1.0:
            raise ValueError(f"Top-K error feedback runs with beta = gamma = 1 (got beta={self.residual.beta}, "
                             f"gamma={self.residual.gamma})")

    def compress_weighted(self, tensor: torch.Tensor, name: str, alpha: float):
        """``compress(fl32(alpha * tensor), name)`` with the weighting fused into the encoder (the
        client weighting param * batch_samples, global_grpc.py:101-123)."""
        self._unit_residual_weights()
        if tensor.dtype in (torch.float16, torch.bfloat16):
            return self._compress_half(tensor, name, alpha)
        if tensor.is_floating_point() and tensor.dtype != torch.float32:
            # fp64: the reference would select on fp64 magnitudes and round the values to fp32 on
            # the wire; this codec's Top-K selects in fp32 / fp16 / bf16 (integer tensors on their
            # exact fp32 values, as the wire's astype(float32) sends them).
            raise ValueError(f"Top-K on the MI355X codec encodes float32/float16/bfloat16 (or integer) "
                             f"tensors, not {tensor.dtype}")
        dev = compute_device(tensor, self.device)
        numel = tensor.numel()
        shape = tensor.size()
        plan = codec.Plan.get([numel], device=dev)
        x = to_arena(tensor, dev, plan)
        res = self.residual.residuals.get(name)
        if res is not None and (res.device != dev or res.numel() != numel or res.dtype != torch.float32):
            res = res.reshape(-1).to(dev, torch.float32).contiguous()
            if res.numel() != numel:
                raise ValueError(f"residual for {name!r} has {res.numel()} elements, tensor has {numel}")
        mode = 1 if res is not None else 2
        if res is None:
            res = torch.empty(numel, dtype=torch.float32, device=dev)
        values, indices, _ = plan.topk_encode(x, self.compress_ratio, residual=res, residual_mode=mode,
                                              alpha=float(alpha), tie_order=self.tie_order)
        self.residual.residuals[name] = res
        ctx = (numel, shape)
        return (values.to(self.device), indices.to(self.device)), ctx

    def _compress_half(self, tensor: torch.Tensor, name: str, alpha: float):
        """fp16 / bf16 tensors, in the tensor's dtype as the reference computes them: the weighting
        (``param * batch_samples``) and ``compensate`` (``beta * residual + gamma * tensor``,
        core.py:26-30) are the reference's own torch expressions, evaluated on the GPU; t' is then
        widened to fp32 (exact) and the selection and the residual update (t' with the selected
        slots zeroed: core.py:32-37's ``t' - desparse``) are the fp32 kernel's, whose magnitude
        order on the widened values is the half-precision order.  Values come back in the tensor's
        dtype (exact), the residual is kept in it."""
        dev = compute_device(tensor, self.device)
        t = tensor.detach().to(dev).reshape(-1)
        if float(alpha) != 1.0:
            t = torch.mul(t, float(alpha))
        res = self.residual.residuals.get(name)
        if res is not None:
            if res.numel() != t.numel():
                raise ValueError(f"residual for {name!r} has {res.numel()} elements, tensor has {t.numel()}")
            t = self.residual.beta * res.to(dev).reshape(-1) + self.residual.gamma * t
        numel, shape = tensor.numel(), tensor.size()
        plan = codec.Plan.get([numel], device=dev)
        x = to_arena(t, dev, plan)  # exact widening (or t itself when the compensate promoted to fp32)
        r = torch.empty(numel, dtype=torch.float32, device=dev)
        values, indices, _ = plan.topk_encode(x, self.compress_ratio, residual=r, residual_mode=2,
                                              tie_order=self.tie_order)
        self.residual.residuals[name] = r.to(t.dtype)
        return (values.to(self.device, t.dtype), indices.to(self.device)), (numel, shape)

    def _residual_arena(self, names, plan):
        """The residual arena of the dict layout (``names``, ``plan``) and the encoder's residual
        mode: each name's current residual copied in unless ``residuals[name]`` already is its
        view of the arena; a name with no residual yet gets -0.0, the additive identity (-0 + a
        = a for every a, signed zeros and NaN payloads included), so one compensating launch
        (mode 1) computes exactly the reference's ``compensate`` for every name (core.py:26-31).
        Mode 2 (no read) when no name has a residual."""
        key = (tuple(names), tuple(plan.sizes), str(plan.device))
        arena = self._arenas.get(key)
        if arena is None:
            if len(self._arenas) >= 4:
                self._arenas.pop(next(iter(self._arenas)))
            arena = torch.empty(max(plan.arena_end, 4), dtype=torch.float32, device=plan.device)
            self._arenas[key] = arena
        base = arena.data_ptr()
        fresh = []
        for t, name in enumerate(names):
            o, n = plan.offsets[t], plan.sizes[t]
            r = self.residual.residuals.get(name)
            if r is None:
                fresh.append(t)
            elif not (r.data_ptr() == base + 4 * o and r.numel() == n and r.dtype == torch.float32
                      and r.device == plan.device):
                if r.numel() != n:
                    raise ValueError(f"residual for {name!r} has {r.numel()} elements, tensor has {n}")
                arena[o:o + n].copy_(r.reshape(-1))
        if len(fresh) == len(names):
            return arena, 2
        for t in fresh:
            arena[plan.offsets[t]:plan.offsets[t] + plan.sizes[t]].fill_(-0.0)
        return arena, 1

    def _residual_arena_half(self, names, plan, dt):
        """``_residual_arena`` for a dict of ``dt`` (fp16 / bf16) tensors: the residuals live in a
        ``dt`` arena (the reference keeps them in the tensor's dtype); a fresh name gets -0.0, the
        additive identity in half precision too.  Returns (arena, any residual present)."""
        key = (tuple(names), tuple(plan.sizes), str(plan.device), dt)
        arena = self._arenas.get(key)
        if arena is None:
            if len(self._arenas) >= 4:
                self._arenas.pop(next(iter(self._arenas)))
            arena = torch.empty(max(plan.arena_end, 4), dtype=dt, device=plan.device)
            self._arenas[key] = arena
        base, isz = arena.data_ptr(), arena.element_size()
        fresh = []
        for t, name in enumerate(names):
            o, n = plan.offsets[t], plan.sizes[t]
            r = self.residual.residuals.get(name)
            if r is None:
                fresh.append(t)
            elif not (r.data_ptr() == base + isz * o and r.numel() == n and r.dtype == dt and r.device == plan.device):
                if r.numel() != n:
                    raise ValueError(f"residual for {name!r} has {r.numel()} elements, tensor has {n}")
                arena[o:o + n].copy_(r.reshape(-1))
        for t in fresh:
            arena[plan.offsets[t]:plan.offsets[t] + plan.sizes[t]].fill_(-0.0)
        return arena, len(fresh) < len(names)

    def _encode_arena_half(self, names, flats, alpha, out):
        """``encode_arena`` for a dict of one half dtype: the weighting and ``compensate`` are the
        reference's torch expressions in that dtype over the whole dict's arena (as _compress_half
        per tensor), then ONE fp32 selection launch on the exactly widened t'."""
        dt = flats[0].dtype
        dev = compute_device(flats[0], self.device)
        plan = codec.Plan.get([int(f.numel()) for f in flats], device=dev)
        ks = plan.topk_ks(self.compress_ratio)
        K = sum(ks)
        h = torch.empty(plan.arena_end, dtype=dt, device=dev)
        for f, o, n in zip(flats, plan.offsets, plan.sizes):
            h[o:o + n].copy_(f.detach().reshape(-1))
        if float(alpha) != 1.0:
            h = torch.mul(h, float(alpha))
        res, present = self._residual_arena_half(names, plan, dt)
        if present:
            h = self.residual.beta * res + self.residual.gamma * h
        x = h.float()  # exact widening (padding is never read)
        r = torch.empty(plan.arena_end, dtype=torch.float32, device=dev)
        if out is None:
            out = torch.empty(topk_index_offset(K) + 8 * K, dtype=torch.uint8, device=dev)
        io = topk_index_offset(K)
        values = out[:4 * K].view(torch.float32)
        indices = out[io:io + 8 * K].view(torch.int64)
        plan.topk_encode(x, self.compress_ratio, residual=r, residual_mode=2, values=values, indices=indices,
                         tie_order=self.tie_order)
        res[:plan.arena_end].copy_(r)  # exact narrowing (t' and zeros are dt values)
        for t, name in enumerate(names):
            o, n = plan.offsets[t], plan.sizes[t]
            self.residual.residuals[name] = res[o:o + n]
        return plan, values, indices, ks

    def encode_arena(self, names, flats, alpha: float = 1.0, out: "torch.Tensor" = None):
        """``compress_weighted(flat, name, alpha)`` for every (name, flat) in ONE encode call
        (flats: non-empty fp32 tensors; the residuals become views of one arena).  Returns
        ``(plan, values, indices, ks)``: tensor t's selection at ``[sum(ks[:t]), + ks[t])``.
        ``out`` (optional uint8 device buffer): values are written at its start and indices at
        byte ``topk_index_offset(K)``, so one device-to-host copy fetches both.  A dict of one
        half dtype (fp16 / bf16) keeps its residuals in that dtype (``_encode_arena_half``)."""
        self._unit_residual_weights()
        if flats[0].dtype in (torch.float16, torch.bfloat16):
            return self._encode_arena_half(names, flats, alpha, out)
        dev = compute_device(flats[0], self.device)
        plan = codec.Plan.get([int(f.numel()) for f in flats], device=dev)
        ks = plan.topk_ks(self.compress_ratio)
        K = sum(ks)
        x = gather_arena(flats, dev, plan)
        res, mode = self._residual_arena(names, plan)
        if out is None:
            out = torch.empty(topk_index_offset(K) + 8 * K, dtype=torch.uint8, device=dev)
        io = topk_index_offset(K)
        values = out[:4 * K].view(torch.float32)
        indices = out[io:io + 8 * K].view(torch.int64)
        plan.topk_encode(x, self.compress_ratio, residual=res, residual_mode=mode, values=values, indices=indices,
                         alpha=float(alpha), tie_order=self.tie_order)
        base = res.data_ptr()
        for t, name in enumerate(names):
            o, n = plan.offsets[t], plan.sizes[t]
            r = self.residual.residuals.get(name)
            if r is None or r.data_ptr() != base + 4 * o or r.numel() != n:
                self.residual.residuals[name] = res[o:o + n]
        return plan, values, indices, ks

    def decompress(self, tensors, ctx):
        numel, shape = ctx
        values, indices = tensors
        return topk_desparse(values, indices, numel, self.device).view(shape)
