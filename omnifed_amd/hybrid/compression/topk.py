"""Top-K sparsification with error feedback on MI355X (mirror of ``src/omnifed/hybrid/compression/topk.py``).

``TopKCompression.compress`` = compensate (t' = residual + x) → select the
k = max(1, int(n·ratio)) largest |t'| → residual := t' − desparse(selection)
(topk.py:33-42, core.py:26-37), all in ``omf_topk_encode``; the per-name
residual lives on the GPU in ``self.residual.residuals[name]`` (flat fp32).
Selection order: descending |t'|, ties by ascending index — torch.topk's order
for k·64 <= n on the reference CPU path (its ties are unspecified).
"""

from __future__ import annotations

import torch

from ... import codec
from .core import Compression, ResidualUpdates, compute_device, to_arena

TOPK_COMPRESSION_NAME = "TopKCompression"


def topk_sparse(tensor: torch.Tensor, compress_ratio: float):
    """topk.py:10-15 without error feedback: ``(values, indices)`` of the flat tensor."""
    dev = compute_device(tensor, torch.device("cpu"))
    n = tensor.numel()
    plan = codec.Plan.get([n], device=dev)
    x = to_arena(tensor, dev, plan)
    values, indices, _ = plan.topk_encode(x, compress_ratio)
    return values.to(tensor.device), indices.to(tensor.device)


def topk_desparse(values: torch.Tensor, indices: torch.Tensor, numel: int, device):
    """topk.py:18-21: zeros of ``numel`` with ``values`` scattered at ``indices``."""
    out_dev = torch.device(device)
    dev = compute_device(values, out_dev)
    y = torch.empty(max(int(numel), 4), dtype=values.dtype if values.dtype == torch.float32 else torch.float32,
                    device=dev)
    codec.topk_decode(values.to(dev, torch.float32), indices.to(dev, torch.int64), int(numel), y=y, mode=0)
    return y[: int(numel)].to(out_dev)


class TopKCompression(Compression):
    """Top-k sparsification with error feedback (largest-magnitude elements)."""

    def __init__(self, device="cpu", compress_ratio: float = 0.01):
        super().__init__()
        self.residual = ResidualUpdates()
        self.device = torch.device(device)
        self.compress_ratio = float(compress_ratio)

    def compress(self, tensor: torch.Tensor, name: str):
        """topk.py:33-42: ``((values, indices), (numel, shape))``; mutates the residual of ``name``."""
        return self.compress_weighted(tensor, name, 1.0)

    def compress_weighted(self, tensor: torch.Tensor, name: str, alpha: float):
        """``compress(fl32(alpha * tensor), name)`` with the weighting fused into the encoder (the
        client weighting param * batch_samples, global_grpc.py:101-123)."""
        if tensor.is_floating_point() and tensor.dtype != torch.float32:
            # The reference selects and keeps its residual in the tensor's dtype; this codec's Top-K
            # is fp32 (integer tensors are selected on their exact fp32 values, as the wire's
            # astype(float32) sends them; a bf16 tensor fails in the reference's wire encode anyway:
            # numpy has no bfloat16).
            raise ValueError(f"Top-K on the MI355X codec encodes float32 (or integer) tensors, not {tensor.dtype}")
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
                                              alpha=float(alpha))
        self.residual.residuals[name] = res
        ctx = (numel, shape)
        return (values.to(self.device), indices.to(self.device)), ctx

    def decompress(self, tensors, ctx):
        numel, shape = ctx
        values, indices = tensors
        return topk_desparse(values, indices, numel, self.device).view(shape)
