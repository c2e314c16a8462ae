"""Top-K oracle: the reference's torch-CPU op sequence, restated — TEST INFRASTRUCTURE ONLY.

Follows ``/root/reference/src/omnifed/hybrid/compression/``:

* ``topk_k``          ↔ ``max(1, int(numel * ratio))`` (topk.py:12)
* ``topk_sparse``     ↔ ``topk_sparse`` (topk.py:10-15): ``torch.topk(|x|, k, sorted=False)``
* ``topk_desparse``   ↔ ``topk_desparse`` (topk.py:18-21)
* ``TopKOracle``      ↔ ``TopKCompression.compress/decompress`` (topk.py:24-47) with
  ``ResidualUpdates`` error feedback (core.py:19-37, beta = gamma = 1)

``torch.topk``'s output order is implementation defined and ties are unspecified
(SURVEY.md §7 hard part 6), so tests compare index *sets* and decoded tensors.
"""

from __future__ import annotations

import torch


def topk_k(numel: int, ratio: float) -> int:
    return max(1, int(numel * float(ratio)))


def topk_sparse(t: torch.Tensor, ratio: float):
    flat = t.flatten()
    k = topk_k(flat.numel(), ratio)
    _, idx = torch.topk(flat.abs(), k, sorted=False)
    return torch.gather(flat, 0, idx), idx


def topk_desparse(values: torch.Tensor, indices: torch.Tensor, numel: int) -> torch.Tensor:
    out = torch.zeros(numel, dtype=values.dtype)
    out.scatter_(0, indices, values)
    return out


class TopKOracle:
    """TopKCompression with error feedback, CPU."""

    def __init__(self, compress_ratio: float = 0.01):
        self.compress_ratio = float(compress_ratio)
        self.residuals = {}

    def compress(self, t: torch.Tensor, name: str):
        t = t.detach().cpu()
        if name in self.residuals:
            t = 1.0 * self.residuals[name] + 1.0 * t
        numel, shape = t.numel(), t.size()
        values, indices = topk_sparse(t, self.compress_ratio)
        dec = topk_desparse(values, indices, numel).view(shape)
        self.residuals[name] = t - dec
        return (values, indices), (numel, shape)

    @staticmethod
    def decompress(tensors, ctx):
        numel, shape = ctx
        values, indices = tensors
        return topk_desparse(values, indices, numel).view(shape)
