"""Compression plugin base types (mirror of ``src/omnifed/hybrid/compression/core.py``).

``Compression`` / ``ResidualMemory`` / ``ResidualUpdates`` keep the reference's
names and semantics (core.py:9-59).  ``TopKCompression`` does not call
``compensate``/``update`` — the HIP encoder fuses both into its first pass — but
the residual store lives here under the same attribute (``residuals``), holding
device tensors.  ``layerwise_decompress`` (core.py:62-71) runs as a GPU
scatter-add followed by an IEEE division.
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import torch

from ... import codec


class ResidualMemory(ABC):
    @abstractmethod
    def compensate(self, tensor, name):
        """Update the tensor with the residuals."""
        raise NotImplementedError("compensate was not implemented.")

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        """Update the residuals."""


class ResidualUpdates(ResidualMemory):
    """Error-feedback memory, core.py:19-37 (beta = gamma = 1 by default)."""

    def __init__(self, beta=1.0, gamma=1.0):
        self.residuals = {}
        self.beta = beta
        self.gamma = gamma
        self.layer_decompress = {}

    def compensate(self, tensor, name):
        if name in self.residuals:
            res = self.residuals[name]
            tensor = self.beta * res.reshape(-1)[: tensor.numel()].view(tensor.shape).to(tensor.device) + \
                self.gamma * tensor
        return tensor

    def update(self, tensor, name, compressor, tensor_compressed, ctx):
        tensor_decompressed = compressor.decompress(tensor_compressed, ctx)
        self.layer_decompress[name] = tensor_decompressed
        self.residuals[name] = tensor - tensor_decompressed.to(tensor.device)


class Compression:
    """Interface for compressing and decompressing a given tensor (core.py:40-59)."""

    def __init__(self, average=True, is_tensor_size_same=True):
        self.average = average
        self.is_tensor_size_same = is_tensor_size_same

    def compress(self, tensor, **kwargs):
        raise NotImplementedError("compress not implemented.")

    def decompress(self, **kwargs):
        raise NotImplementedError("decompress not implemented.")

    def loss_scaling(self, loss):
        raise NotImplementedError("loss_scaling not implemented.")

    def gradient_unscaling(self, **kwargs):
        raise NotImplementedError("gradient_unscaling not implemented.")


def compute_device(t: torch.Tensor, preferred: torch.device) -> torch.device:
    """Where the codec runs for ``t``: its own GPU, the compressor's GPU, or the current GPU."""
    if t.is_cuda:
        return t.device
    if preferred.type == "cuda":
        return preferred if preferred.index is not None else torch.device("cuda", torch.cuda.current_device())
    if not torch.cuda.is_available():
        raise RuntimeError("the omnifed_amd codec runs on an MI355X GPU; no GPU is visible (there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def to_arena(t: torch.Tensor, dev: torch.device, plan: "codec.Plan") -> torch.Tensor:
    """A 16-byte aligned fp32 arena on ``dev`` holding ``t`` flattened (no copy when already suitable)."""
    flat = t.detach().reshape(-1)
    if flat.dtype == torch.float32 and flat.device == dev and flat.is_contiguous() and flat.data_ptr() % 16 == 0:
        return flat
    buf = torch.empty(max(plan.arena_end, 1), dtype=torch.float32, device=dev)
    buf[: flat.numel()].copy_(flat, non_blocking=False)
    return buf


def shared_arena(flats, dev: torch.device, plan: "codec.Plan"):
    """The arena ``flats`` already form, if they do: every flat is a contiguous fp32 view of ONE
    storage on ``dev`` at ``base + plan.offsets[t]`` (a model's flat gradient buffer, the PS's
    average arena), 16-byte aligned and long enough for the plan — then that storage is the
    arena (no copy).  None otherwise."""
    f0 = flats[0]
    if f0.dtype != torch.float32 or f0.device != dev:
        return None
    st = f0.untyped_storage()
    sptr = st.data_ptr()
    base = f0.storage_offset() - plan.offsets[0]
    if base < 0 or (sptr + 4 * base) % 16 or st.nbytes() < 4 * (base + plan.arena_end):
        return None
    for f, o in zip(flats, plan.offsets):
        if (f.dtype != torch.float32 or not f.is_contiguous() or f.storage_offset() != base + o
                or f.untyped_storage().data_ptr() != sptr):
            return None
    return torch.empty(0, dtype=torch.float32, device=dev).set_(st, base, (plan.arena_end,))


def gather_arena(flats, dev: torch.device, plan: "codec.Plan") -> torch.Tensor:
    """The fp32 update arena of ``flats`` (flat tensors in plan order): the storage they already
    share (``shared_arena``), else a fresh arena they are copied into (bf16/fp16 -> fp32 exact)."""
    if len(flats) == 1:
        return to_arena(flats[0], dev, plan)
    x = shared_arena(flats, dev, plan)
    if x is not None:
        return x
    x = torch.empty(plan.arena_end, dtype=torch.float32, device=dev)
    for f, o, n in zip(flats, plan.offsets, plan.sizes):
        x[o:o + n].copy_(f.detach().reshape(-1))
    return x


def layerwise_decompress(collected_vals, collected_ix, tensor_shape, client_count, device):
    """core.py:62-71 on the GPU: scatter-add every client's (values, indices), then ``/ client_count``."""
    dev = compute_device(collected_vals[0] if collected_vals else torch.empty(0), torch.device(device))
    n = 1
    for d in tensor_shape:
        n *= int(d)
    acc = torch.zeros(max(n, 4), dtype=torch.float32, device=dev)
    for v, ix in zip(collected_vals, collected_ix):
        codec.topk_decode(v.to(dev, torch.float32), ix.to(dev, torch.int64), n, y=acc, mode=2)
    codec.div_(acc, float(client_count))
    return acc[:n].reshape(tensor_shape).to(torch.device(device))
