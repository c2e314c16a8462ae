"""TopK and QSGD encode/decode for hybrid global ``LayerState`` messages — GPU-backed drop-in.

Mirror of ``src/omnifed/hybrid/communicator/global_grpc_compression.py``: same
function names, keyword arguments, dispatch rules, wire fields, dtype strings
and ``ValueError``/``TypeError`` behaviour (:23-223).  Differences are where the
work happens, not what is produced:

* the codec runs on the GPU; only the payload crosses PCIe (w·N bytes instead of
  the reference's 4·N ``.cpu()`` copy at :105);
* ``encode_updates_dict`` encodes every QSGD tensor of the dict in ONE kernel
  launch (``omf_qsgd_encode`` over an update arena) and fetches the payload
  arena through pinned staging in chunks, the host copies into ``bytes`` done by
  worker threads while earlier messages are built (``omnifed_amd.hostio``);
* ``decode_updates_dict`` decodes every QSGD layer of a message in ONE launch from
  pinned staging (chunked host-to-device copies overlapped with the reading of
  later messages), and
  ``decode_updates_into`` (client downlink, global_grpc_client.py:98-111) writes the
  decoded tensors straight into the model's device tensors;
* decoders take an optional ``device=`` (default: the reference's placement —
  ``base_tensor.device`` when given, else CPU);
* the first batched encode / decode sets the process's host-memory policy
  (``hostio.retain_host_memory``: freed message memory is kept for the next round instead
  of being unmapped and faulted in again, 4 KiB at a time) — ``OMF_RETAIN_HOST_MEMORY=0``
  leaves glibc's defaults alone.
"""

from __future__ import annotations

import logging
import os
from typing import Dict, List, Optional, Union

import numpy as np
import torch

from . import global_grpc_pb2
from ..compression.qsgd import (
    QSGD_COMPRESSION_NAME,
    QSGD_PACKED_COMPRESSION_NAME,
    QSGDQuantCompression,
    choose_qsgd_storage_width,
    should_compress_tensor,
)
from ..compression.topk import TOPK_COMPRESSION_NAME, TopKCompression, topk_index_offset
from ..compression.core import compute_device
from ... import codec, hostio

GlobalHybridCompressor = Union[TopKCompression, QSGDQuantCompression]

_QSGD_NUMPY_DTYPES = {8: np.int8, 32: np.int32}
_QSGD_TORCH_DTYPES = {8: torch.int8, 32: torch.int32}
_QSGD_TYPES = (QSGD_COMPRESSION_NAME, QSGD_PACKED_COMPRESSION_NAME)


_STAGING = hostio.STAGING
_HOST_POLICY: Optional[bool] = None


def _host_memory_policy() -> bool:
    """Once per process: retain freed host memory (hostio.retain_host_memory) unless
    OMF_RETAIN_HOST_MEMORY=0.  The payload messages of a round are ~w·N bytes of fresh memory;
    with glibc's defaults they are unmapped when freed and every 4 KiB page of the next round's
    faults on first touch (98 -> 29 ms per Llama-400M encode_updates_dict)."""
    global _HOST_POLICY
    if _HOST_POLICY is None:
        _HOST_POLICY = os.environ.get("OMF_RETAIN_HOST_MEMORY", "1") != "0" and hostio.retain_host_memory()
        if _HOST_POLICY:
            logging.getLogger("omnifed_amd").info(
                "omnifed_amd: glibc malloc now keeps freed wire-message memory for reuse (mmap threshold 32 MiB, "
                "trim threshold 1 GiB per arena; resident size may stay ~one round's payload higher), and "
                "decoded arenas returned on the CPU reuse pooled pageable pages (hostio.HOST_ARENAS, up to 8 GiB "
                "kept; page-locked only if OMF_PIN_HOST_ARENAS gives them a budget). OMF_RETAIN_HOST_MEMORY=0 "
                "leaves glibc's defaults alone and allocates every arena afresh (INTEGRATION.md §3c).")
    return _HOST_POLICY


def compression_mode_name(compressor: Optional[GlobalHybridCompressor]) -> str:
    """global_grpc_compression.py:24-31."""
    if compressor is None:
        return "dense"
    if isinstance(compressor, TopKCompression):
        return "TopK"
    if isinstance(compressor, QSGDQuantCompression):
        return "QSGD"
    return type(compressor).__name__


def build_global_compressor(*, enabled: bool, scheme: str = "topk", compress_ratio: float = 0.01,
                            bit_width: int = 8, device="cpu", packed_wire: bool = False) -> Optional[GlobalHybridCompressor]:
    """global_grpc_compression.py:35-52.  ``packed_wire`` (QSGD only, default off): the opt-in
    bit-packed wire (``QSGDBitPackedCompression``, not readable by the reference)."""
    if not enabled:
        return None
    scheme_norm = str(scheme).lower()
    if scheme_norm == "topk":
        return TopKCompression(device=device, compress_ratio=float(compress_ratio))
    if scheme_norm == "qsgd":
        return QSGDQuantCompression(bit_width=int(bit_width), device=device, packed_wire=bool(packed_wire))
    raise ValueError(f"Unsupported global_compression.scheme={scheme!r}; expected 'topk' or 'qsgd'")


def _select(cfg, key: str, default):
    """OmegaConf.select-compatible lookup over OmegaConf configs, dicts or attribute objects."""
    try:  # an OmegaConf config, when omegaconf is installed
        from omegaconf import OmegaConf  # type: ignore

        if type(cfg).__module__.startswith("omegaconf"):
            return OmegaConf.select(cfg, key, default=default)
    except ImportError:
        pass
    cur = cfg
    for part in key.split("."):
        if isinstance(cur, dict):
            if part not in cur:
                return default
            cur = cur[part]
        elif hasattr(cur, part):
            cur = getattr(cur, part)
        else:
            return default
        if cur is None:
            return default
    return cur


def hybrid_global_compressor_from_cfg(cfg, device="cpu") -> Optional[GlobalHybridCompressor]:
    """global_grpc_compression.py:55-73 (keys engine.hybrid.global_compression.*)."""
    enabled = bool(_select(cfg, "engine.hybrid.global_compression.enabled", False))
    scheme = str(_select(cfg, "engine.hybrid.global_compression.scheme", "topk"))
    ratio = float(_select(cfg, "engine.hybrid.global_compression.compress_ratio", 0.01))
    bit_width = int(_select(cfg, "engine.hybrid.global_compression.bit_width", 8))
    packed = bool(_select(cfg, "engine.hybrid.global_compression.packed_wire", False))  # opt-in, ours
    return build_global_compressor(enabled=enabled, scheme=scheme, compress_ratio=ratio, bit_width=bit_width,
                                   device=device, packed_wire=packed)


# ---------------------------------------------------------------- layer builders (host)

def _encode_dense_layer(name: str, tensor: torch.Tensor):
    """global_grpc_compression.py:76-81."""
    layer = global_grpc_pb2.layer_state(layer_name=name)
    t = tensor.detach().cpu()
    layer.param_shape.extend(list(t.shape))
    layer.param_update.extend(t.flatten().tolist())
    return layer


def qsgd_layer_from_payload(name: str, shape, payload: bytes, norm: float, width: int, levels: int):
    """The QSGD ``LayerState`` of global_grpc_compression.py:111-123 from an encoded payload."""
    layer = global_grpc_pb2.layer_state(layer_name=name)
    layer.compression_type = QSGD_COMPRESSION_NAME
    layer.values_data = payload
    layer.values_dtype = f"torch.int{width}"
    layer.original_shape.extend(list(shape))
    layer.meta_tensor = np.array([float(norm)], dtype=np.float32).tobytes()
    layer.meta_tensor_dtype = "torch.float32"
    layer.width = int(width)
    layer.level = int(levels)
    return layer


def qsgd_packed_layer_from_payload(name: str, shape, packed: bytes, norm: float, levels: int):
    """The opt-in bit-packed QSGD ``LayerState``: the fields of the QSGD layer with
    ``values_data`` = the codes q + L in ``width`` = ceil(log2(2L+1)) bits each, LSB first."""
    layer = global_grpc_pb2.layer_state(layer_name=name)
    layer.compression_type = QSGD_PACKED_COMPRESSION_NAME
    layer.values_data = packed
    bits = codec.packed_bits(levels)
    layer.values_dtype = f"packed.u{bits}"
    layer.original_shape.extend(list(shape))
    layer.meta_tensor = np.array([float(norm)], dtype=np.float32).tobytes()
    layer.meta_tensor_dtype = "torch.float32"
    layer.width = bits
    layer.level = int(levels)
    return layer


def topk_layer_from_payload(name: str, shape, values: np.ndarray, indices: np.ndarray):
    """The Top-K ``LayerState`` of global_grpc_compression.py:88-98."""
    layer = global_grpc_pb2.layer_state(layer_name=name)
    layer.compression_type = TOPK_COMPRESSION_NAME
    layer.values_data = np.ascontiguousarray(values, dtype=np.float32).tobytes()
    layer.indices_data = np.ascontiguousarray(indices, dtype=np.int64).tobytes()
    layer.values_dtype = "torch.float32"
    layer.indices_dtype = "torch.int64"
    layer.original_shape.extend(list(shape))
    return layer


def topk_layer_from_bytes(name: str, shape, values: bytes, indices: bytes):
    """``topk_layer_from_payload`` from the payload bytes themselves (fp32 values, int64 indices)."""
    layer = global_grpc_pb2.layer_state(layer_name=name)
    layer.compression_type = TOPK_COMPRESSION_NAME
    layer.values_data = values
    layer.indices_data = indices
    layer.values_dtype = "torch.float32"
    layer.indices_dtype = "torch.int64"
    layer.original_shape.extend(list(shape))
    return layer


def _weighted(tensor: torch.Tensor, weight) -> torch.Tensor:
    """``torch.mul(tensor, batch_samples)`` of GrpcCommunicator.aggregate (global_grpc.py:104, 121)."""
    return tensor if weight is None else torch.mul(tensor.detach(), weight)


def _alpha(weight) -> float:
    return 1.0 if weight is None else float(weight)


def _encode_topk_layer(name: str, tensor: torch.Tensor, compressor: TopKCompression, weight=None):
    (values, indices), _ctx = compressor.compress_weighted(tensor.detach(), name, _alpha(weight))
    return topk_layer_from_payload(name, tuple(tensor.shape), values.detach().cpu().numpy(),
                                   indices.detach().cpu().numpy())


def _encode_qsgd_layer(name: str, tensor: torch.Tensor, compressor: QSGDQuantCompression, weight=None):
    """global_grpc_compression.py:101-123, payload produced on the GPU."""
    if not should_compress_tensor(tensor):
        return _encode_dense_layer(name, _weighted(tensor, weight))
    if getattr(compressor, "packed_wire", False) or tensor.dtype != torch.float32:
        return encode_updates_dict({name: tensor}, compressor, weight=weight)[0]
    (q, norm, width, levels), = compressor.encode_flat([tensor.detach().reshape(-1)], alpha=_alpha(weight))
    if width == -1:
        return _encode_dense_layer(name, _weighted(tensor, weight))
    payload = q.cpu().numpy().tobytes()
    return qsgd_layer_from_payload(name, tuple(tensor.shape), payload, norm, width, levels)


def encode_layer_state(name: str, tensor: torch.Tensor, compressor: Optional[GlobalHybridCompressor], *,
                       weight=None):
    """global_grpc_compression.py:126-137.

    ``weight`` (optional, ours): encode ``torch.mul(tensor, weight)`` — the client weighting
    ``param * batch_samples`` of GrpcCommunicator.aggregate (global_grpc.py:101-123) — with the
    multiply fused into the GPU encoder (same bits as multiplying first)."""
    if compressor is None:
        return _encode_dense_layer(name, _weighted(tensor, weight))
    if isinstance(compressor, TopKCompression):
        return _encode_topk_layer(name, tensor, compressor, weight)
    if isinstance(compressor, QSGDQuantCompression):
        return _encode_qsgd_layer(name, tensor, compressor, weight)
    raise TypeError(f"Unsupported compressor type: {type(compressor)!r}")


# ---------------------------------------------------------------- decode

def _out_device(base_tensor, device):
    if device is not None:
        return torch.device(device)
    if base_tensor is not None:
        return base_tensor.device
    return torch.device("cpu")


def _gpu_for(out_dev: torch.device) -> torch.device:
    """The GPU that decodes for an output placed on ``out_dev``."""
    return compute_device(torch.empty(0), out_dev)


def _last_wins(v: torch.Tensor, ix: torch.Tensor, n: int):
    """The (values, indices) that numpy's ``dense[indices] = values`` leaves when an index repeats:
    the last one per index (a GPU scatter would keep an arbitrary one).  Only for selections that
    must repeat an index (k > n: a malformed message); the encoders' selections never do."""
    pos = torch.arange(ix.numel(), device=ix.device)
    last = torch.full((n,), -1, dtype=torch.int64, device=ix.device).scatter_reduce_(0, ix, pos, "amax")
    keep = last[ix] == pos
    return v[keep], ix[keep]


def _decode_topk_layer(layer, *, base_tensor: Optional[torch.Tensor] = None, device=None,
                       last_wins: bool = False) -> torch.Tensor:
    """global_grpc_compression.py:140-160: overlay on ``base_tensor`` or zero-filled dense.
    ``last_wins``: the layer repeats an index (omf_topk_check_duplicates): numpy's rule, the last
    value per index (always applied when there are more values than elements)."""
    if not layer.values_data or not layer.indices_data:
        raise ValueError(f"Compressed layer {layer.layer_name!r} missing values/indices")
    values = np.frombuffer(layer.values_data, dtype=np.float32)
    indices = np.frombuffer(layer.indices_data, dtype=np.int64)
    original_shape = tuple(layer.original_shape)
    numel = int(np.prod(original_shape))
    if values.shape[0] != indices.shape[0]:
        raise ValueError(f"Compressed layer {layer.layer_name!r}: {values.shape[0]} values, {indices.shape[0]} indices")
    if indices.size and (indices.min() < -numel or indices.max() >= numel):
        raise IndexError(f"Compressed layer {layer.layer_name!r}: index out of bounds for size {numel}")
    if indices.size and indices.min() < 0:  # numpy fancy indexing semantics
        indices = np.where(indices < 0, indices + numel, indices)
    out_dev = _out_device(base_tensor, device)
    dev = _gpu_for(out_dev)
    v = torch.from_numpy(values.copy()).to(dev)
    ix = torch.from_numpy(np.array(indices, dtype=np.int64, copy=True)).to(dev)
    if last_wins or ix.numel() > numel:
        v, ix = _last_wins(v, ix, numel)
    if base_tensor is not None:
        # the reference overlays a numpy copy of the base, so the result has the base's dtype
        # (fp32 values cast on assignment: round-to-nearest for fp16, truncation for integers) and
        # a bf16 base fails in .numpy() as it does there
        bdt = base_tensor.dtype
        if bdt == torch.bfloat16:
            raise TypeError("Got unsupported ScalarType BFloat16")
        if bdt == torch.float64 or not (bdt.is_floating_point or bdt.is_complex):
            # the fp32 kernel cannot hold the base exactly (fp64, or integers above 2^24): the base
            # stays in its own dtype and only the assigned values are cast, as numpy's overlay does
            flat = base_tensor.detach().reshape(-1).to(dev, copy=True)
            flat[ix] = v.to(bdt)
            return flat.reshape(original_shape).to(out_dev)
        y = torch.empty(max(numel, 4), dtype=torch.float32, device=dev)
        y[:numel].copy_(base_tensor.detach().reshape(-1).to(dev, torch.float32))
        codec.topk_decode(v, ix, numel, y=y, mode=1)
        out = y[:numel].reshape(original_shape)
        return (out if bdt == torch.float32 else out.to(bdt)).to(out_dev)
    y = torch.empty(max(numel, 4), dtype=torch.float32, device=dev)
    codec.topk_decode(v, ix, numel, y=y, mode=0)
    return y[:numel].reshape(original_shape).to(out_dev)


# protobuf (upb) copies a bytes field on every read, so the payload checks take the payload the
# caller already holds (``payload``); the batched decoders check the fields first and each
# payload's size as they stage it, before anything is decoded.

def _payload_nbytes(layer) -> int:
    n = int(np.prod(tuple(layer.original_shape)))
    if layer.compression_type == QSGD_PACKED_COMPRESSION_NAME:
        return (n * layer.width + 7) // 8
    return n * (layer.width // 8)


def _check_qsgd_payload(layer, payload: bytes) -> None:
    """The size check of global_grpc_compression.py:173 (np.frombuffer(...).reshape(shape)
    raises ValueError on a mismatch) and the empty-payload check of :164-165."""
    if not payload:
        raise ValueError(f"QSGD layer {layer.layer_name!r} missing values_data")
    if len(payload) != _payload_nbytes(layer):
        kind = "packed QSGD" if layer.compression_type == QSGD_PACKED_COMPRESSION_NAME else "QSGD"
        raise ValueError(f"cannot reshape {kind} payload of {len(payload)} bytes into {tuple(layer.original_shape)}")


def _field_error(layer, msg: str):
    """Raise the reference's first error (global_grpc_compression.py:164-171 checks values_data
    before the other fields; reading it is a copy, so only on this error path)."""
    if not layer.values_data:
        raise ValueError(f"QSGD layer {layer.layer_name!r} missing values_data")
    raise ValueError(msg)


def _check_qsgd_fields(layer):
    """global_grpc_compression.py:164-171 without the payload's size (see _check_qsgd_payload)."""
    if not layer.meta_tensor:
        _field_error(layer, f"QSGD layer {layer.layer_name!r} missing meta_tensor (norm)")
    if layer.width not in _QSGD_NUMPY_DTYPES:
        _field_error(layer, f"QSGD layer {layer.layer_name!r} has unsupported width={layer.width}")
    if layer.level <= 0:
        _field_error(layer, f"QSGD layer {layer.layer_name!r} has invalid level={layer.level}")


def _check_packed_fields(layer):
    """The packed layer's fields, checked like _check_qsgd_fields checks the reference's."""
    if not layer.meta_tensor:
        _field_error(layer, f"QSGD layer {layer.layer_name!r} missing meta_tensor (norm)")
    if layer.level <= 0:
        _field_error(layer, f"QSGD layer {layer.layer_name!r} has invalid level={layer.level}")
    if layer.width != codec.packed_bits(layer.level):
        _field_error(layer, f"QSGD layer {layer.layer_name!r} has unsupported width={layer.width}")


def _check_qsgd_layer(layer, payload: bytes):
    _check_qsgd_fields(layer)
    _check_qsgd_payload(layer, payload)


def _check_packed_layer(layer, payload: bytes):
    _check_packed_fields(layer)
    _check_qsgd_payload(layer, payload)


def _decode_qsgd_layer(layer, *, device=None) -> torch.Tensor:
    """global_grpc_compression.py:163-182, decoded on the GPU."""
    if layer.compression_type == QSGD_PACKED_COMPRESSION_NAME:
        _check_packed_layer(layer, layer.values_data)
        shape = tuple(layer.original_shape)
        out_dev = _out_device(None, device)
        if int(np.prod(shape)) == 0:
            return torch.zeros(shape, dtype=torch.float32, device=out_dev)
        y, plan = _decode_qsgd_batch([layer], _gpu_for(out_dev))
        return y[:plan.sizes[0]].reshape(shape).to(out_dev)
    payload = layer.values_data  # one copy out of the message
    _check_qsgd_layer(layer, payload)
    shape = tuple(layer.original_shape)
    n = int(np.prod(shape))
    q = np.frombuffer(payload, dtype=_QSGD_NUMPY_DTYPES[layer.width])
    norm = float(np.frombuffer(layer.meta_tensor, dtype=np.float32).reshape(-1)[0])
    out_dev = _out_device(None, device)
    dev = _gpu_for(out_dev)
    if n == 0:
        return torch.zeros(shape, dtype=torch.float32, device=out_dev)
    plan = codec.Plan.get([n], device=dev)
    qd = torch.from_numpy(q.copy()).to(dev)
    nrm = torch.tensor([norm], dtype=torch.float32, device=dev)
    y = plan.qsgd_decode(qd, layer.width, layer.level, nrm)
    return y[:n].reshape(shape).to(out_dev)


def decode_layer_tensor(layer, *, base_tensor: Optional[torch.Tensor] = None, device=None) -> torch.Tensor:
    """global_grpc_compression.py:185-204."""
    compression_type = layer.compression_type or None
    if compression_type is None or compression_type == "":
        if not layer.param_shape:
            raise ValueError(f"Dense layer {layer.layer_name!r} missing param_shape")
        arr = np.array(layer.param_update, dtype=np.float32).reshape(tuple(layer.param_shape))
        out = torch.from_numpy(arr.copy())
        return out if device is None else out.to(device)
    if compression_type == TOPK_COMPRESSION_NAME:
        return _decode_topk_layer(layer, base_tensor=base_tensor, device=device)
    if compression_type in _QSGD_TYPES:
        return _decode_qsgd_layer(layer, device=device)
    raise ValueError(f"Unsupported compression_type={compression_type!r}")


# ---------------------------------------------------------------- dict helpers (batched)

def wire_size(layers) -> Dict[str, int]:
    """Wire-size figures of a list of ``LayerState``s, for the caller's metrics (SURVEY.md §5;
    the reference's docs/HYBRID_QSGD_IMPLEMENTATION_STEPS.md:373 notes QSGD's wire size is not
    yet in its CSV): ``wire_bytes`` = the serialised size of the layers (what a ModelUpdate /
    ModelParameters carries for them), ``payload_bytes`` = their values/indices/dense data,
    ``dense_fp32_bytes`` = 4 bytes per element (the uncompressed update), ``layers``."""
    wire = payload = dense = 0
    for L in layers:
        wire += L.ByteSize()
        if L.compression_type in _QSGD_TYPES:  # from the metadata: reading values_data copies it
            payload += _payload_nbytes(L)
        else:
            payload += len(L.values_data) + len(L.indices_data) + 4 * len(L.param_update)
        shape = tuple(L.original_shape) or tuple(L.param_shape)
        dense += 4 * int(np.prod(shape)) if shape else 0
    return {"wire_bytes": wire, "payload_bytes": payload, "dense_fp32_bytes": dense, "layers": len(layers)}


def encode_updates_dict(updates: Dict[str, torch.Tensor], compressor: Optional[GlobalHybridCompressor], *,
                        weight=None, stats: Optional[Dict[str, int]] = None) -> list:
    """global_grpc_compression.py:207-211; QSGD tensors go through ONE batched launch.

    ``weight``: as encode_layer_state (the client's ``batch_samples``, fused into the encoder).
    ``stats`` (optional dict, ours): receives ``wire_size`` of the returned layers."""
    _host_memory_policy()
    layers = _encode_updates(updates, compressor, weight)
    if stats is not None:
        stats.update(wire_size(layers))
    return layers


def _topk_batchable(tensors) -> bool:
    """The batched Top-K path takes non-empty tensors of one dtype, fp32 or fp16 (others: the
    per-layer path — a bf16 dict there raises the reference's TypeError at its first layer)."""
    if not tensors or not all(isinstance(t, torch.Tensor) and t.numel() > 0 for t in tensors):
        return False
    dts = {t.dtype for t in tensors}
    return dts == {torch.float32} or dts == {torch.float16}


def _encode_topk_updates(updates, compressor: TopKCompression, weight) -> list:
    """Every tensor of the dict in ONE Top-K encode (``TopKCompression.encode_arena``: error
    feedback for each name, the client weighting fused), then one chunked device-to-host copy of
    the (values, indices) buffer through pinned staging, each layer's ``bytes`` filled by worker
    threads (hostio.device_to_bytes).  Same LayerStates as the per-layer loop of
    global_grpc_compression.py:84-98 / 207-211 (the selection does not depend on the batching)."""
    names = list(updates.keys())
    flats = [updates[n].detach().reshape(-1) for n in names]
    plan, values, indices, ks = compressor.encode_arena(names, flats, _alpha(weight))
    nt = len(names)
    koff = [0]
    for k in ks:
        koff.append(koff[-1] + k)
    io = topk_index_offset(koff[-1])
    spans = [(4 * koff[t], 4 * ks[t]) for t in range(nt)] + [(io + 8 * koff[t], 8 * ks[t]) for t in range(nt)]
    buf = values.untyped_storage()
    src = torch.empty(0, dtype=torch.uint8, device=values.device).set_(buf, values.storage_offset() * 4,
                                                                         (io + 8 * koff[-1],))
    layers: List = [None] * nt
    vals: List[Optional[bytes]] = [None] * nt
    for i, payload in hostio.device_to_bytes(src, spans, key="topk_encode"):
        if i < nt:
            vals[i] = payload
        else:
            t = i - nt
            layers[t] = topk_layer_from_bytes(names[t], tuple(updates[names[t]].shape), vals[t], payload)
            vals[t] = None
    if compressor.tie_order != "torch":  # (torch order checked the plan already) an exact-tail expiry raises
        plan.check()
    return layers


def qsgd_layers_from_arena(plan, q: torch.Tensor, norms: torch.Tensor, names, shapes, levels: int,
                           packed: bool = False, stream=None) -> list:
    """The QSGD ``LayerState``s of an encoded payload arena (plan order): the norms copied first,
    then the payload arena device-to-host in chunks through pinned staging, each chunk's ``bytes``
    filled by worker threads while the previous chunk's LayerStates are built
    (hostio.device_to_bytes; protobuf copies the bytes into its message).  ``packed``: the opt-in
    bit-packed wire, packed on the GPU first.  A zero-norm tensor gets ``None`` (the caller emits
    the reference's dense passthrough); an in-kernel encoder timeout raises."""
    stream = torch.cuda.current_stream(plan.device) if stream is None else stream
    width, _ = choose_qsgd_storage_width(levels)
    with _STAGING.lease("encode_norms", 4 * plan.nt) as h:
        nh = h.buf.view(torch.float32)
        with torch.cuda.stream(stream):
            nh.copy_(norms[:plan.nt], non_blocking=True)  # queued before the payload chunks: it lands first
        ev = torch.cuda.Event()
        ev.record(stream)
        if packed:  # pack on the GPU; (b/8) bytes per element cross PCIe
            src = plan.qsgd_pack(q, width, levels, stream=stream.cuda_stream)
            b = codec.packed_bits(levels)
            spans = [(o * b // 8, (n * b + 7) // 8) for o, n in zip(plan.offsets, plan.sizes)]
        else:  # the payload arena: w bytes per element
            src, isz = q, q.element_size()
            spans = [(o * isz, n * isz) for o, n in zip(plan.offsets, plan.sizes)]
        ev.synchronize()
        host_norms = nh.tolist()
    spans = [(off, ln if nv != 0 else 0) for (off, ln), nv in zip(spans, host_norms)]  # zero norm: dense
    layers: List = [None] * plan.nt
    for k, payload in hostio.device_to_bytes(src, spans, stream=stream):
        if packed:
            layers[k] = qsgd_packed_layer_from_payload(names[k], shapes[k], payload, host_norms[k], levels)
        else:
            layers[k] = qsgd_layer_from_payload(names[k], shapes[k], payload, host_norms[k], width, levels)
    plan.check(stream.cuda_stream)  # an in-kernel timeout raises: the payload would be invalid
    return layers


def _encode_updates(updates, compressor, weight) -> list:
    if isinstance(compressor, TopKCompression) and _topk_batchable(list(updates.values())):
        return _encode_topk_updates(updates, compressor, weight)
    if not isinstance(compressor, QSGDQuantCompression):
        return [encode_layer_state(name, tensor, compressor, weight=weight) for name, tensor in updates.items()]
    names = list(updates.keys())
    comp_idx = [i for i, n in enumerate(names) if should_compress_tensor(updates[n])]
    layers: List = [None] * len(names)
    if comp_idx:
        if not (0 <= compressor.s <= 30):
            raise ValueError(f"QSGD bit_width={compressor.s} out of range [0, 30]")
        flats = [updates[names[i]].detach().reshape(-1) for i in comp_idx]
        dev = compute_device(flats[0], compressor.device)
        from ..compression.qsgd import encode_groups

        groups = encode_groups(flats, compressor.s, dev, compressor.rng, compressor._next_call(),
                               alpha=_alpha(weight), key=compressor.philox_key())
        levels = 2**compressor.s
        for plan, q, norms, members in groups:  # one group per dtype (normally one)
            idx = [comp_idx[m] for m in members]
            got = qsgd_layers_from_arena(plan, q, norms, [names[i] for i in idx],
                                         [tuple(updates[names[i]].shape) for i in idx], levels, compressor.packed_wire)
            for i, L in zip(idx, got):
                layers[i] = L
    for i, name in enumerate(names):
        if layers[i] is None:
            layers[i] = _encode_dense_layer(name, _weighted(updates[name], weight))
    return layers


def _decode_qsgd_batch(layers, dev: torch.device, host: bool = False):
    """Decode QSGD layers that share (width, level) in ONE launch.

    The payloads are staged in a plan's arena layout through pinned memory, chunk by chunk
    (hostio.bytes_to_device: each chunk's host-to-device copy overlaps the reading of the next
    chunk's payloads), and decoded by one ``omf_qsgd_decode``; returns the decoded fp32 arena
    and the plan (layer i at ``[plan.offsets[i], + plan.sizes[i])``).  ``host``: the arena is
    returned on the CPU (``_decode_qsgd_to_host``).
    """
    if host and layers[0].compression_type != QSGD_PACKED_COMPRESSION_NAME:
        return _decode_qsgd_to_host(layers, dev)
    width, level = layers[0].width, layers[0].level
    sizes = [max(int(np.prod(tuple(L.original_shape))), 1) for L in layers]
    plan = codec.Plan.get(sizes, device=dev)
    norms = np.zeros(plan.nt, dtype=np.float32)
    for i, L in enumerate(layers):
        norms[i] = np.frombuffer(L.meta_tensor, dtype=np.float32).reshape(-1)[0]
    nd = torch.from_numpy(norms).to(dev)
    if layers[0].compression_type == QSGD_PACKED_COMPRESSION_NAME:  # tensor t at byte offsets[t] * b / 8
        words = plan.packed_words(level)
        qd = torch.empty(words, dtype=torch.int32, device=dev)
        items = [(o * width // 8, (lambda L=L: L.values_data)) for L, o in zip(layers, plan.offsets)]
        hostio.bytes_to_device(items, qd, 4 * words, check=lambda i, p: _check_qsgd_payload(layers[i], p))
        y = plan.qsgd_decode_packed(qd, level, nd)
    else:
        isz = width // 8
        qd = torch.empty(plan.arena_end, dtype=_QSGD_TORCH_DTYPES[width], device=dev)
        items = [(o * isz, (lambda L=L: L.values_data)) for L, o in zip(layers, plan.offsets)]
        hostio.bytes_to_device(items, qd, isz * plan.arena_end, check=lambda i, p: _check_qsgd_payload(layers[i], p))
        y = plan.qsgd_decode(qd, width, level, nd)
    return y, plan  # stream-ordered (the staging's lease carries the event its copies complete by)


def _decode_qsgd_to_host(layers, dev: torch.device):
    """The CPU placement of a QSGD batch, pipelined: as each staged chunk's payload is queued
    host-to-device, the decode blocks it completes are decoded (omf_qsgd_decode_range) and an
    event recorded, and a second stream copies those decoded elements into the host arena while
    the next chunk is read out of its messages — the payload in and the fp32 out overlap on the
    full-duplex link.  Same bytes as
    one decode followed by one copy.  The arena is a page-locked pooled one when the opt-in budget
    of hostio.set_pinned_arenas holds it (each chunk is one DMA); otherwise pageable memory —
    pooled under the host-memory policy (hostio.HOST_ARENAS), else fresh — fed through a
    hostio.D2HRing."""
    width, level = layers[0].width, layers[0].level
    sizes = [max(int(np.prod(tuple(L.original_shape))), 1) for L in layers]
    plan = codec.Plan.get(sizes, device=dev)
    norms = np.zeros(plan.nt, dtype=np.float32)
    for i, L in enumerate(layers):
        norms[i] = np.frombuffer(L.meta_tensor, dtype=np.float32).reshape(-1)[0]
    st = torch.cuda.current_stream(dev)
    nd = torch.from_numpy(norms).to(dev)
    isz = width // 8
    N = plan.arena_end
    qd = torch.empty(N, dtype=_QSGD_TORCH_DTYPES[width], device=dev)
    y = torch.empty(N, dtype=torch.float32, device=dev)
    yb = y.view(torch.uint8)
    ob = hostio.pinned_arena(4 * N) if _HOST_POLICY else None
    pinned = ob is not None
    if ob is None:
        ob = hostio.HOST_ARENAS.empty(4 * N) if _HOST_POLICY else torch.empty(4 * N, dtype=torch.uint8)
    out = ob.view(torch.float32)
    blk = codec.DECODE_BLOCK
    side = torch.cuda.Stream(dev)
    done = [0]
    ring = None if pinned else hostio.D2HRing(out.data_ptr(), side, key="d2h_qsgd")
    try:
        def emit(upto: int) -> None:
            if upto <= done[0]:
                return
            plan.qsgd_decode(qd, width, level, nd, y_out=y, elems=(done[0], upto), stream=st.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(st)
            a, b = 4 * done[0], 4 * upto
            if pinned:  # the decoded chunk's DMA into the page-locked arena, on the side stream
                with torch.cuda.stream(side):
                    side.wait_event(ev)
                    ob[a:b].copy_(yb[a:b], non_blocking=True)
            else:
                ring.submit(yb[a:b], a, after=ev)
            done[0] = upto

        items = [(o * isz, (lambda L=L: L.values_data)) for L, o in zip(layers, plan.offsets)]
        hostio.bytes_to_device(items, qd, isz * N, stream=st, check=lambda i, p: _check_qsgd_payload(layers[i], p),
                               after_flush=lambda a, b: emit((b // isz) // blk * blk))
        emit(N)
    finally:
        if ring is not None:
            ring.close()
        side.synchronize()
    return out, plan


def read_topk_layer(layer):
    """The Top-K layer's payloads, checked as the reference's decoder checks them before any
    work (global_grpc_compression.py:145-146; np.frombuffer raises ValueError on a size that is
    not a whole number of elements, the fancy assignment on a length mismatch): ``(values bytes,
    indices bytes, k)``.  Each payload is read once (protobuf copies a bytes field on every read)."""
    v = layer.values_data
    i = layer.indices_data
    if not v or not i:
        raise ValueError(f"Compressed layer {layer.layer_name!r} missing values/indices")
    if len(v) % 4 or len(i) % 8:
        raise ValueError(f"Compressed layer {layer.layer_name!r}: buffer size must be a multiple of element size")
    if len(v) // 4 != len(i) // 8:
        raise ValueError(f"Compressed layer {layer.layer_name!r}: {len(v) // 4} values, {len(i) // 8} indices")
    return v, i, len(v) // 4


def _validate_layer(layer):
    """The checks decode_layer_tensor makes before any work (global_grpc_compression.py:
    145-146, 164-171, 193-194, 204), so a batched decode raises for the same first layer.
    Returns the Top-K payloads (read_topk_layer) for a Top-K layer, else None."""
    ct = layer.compression_type or ""
    if ct == "":
        if not layer.param_shape:
            raise ValueError(f"Dense layer {layer.layer_name!r} missing param_shape")
    elif ct == TOPK_COMPRESSION_NAME:
        return read_topk_layer(layer)
    elif ct == QSGD_COMPRESSION_NAME:
        _check_qsgd_fields(layer)  # the payload's size: checked as it is staged (_decode_qsgd_batch)
    elif ct == QSGD_PACKED_COMPRESSION_NAME:
        _check_packed_fields(layer)
    else:
        raise ValueError(f"Unsupported compression_type={ct!r}")
    return None


def _scan_layers(proto_layers):
    """Validate every layer in message order.  Returns the QSGD layers grouped by (type, width,
    level) and the Top-K layers with their payloads ``[(layer, values, indices, k)]``."""
    groups: Dict[tuple, list] = {}
    topk: List[tuple] = []
    for L in proto_layers:
        got = _validate_layer(L)
        if got is not None:
            topk.append((L, *got))
        elif L.compression_type in _QSGD_TYPES:
            groups.setdefault((L.compression_type, L.width, L.level), []).append(L)
    return groups, topk


def _layer_numel(layer) -> int:
    return int(np.prod(tuple(layer.original_shape)))


def _topk_batch_ok(topk) -> bool:
    """A message's Top-K layers decode in one call when their names are distinct (a repeated
    name: the reference's dict keeps the last decode) and every k fits its tensor."""
    names = set()
    for L, _v, _i, k in topk:
        n = _layer_numel(L)
        if n < 1 or k > n or L.layer_name in names:
            return False
        names.add(L.layer_name)
    return True


def stage_topk(pairs, dev: torch.device, key: str):
    """One device buffer holding a message's Top-K selections in plan order — values (fp32) at
    its start, indices (int64) from ``topk_index_offset(K)`` — through pinned staging in chunks
    (hostio.bytes_to_device).  ``pairs``: ``[(values bytes, indices bytes)]`` per plan tensor
    (``(b"", b"")`` for a tensor absent from the message).  Returns ``(counts, values, indices)``
    (stream-ordered)."""
    counts = [len(v) // 4 for v, _ in pairs]
    koff = [0]
    for k in counts:
        koff.append(koff[-1] + k)
    K = koff[-1]
    io = topk_index_offset(K)
    buf = torch.empty(max(io + 8 * K, 256), dtype=torch.uint8, device=dev)
    items = [(4 * koff[t], (lambda v=v: v)) for t, (v, _) in enumerate(pairs)]
    items += [(io + 8 * koff[t], (lambda i=i: i)) for t, (_, i) in enumerate(pairs)]
    hostio.bytes_to_device(items, buf, io + 8 * K, key=key)
    return counts, buf[:4 * K].view(torch.float32), buf[io:io + 8 * K].view(torch.int64)


def check_topk_indices(plan, counts, indices, names) -> None:
    """Wrap negative indices and raise the reference's IndexError for one out of range
    (omf_topk_check_indices); synchronises the stream."""
    bad = int(plan.topk_check_indices(counts, indices).item())
    if bad < plan.nt:
        raise IndexError(f"Compressed layer {names[bad]!r}: index out of bounds for size {plan.sizes[bad]}")


def _decode_topk_batch(topk, dev: torch.device):
    """Decode a message's Top-K layers (zero-filled, no base) in one call: returns the decoded
    fp32 arena and the plan (layer t at ``[plan.offsets[t], + plan.sizes[t])``).  A layer that
    repeats an index is decoded again by itself with numpy's last-value rule (never for a
    selection an encoder produced)."""
    plan = codec.Plan.get([_layer_numel(L) for L, *_ in topk], device=dev)
    counts, values, indices = stage_topk([(v, i) for _L, v, i, _k in topk], dev, "topk_decode")
    bad = plan.topk_check_indices(counts, indices)
    dup = plan.topk_check_duplicates(counts, indices)
    y = plan.topk_decode_counts(counts, values, indices, mode=0)  # out-of-range indices are skipped
    flags = torch.cat([bad, dup]).cpu()  # synchronises: the staging is free again
    b = int(flags[0])
    if b < plan.nt:
        raise IndexError(f"Compressed layer {topk[b][0].layer_name!r}: index out of bounds for size {plan.sizes[b]}")
    for t in flags[1:].nonzero().flatten().tolist():
        o, n = plan.offsets[t], plan.sizes[t]
        y[o:o + n] = _decode_topk_layer(topk[t][0], device=dev, last_wins=True).reshape(-1)
    return y, plan


def decode_updates_dict(proto_layers, *, base_updates: Optional[Dict[str, torch.Tensor]] = None,
                        device=None) -> Dict[str, torch.Tensor]:
    """global_grpc_compression.py:214-223; every QSGD layer of a (width, level) in one launch.

    Placement as the reference: CPU tensors unless ``device`` is given (QSGD ignores
    ``base_tensor``, :198-202); with ``device="cuda"`` nothing but the payload crosses PCIe.
    """
    _host_memory_policy()
    proto_layers = list(proto_layers)
    out_dev = _out_device(None, device)
    decoded: Dict[str, torch.Tensor] = {}
    topk_done = set()
    groups, topk = _scan_layers(proto_layers)
    if groups:
        dev = _gpu_for(out_dev)
        for layers in groups.values():
            y, plan = _decode_qsgd_batch(layers, dev, host=out_dev.type == "cpu")
            if out_dev.type == "cpu" and y.is_cuda:  # the packed wire: one chunked D2H
                y = hostio.device_to_host(y, pool_memory=_HOST_POLICY)
            for L, o, n in zip(layers, plan.offsets, plan.sizes):
                decoded[L.layer_name] = y[o:o + n].view(tuple(L.original_shape))
    if base_updates is not None:  # overlays decode layer by layer, on their bases' devices
        topk = [e for e in topk if e[0].layer_name not in base_updates]
    if topk and _topk_batch_ok(topk):
        y, plan = _decode_topk_batch(topk, _gpu_for(out_dev))
        if out_dev.type == "cpu":
            y = hostio.device_to_host(y, pool_memory=_HOST_POLICY)
        for (L, *_), o, n in zip(topk, plan.offsets, plan.sizes):
            decoded[L.layer_name] = y[o:o + n].view(tuple(L.original_shape))
            topk_done.add(id(L))
    out: Dict[str, torch.Tensor] = {}
    for layer in proto_layers:
        ct = layer.compression_type
        if layer.layer_name in decoded and (ct in _QSGD_TYPES or (ct == TOPK_COMPRESSION_NAME and id(layer) in topk_done)):
            out[layer.layer_name] = decoded[layer.layer_name]
            continue
        base = None if base_updates is None else base_updates.get(layer.layer_name)
        out[layer.layer_name] = decode_layer_tensor(layer, base_tensor=base, device=device)
    return out


def decode_updates_into(proto_layers, targets: Dict[str, torch.Tensor]) -> None:
    """Client downlink (global_grpc_client.py:98-111): decode each layer into ``targets[name]``.

    Equivalent to ``target.copy_(decode_layer_tensor(layer, base_tensor=target).to(...))``
    for every layer whose name is in ``targets``: QSGD layers are decoded in one launch per
    (width, level) and copied device-to-device; Top-K layers are scattered onto the target
    in place (the reference's overlay-on-a-copy); dense layers are copied.
    """
    proto_layers = [L for L in proto_layers if L.layer_name in targets]
    groups, topk = _scan_layers(proto_layers)
    done = set()
    if topk and _topk_batch_ok(topk):
        done = _overlay_topk_into(topk, targets)
    for layers in groups.values():
        dev = _gpu_for(targets[layers[0].layer_name].device)
        y, plan = _decode_qsgd_batch(layers, dev)
        for L, o, n in zip(layers, plan.offsets, plan.sizes):
            t = targets[L.layer_name]
            t.copy_(y[o:o + n].view(tuple(L.original_shape)).to(t.dtype))
    for L in proto_layers:
        if L.compression_type in _QSGD_TYPES or id(L) in done:
            continue
        t = targets[L.layer_name]
        dec = decode_layer_tensor(L, base_tensor=t, device=t.device)
        t.copy_(dec.to(t.dtype))


def _overlay_topk_into(topk, targets) -> set:
    """The Top-K part of decode_updates_into: the values set at their indices in each target
    (the reference's overlay on ``param.data``, global_grpc_client.py:98-111), in place.  Layers
    whose target is a contiguous fp32 GPU tensor of the layer's size are staged together (one
    chunked H2D), checked (one index check; an out-of-range index raises before any target is
    written) and scattered — as one launch when the targets are views of one arena, else one
    launch per target.  Returns the ids of the layers handled; the caller decodes the rest."""
    first = targets[topk[0][0].layer_name]
    if not first.is_cuda:
        return set()
    dev = first.device
    mine = [e for e in topk if (lambda t: t.is_cuda and t.device == dev and t.dtype == torch.float32
                                and t.is_contiguous() and t.numel() == _layer_numel(e[0]))(targets[e[0].layer_name])]
    if not mine:
        return set()
    names = [L.layer_name for L, *_ in mine]
    plan = codec.Plan.get([_layer_numel(L) for L, *_ in mine], device=dev)
    counts, values, indices = stage_topk([(v, i) for _L, v, i, _k in mine], dev, "topk_overlay")
    check_topk_indices(plan, counts, indices, names)
    dup = plan.topk_check_duplicates(counts, indices)
    flats = [targets[n].detach().reshape(-1) for n in names]
    from ..compression.core import shared_arena

    arena = shared_arena(flats, dev, plan)
    if arena is not None:
        plan.topk_decode_counts(counts, values, indices, y=arena, mode=1)
    else:
        K = 0
        for f, k in zip(flats, counts):
            codec.topk_decode(values[K:K + k], indices[K:K + k], f.numel(), y=f, mode=1)
            K += k
    rep = dup.nonzero().flatten().tolist()  # (synchronises) layers that repeat an index: the last value wins
    koff = [0]
    for k in counts:
        koff.append(koff[-1] + int(k))
    for t in rep:
        v, ix = _last_wins(values[koff[t]:koff[t + 1]], indices[koff[t]:koff[t + 1]], plan.sizes[t])
        codec.topk_decode(v.contiguous(), ix.contiguous(), flats[t].numel(), y=flats[t], mode=1)
    return {id(L) for L, *_ in mine}


__all__: List[str] = [
    "GlobalHybridCompressor",
    "build_global_compressor",
    "compression_mode_name",
    "decode_layer_tensor",
    "decode_updates_dict",
    "decode_updates_into",
    "encode_layer_state",
    "encode_updates_dict",
    "hybrid_global_compressor_from_cfg",
    "qsgd_layer_from_payload",
    "qsgd_layers_from_arena",
    "qsgd_packed_layer_from_payload",
    "topk_layer_from_bytes",
    "topk_layer_from_payload",
    "wire_size",
]
