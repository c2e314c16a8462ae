"""Parameter-server aggregate-after-decode, on one GPU and across the GPUs of a node.

One GPU — ``DeviceAggregator`` mirrors ``CentralServerServicer``'s
``_initialize_accumulated_updates`` / ``_accumulate_model_updates`` /
``_apply_model_updates`` (src/omnifed/hybrid/communicator/global_grpc_server.py:58-171):
every client's ``LayerState`` list is decoded straight into one fp32 accumulator
arena (``omf_qsgd_decode`` with accumulate=1: acc += norm·q/L in one launch for all
QSGD tensors; Top-K layers scatter-add; dense layers add), then divided by the
total sample count.  Clients are summed in call (= arrival) order, as the reference.

Several GPUs of one node (one synthetic client per rank) — the
weighted sum Σ_i decode(Q(w_i·x_i)) / Σ_i w_i is the path's only exchange step:
* ``weighted_sum_reduce``: each rank decodes its own payload, then one RCCL
  ``reduce(SUM)`` of the fp32 arena to the root, which divides by Σw;
* ``weighted_sum_gather``: RCCL ``gather`` of the int8/int32 payloads + norms to
  the root (w/4 of the fp32 bytes over xGMI), which decode-accumulates them in
  rank order (deterministic) and divides.
Both take an ``ops`` object so the orchestration is testable with gloo on CPU.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import codec
from .shapes import numel


class GpuOps:
    """The device operations the PS steps use (HIP C ABI)."""

    def __init__(self, plan: "codec.Plan"):
        self.plan = plan

    def decode(self, q, width, levels, norms, y, accumulate):
        return self.plan.qsgd_decode(q, width, levels, norms, y_out=y, accumulate=accumulate)

    def div_(self, y, d):
        return codec.div_(y, d)


class DeviceAggregator:
    """PS accumulator arena for one model (one GPU)."""

    def __init__(self, named_shapes: Sequence[Tuple[str, tuple]], device=None, compute_mean: bool = True):
        self.names = [n for n, _ in named_shapes]
        self.shapes = {n: tuple(s) for n, s in named_shapes}
        sizes = [max(numel(s), 1) for _, s in named_shapes]
        self.plan = codec.Plan.get(sizes, device=device)
        self.device = self.plan.device
        self.index = {n: i for i, n in enumerate(self.names)}
        self.compute_mean = compute_mean
        self.acc = torch.zeros(self.plan.arena_end, dtype=torch.float32, device=self.device)
        self.update_count = 0
        self.total_samples = 0
        self._q8 = None
        self._q32 = None

    def reset(self):
        """_initialize_accumulated_updates (global_grpc_server.py:58-62)."""
        self.acc.zero_()
        self.update_count = 0
        self.total_samples = 0

    def _slice(self, name):
        i = self.index[name]
        o, n = self.plan.offsets[i], self.plan.sizes[i]
        return self.acc[o:o + n]

    def accumulate_layers(self, layers, number_samples: int = 0):
        """Decode one client's update into the accumulator (global_grpc_server.py:108-111, 147-153)."""
        qsgd = [L for L in layers if L.compression_type == "QSGDQuantCompression" and L.layer_name in self.index]
        if qsgd:
            width, level = qsgd[0].width, qsgd[0].level
            if any(L.width != width or L.level != level for L in qsgd):
                raise ValueError("mixed QSGD width/level within one update")
            if width not in (8, 32) or level <= 0:
                raise ValueError(f"unsupported QSGD width={width} / level={level}")
            np_dt = np.int8 if width == 8 else np.int32
            host = np.zeros(self.plan.arena_end, dtype=np_dt)
            norms = np.zeros(self.plan.nt, dtype=np.float32)  # absent tensors: norm 0 adds +0
            for L in qsgd:
                i = self.index[L.layer_name]
                o, n = self.plan.offsets[i], self.plan.sizes[i]
                q = np.frombuffer(L.values_data, dtype=np_dt)
                if q.size != n:
                    raise ValueError(f"QSGD layer {L.layer_name!r}: {q.size} values, expected {n}")
                host[o:o + n] = q
                norms[i] = np.frombuffer(L.meta_tensor, dtype=np.float32).reshape(-1)[0]
            qd = torch.from_numpy(host).to(self.device)
            nd = torch.from_numpy(norms).to(self.device)
            # Tensors absent from this update keep acc += (0 * q)/L = +0 (q is zero there).
            self.plan.qsgd_decode(qd, width, level, nd, y_out=self.acc, accumulate=True)
        for L in layers:
            if L.layer_name not in self.index or L.compression_type == "QSGDQuantCompression":
                continue
            dst = self._slice(L.layer_name)
            if L.compression_type == "TopKCompression":
                v = torch.from_numpy(np.frombuffer(L.values_data, dtype=np.float32).copy()).to(self.device)
                ix = torch.from_numpy(np.frombuffer(L.indices_data, dtype=np.int64).copy()).to(self.device)
                codec.topk_decode(v, ix, dst.numel(), y=dst, mode=2)
            elif L.compression_type == "":
                arr = torch.tensor(list(L.param_update), dtype=torch.float32).to(self.device)
                dst.add_(arr.reshape(-1))
            else:
                raise ValueError(f"Unsupported compression_type={L.compression_type!r}")
        self.update_count += 1
        self.total_samples += int(number_samples)

    def apply_and_encode(self, compressor, total_samples: Optional[int] = None):
        """Fused ``_apply_model_updates`` + the first downlink ``_send_current_model``
        (global_grpc_server.py:155-171, 213-234): one launch divides the accumulator by the
        sample count (in place: it becomes the averaged model, as ``param.data = avg``) and
        QSGD-encodes the average.  Returns ``(avg views by name, LayerState list)``; later
        requests re-encode the average independently, as the reference does per request.
        """
        from .hybrid.compression.qsgd import QSGDQuantCompression, choose_qsgd_storage_width
        from .hybrid.communicator.global_grpc_compression import qsgd_layer_from_payload, _encode_dense_layer

        if (not isinstance(compressor, QSGDQuantCompression) or not self.compute_mean
                or compressor.rng != "philox"):  # parity mode draws MT19937 uniforms on the host
            avg = self.apply(total_samples)
            from .hybrid.communicator.global_grpc_compression import encode_updates_dict
            return avg, encode_updates_dict(avg, compressor)
        total = self.total_samples if total_samples is None else int(total_samples)
        s = compressor.s
        seed = int(torch.randint(0, 2**62, (1,)).item())
        _, q, norms = self.plan.ps_apply_encode(self.acc, float(total), s, avg_out=self.acc, seed=seed,
                                                offset=compressor._next_call())
        levels = 2**s
        width, _ = choose_qsgd_storage_width(levels)
        qh = q.cpu().numpy()
        nh = norms.cpu().tolist()
        avg = {n: self._slice(n).view(self.shapes[n]) for n in self.names}
        layers = []
        for i, n in enumerate(self.names):
            o, k = self.plan.offsets[i], self.plan.sizes[i]
            if nh[i] != 0 and int(np.prod(self.shapes[n])) > 0:
                layers.append(qsgd_layer_from_payload(n, self.shapes[n], qh[o:o + k].tobytes(), nh[i], width, levels))
            else:
                layers.append(_encode_dense_layer(n, avg[n]))
        return avg, layers

    def apply(self, total_samples: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """_apply_model_updates (global_grpc_server.py:155-171): acc / total_samples per tensor."""
        total = self.total_samples if total_samples is None else int(total_samples)
        if self.compute_mean:
            codec.div_(self.acc, float(total))
        return {n: self._slice(n).view(self.shapes[n]) for n in self.names}


def weighted_sum_reduce(y: torch.Tensor, total_weight: float, ops, group=None, dst: int = 0) -> torch.Tensor:
    """RCCL reduce(SUM) of every rank's decoded fp32 arena to ``dst``, then ``/ total_weight`` there."""
    dist.reduce(y, dst=dst, op=dist.ReduceOp.SUM, group=group)
    if dist.get_rank(group) == dst:
        ops.div_(y, float(total_weight))
    return y


def weighted_sum_gather(q: torch.Tensor, norms: torch.Tensor, width: int, levels: int, acc: torch.Tensor,
                        total_weight: float, ops, group=None, dst: int = 0,
                        bufs: Optional[List[Tuple[torch.Tensor, torch.Tensor]]] = None) -> torch.Tensor:
    """Gather every rank's payload (+ norms) to ``dst``; it decode-accumulates them in rank order and divides."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank == dst:
        if bufs is None:
            bufs = [(torch.empty_like(q), torch.empty_like(norms)) for _ in range(world)]
        dist.gather(q, gather_list=[b[0] for b in bufs], dst=dst, group=group)
        dist.gather(norms, gather_list=[b[1] for b in bufs], dst=dst, group=group)
        acc.zero_()
        for qb, nb in bufs:
            ops.decode(qb, width, levels, nb, acc, True)
        ops.div_(acc, float(total_weight))
    else:
        dist.gather(q, dst=dst, group=group)
        dist.gather(norms, dst=dst, group=group)
    return acc
