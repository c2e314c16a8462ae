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
* ``qsgd_weighted_round``: each rank encodes its client with the weighting fused
  (alpha = w_i, global_grpc.py:101-123), then one of
* ``weighted_sum_reduce``: each rank decodes its own payload, then one RCCL
  ``reduce(SUM)`` of the fp32 arena to the root, which divides by Σw;
* ``weighted_sum_gather``: RCCL ``gather`` of the int8/int32 payloads + norms to
  the root (w/4 of the fp32 bytes over xGMI), which decode-accumulates them in
  rank order (deterministic) and divides.
Top-K across GPUs (``topk_sparse_aggregate``): the reference's sparse aggregate
(torch_mpi.py:302-359 → core.layerwise_decompress, core.py:62-71): every rank's
(values, indices) all-gathered (or gathered to one root), scatter-added in rank order
and divided by the client count.  Every rank selects k = max(1, int(n·ratio)) per
tensor of the same plan, so no padding is needed (the reference pads to the largest
k with index 0 / value 0, which is a no-op whenever the k agree).
All of them take an ``ops`` object so the orchestration is testable with gloo on CPU.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import codec, hostio
from .shapes import numel


def rank_key(seed: int, rank: int) -> int:
    """64-bit Philox key of one client: splitmix64 of (seed, rank).  Clients that share a seed
    (every process calling the reference's ``set_seed(1234)``) still draw independent streams,
    so averaging N clients keeps QSGD's 1/N variance reduction."""
    z = (int(seed) * 0x9E3779B97F4A7C15 + (int(rank) + 1) * 0xD1B54A32D192ED03) & (2**64 - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
    return z ^ (z >> 31)


def _rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


class GpuOps:
    """The device operations the PS steps use (HIP C ABI).

    ``seed``: the Philox key is ``rank_key(seed, rank)`` (``rank`` defaults to this process's
    rank in the default group), so ranks that pass one seed still draw independently."""

    def __init__(self, plan: "codec.Plan", seed: int = 0, rank: Optional[int] = None):
        self.plan = plan
        self.seed = int(seed)
        self.rank = _rank() if rank is None else int(rank)
        self.key = rank_key(self.seed, self.rank)

    def encode(self, x, bit_width, alpha, call, q=None, norms=None):
        """Q(fl32(alpha·x)) of the whole arena (Philox keyed by ``key``, stream ``call``)."""
        return self.plan.qsgd_encode(x, bit_width, q_out=q, norm_out=norms, alpha=alpha, seed=self.key, offset=call)

    def encode_status(self) -> int:
        """1 if the plan's launches since the last check hit an in-kernel timeout (the payload is
        invalid), else 0; synchronises the current stream."""
        try:
            self.plan.check()
        except codec.CodecError:
            return 1
        return 0

    def decode(self, q, width, levels, norms, y, accumulate):
        return self.plan.qsgd_decode(q, width, levels, norms, y_out=y, accumulate=accumulate)

    def div_(self, y, d):
        return codec.div_(y, d)

    def topk_encode(self, x, ratio, residual, residual_mode, alpha, values=None, indices=None, tie_order="torch"):
        """The client's Top-K encode (the reference's selection where magnitudes tie: tie_order)."""
        values, indices, _ = self.plan.topk_encode(x, ratio, residual=residual, residual_mode=residual_mode,
                                                   values=values, indices=indices, alpha=alpha, tie_order=tie_order)
        return values, indices

    def topk_decode(self, values, indices, ratio, y, mode):
        return self.plan.topk_decode_arena(values, indices, ratio, y=y, mode=mode)


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
        self.avg: Optional[torch.Tensor] = None  # the fused step's output arena (disjoint from acc)
        self.update_count = 0
        self.total_samples = 0
        # set by accumulate_apply_encode(keep_sum=False): acc lacks the last client's term, so
        # every call that reads or extends the sum raises until reset()
        self._stale = False

    def reset(self):
        """_initialize_accumulated_updates (global_grpc_server.py:58-62)."""
        self.acc.zero_()
        self.update_count = 0
        self.total_samples = 0
        self._stale = False

    def _check_fresh(self):
        if self._stale:
            raise RuntimeError("the accumulator lacks the last client's term (accumulate_apply_encode with "
                               "keep_sum=False): reset() it before the next round")

    def _slice(self, name):
        i = self.index[name]
        o, n = self.plan.offsets[i], self.plan.sizes[i]
        return self.acc[o:o + n]

    def _avg_slice(self, name):
        i = self.index[name]
        o, n = self.plan.offsets[i], self.plan.sizes[i]
        return self.avg[o:o + n]

    def accumulate_layers(self, layers, number_samples: int = 0):
        """Decode one client's update into the accumulator (global_grpc_server.py:108-111, 147-153).

        Every layer is checked and staged before the accumulator is touched (the reference decodes
        the whole update, then accumulates: a bad layer leaves acc as it was).  All QSGD layers go
        through ONE decode-accumulate launch, all Top-K layers through ONE index check and ONE
        scatter-add (omf_topk_decode_counts), both fed by chunked pinned staging.  A repeated name:
        the last layer, as the reference's decoded dict.  The scatter-add assumes the indices of a
        Top-K layer are distinct, as every encoder's selection (torch.topk's, the reference's) is; a
        layer with more values than elements (which must repeat indices) is decoded alone with
        numpy's last-wins rule and added."""
        from .hybrid.communicator.global_grpc_compression import (_decode_topk_layer, _validate_layer,
                                                                  check_topk_indices, stage_topk)

        self._check_fresh()
        last: Dict[str, object] = {}
        topk_payload: Dict[str, tuple] = {}
        for L in layers:
            got = _validate_layer(L)  # the reference decoder's checks, in message order
            if L.layer_name not in self.index:
                continue
            last[L.layer_name] = L
            if got is not None:
                topk_payload[L.layer_name] = got
        kept = sorted(last.values(), key=lambda L: self.index[L.layer_name])  # ascending arena offsets
        qsgd = [L for L in kept if L.compression_type == "QSGDQuantCompression"]
        topk = [L for L in kept if L.compression_type == "TopKCompression"]
        dense = [L for L in kept if L.compression_type == ""]
        if any(L.compression_type not in ("QSGDQuantCompression", "TopKCompression", "") for L in kept):
            bad = next(L for L in kept if L.compression_type not in ("QSGDQuantCompression", "TopKCompression", ""))
            raise ValueError(f"Unsupported compression_type={bad.compression_type!r}")
        # --- stage and check everything
        q_args = None
        if qsgd:
            width, level = qsgd[0].width, qsgd[0].level
            if any(L.width != width or L.level != level for L in qsgd):
                raise ValueError("mixed QSGD width/level within one update")
            isz = width // 8
            norms = np.zeros(self.plan.nt, dtype=np.float32)  # absent tensors: norm 0 adds +0
            items = []
            for L in qsgd:
                i = self.index[L.layer_name]
                norms[i] = np.frombuffer(L.meta_tensor, dtype=np.float32).reshape(-1)[0]
                items.append((self.plan.offsets[i] * isz, (lambda L=L: L.values_data)))

            def check(k, payload):
                n = self.plan.sizes[self.index[qsgd[k].layer_name]]
                if len(payload) != n * isz:
                    raise ValueError(f"QSGD layer {qsgd[k].layer_name!r}: {len(payload) // isz} values, expected {n}")

            qd = torch.empty(self.plan.payload_elems(width), dtype=torch.int8 if width == 8 else torch.int32,
                             device=self.device)
            nd = torch.from_numpy(norms).to(self.device)
            hostio.bytes_to_device(items, qd, isz * self.plan.payload_elems(width), key="ps_decode", check=check)
            q_args = (qd, width, level, nd)
        t_args = None
        # a Top-K layer with more values than its tensor's elements repeats indices: decoded alone
        # with numpy's last-wins rule (_decode_topk_layer), as decode_updates_dict does
        odd = [L for L in topk if topk_payload[L.layer_name][2] > self.plan.sizes[self.index[L.layer_name]]]
        odd_args = [(L.layer_name, _decode_topk_layer(L, device=self.device).reshape(-1)) for L in odd]
        topk = [L for L in topk if L not in odd]
        if topk:
            pairs = [(b"", b"")] * self.plan.nt
            for L in topk:
                i = self.index[L.layer_name]
                v, ix, k = topk_payload[L.layer_name]
                pairs[i] = (v, ix)
            counts, values, indices = stage_topk(pairs, self.device, "ps_topk")
            check_topk_indices(self.plan, counts, indices, self.names)  # synchronises
            dup = self.plan.topk_check_duplicates(counts, indices).cpu()
            rep = [L for L in topk if dup[self.index[L.layer_name]]]
            if rep:  # a layer repeating an index (never an encoder's): alone, numpy's last value per index
                odd_args += [(L.layer_name, _decode_topk_layer(L, device=self.device, last_wins=True).reshape(-1))
                             for L in rep]
                for L in rep:
                    pairs[self.index[L.layer_name]] = (b"", b"")
                counts, values, indices = stage_topk(pairs, self.device, "ps_topk")
                check_topk_indices(self.plan, counts, indices, self.names)
            t_args = (counts, values, indices)
        dense_args = []
        for L in dense:
            arr = torch.tensor(list(L.param_update), dtype=torch.float32)
            n = self.plan.sizes[self.index[L.layer_name]]
            if arr.numel() != n:
                raise ValueError(f"Dense layer {L.layer_name!r}: {arr.numel()} values, expected {n}")
            dense_args.append((L.layer_name, arr.to(self.device, non_blocking=False)))
        # --- accumulate (client terms in the reference's per-name order: one term per name)
        if q_args is not None:
            # Tensors absent from this update keep acc += (0 * q)/L = +0 (whatever q holds there:
            # any int8 / int32 level times a zero norm is a zero).
            qd, width, level, nd = q_args
            self.plan.qsgd_decode(qd, width, level, nd, y_out=self.acc, accumulate=True)
        if t_args is not None:
            self.plan.topk_decode_counts(*t_args, y=self.acc, mode=2)
        for name, arr in dense_args + odd_args:
            self._slice(name).add_(arr.reshape(-1))
        self.update_count += 1
        self.total_samples += int(number_samples)

    def accumulate_updates(self, updates: Dict[str, torch.Tensor], compressor, number_samples: int = 0,
                           weight=None):
        """One in-process client's whole round trip into the accumulator, without the wire:
        ``encode_updates_dict(updates, compressor, weight=weight)`` then ``accumulate_layers`` —
        for a QSGD compressor as ONE weighted encode launch (alpha = weight) and ONE
        decode-accumulate launch on the device (no host copy).  Bit-identical to the wire path
        for the same draws (same kernels, same payload and norms)."""
        from .hybrid.compression.qsgd import QSGDQuantCompression, encode_groups, should_compress_tensor

        self._check_fresh()
        names = [n for n in self.names if n in updates]
        if (not isinstance(compressor, QSGDQuantCompression) or compressor.packed_wire
                or not all(should_compress_tensor(updates[n]) and updates[n].dtype == torch.float32 for n in names)
                or [n for n in updates if n not in self.index]):
            from .hybrid.communicator.global_grpc_compression import encode_updates_dict
            return self.accumulate_layers(encode_updates_dict(updates, compressor, weight=weight), number_samples)
        x = torch.zeros(self.plan.arena_end, dtype=torch.float32, device=self.device)
        for n in names:
            i = self.index[n]
            x[self.plan.offsets[i]:self.plan.offsets[i] + self.plan.sizes[i]].copy_(updates[n].detach().reshape(-1))
        alpha = 1.0 if weight is None else float(weight)
        if compressor.rng == "philox":
            q, norms = self.plan.qsgd_encode(x, compressor.s, alpha=alpha, seed=compressor.philox_key(),
                                             offset=compressor._next_call())
        else:  # the reference's MT19937 stream over the named tensors present, in order
            flats = [updates[n].detach().reshape(-1) for n in names]
            (plan, qg, ng, _), = encode_groups(flats, compressor.s, self.device, "mt19937", compressor._next_call(),
                                              alpha=alpha)
            q = torch.zeros(self.plan.payload_elems(8 if 2**compressor.s <= 127 else 32), dtype=qg.dtype,
                            device=self.device)
            norms = torch.zeros(self.plan.nt, dtype=torch.float32, device=self.device)
            for k, n in enumerate(names):
                i = self.index[n]
                o, m = self.plan.offsets[i], self.plan.sizes[i]
                q[o:o + m].copy_(qg[plan.offsets[k]:plan.offsets[k] + m])
                norms[i] = ng[k]
        levels = 2**compressor.s
        # An in-kernel encoder timeout raises here, before anything touches the accumulator (the
        # reference decodes a whole update before it accumulates, global_grpc_server.py:108-111,
        # so a failed SendUpdate leaves acc as it was and answers success=False).
        self.plan.check()
        # absent tensors have q = 0 (x was zero there): acc += +0, as accumulate_layers
        self.plan.qsgd_decode(q, 8 if levels <= 127 else 32, levels, norms, y_out=self.acc, accumulate=True)
        self.update_count += 1
        self.total_samples += int(number_samples)

    def apply_and_encode(self, compressor, total_samples: Optional[int] = None):
        """Fused ``_apply_model_updates`` + the first downlink ``_send_current_model``
        (global_grpc_server.py:155-171, 213-234): the average ``acc / total_samples`` is written
        to ``self.avg`` (the accumulator keeps the sum) and QSGD-encoded — for a Philox QSGD
        compressor in one launch that reads the accumulator once (omf_ps_apply_encode).
        Returns ``(avg views by name, LayerState list)``; later requests re-encode the average
        independently, as the reference does per request.  An in-kernel encoder timeout raises
        ``RuntimeError``.
        """
        from .hybrid.compression.qsgd import QSGDQuantCompression
        from .hybrid.communicator.global_grpc_compression import _encode_dense_layer, qsgd_layers_from_arena

        self._check_fresh()
        total = self.total_samples if total_samples is None else int(total_samples)
        if self.avg is None:
            self.avg = torch.empty_like(self.acc)
        if (not isinstance(compressor, QSGDQuantCompression) or not self.compute_mean
                or compressor.rng != "philox"):  # parity mode draws MT19937 uniforms on the host
            self.avg.copy_(self.acc)
            if self.compute_mean:
                codec.div_(self.avg, float(total))
            avg = {n: self._avg_slice(n).view(self.shapes[n]) for n in self.names}
            from .hybrid.communicator.global_grpc_compression import encode_updates_dict
            return avg, encode_updates_dict(avg, compressor)
        s = compressor.s
        # avg_out disjoint from acc: the one-launch path (omf_ps_apply_encode)
        _, q, norms = self.plan.ps_apply_encode(self.acc, float(total), s, avg_out=self.avg,
                                                seed=compressor.philox_key(), offset=compressor._next_call())
        avg = {n: self._avg_slice(n).view(self.shapes[n]) for n in self.names}
        # the payload arena through the wire pipeline (chunked pinned D2H, worker-filled bytes);
        # raises on an in-kernel encoder timeout
        got = qsgd_layers_from_arena(self.plan, q, norms, self.names, [self.shapes[n] for n in self.names], 2**s,
                                     compressor.packed_wire)
        layers = []
        for n, L in zip(self.names, got):
            layers.append(L if L is not None and int(np.prod(self.shapes[n])) > 0 else _encode_dense_layer(n, avg[n]))
        return avg, layers

    def accumulate_apply_encode(self, layers, number_samples: int, compressor, keep_sum: bool = True):
        """The last arriving client's ``SendUpdate`` and the round's first ``GetUpdatedModel`` in one
        pass (global_grpc_server.py:108-125, 147-171, 213-234): ``acc + decode(update)``, the
        average over ``total_samples`` (this client's included) and its QSGD downlink — for a QSGD
        update and a Philox QSGD compressor on a bracketed plan, ONE encoder pass that reads the
        accumulator and the update's payload once (omf_ps_accumulate_apply_encode; 10 B per element
        at s = 4 instead of 18 for accumulate_layers + apply_and_encode).  ``keep_sum`` (default)
        stores the sum in the accumulator, as the two calls leave it (4 more bytes per element);
        ``keep_sum=False`` skips that store — the reference reads the sum only in
        _apply_model_updates and re-initialises it at the next round's first update (:86-92) — and
        marks the accumulator stale: every later call that reads or extends it raises until
        ``reset()``.  The counters advance once the sum (stored or not) has been formed; a payload
        that fails its checks leaves accumulator and counters as they were.  Same return as
        ``apply_and_encode``; bytes equal to ``accumulate_layers`` followed by it.  Any other
        message or compressor takes those two calls."""
        from .hybrid.compression.qsgd import QSGDQuantCompression
        from .hybrid.communicator.global_grpc_compression import (_encode_dense_layer, _validate_layer,
                                                                  qsgd_layers_from_arena)

        self._check_fresh()
        layers = list(layers)
        last: Dict[str, object] = {}
        for L in layers:
            _validate_layer(L)
            if L.layer_name in self.index:
                last[L.layer_name] = L
        kept = sorted(last.values(), key=lambda L: self.index[L.layer_name])
        fusable = (isinstance(compressor, QSGDQuantCompression) and compressor.rng == "philox" and self.compute_mean
                   and not compressor.packed_wire and kept
                   and all(L.compression_type == "QSGDQuantCompression" for L in kept)
                   and len({(L.width, L.level) for L in kept}) == 1)
        if not fusable:
            self.accumulate_layers(layers, number_samples)
            return self.apply_and_encode(compressor)
        width, level = kept[0].width, kept[0].level
        isz = width // 8
        norms = np.zeros(self.plan.nt, dtype=np.float32)  # absent tensors: norm 0 adds +0
        items = []
        for L in kept:
            i = self.index[L.layer_name]
            norms[i] = np.frombuffer(L.meta_tensor, dtype=np.float32).reshape(-1)[0]
            items.append((self.plan.offsets[i] * isz, (lambda L=L: L.values_data)))

        def check(k, payload):
            n = self.plan.sizes[self.index[kept[k].layer_name]]
            if len(payload) != n * isz:
                raise ValueError(f"QSGD layer {kept[k].layer_name!r}: {len(payload) // isz} values, expected {n}")

        qd = torch.empty(self.plan.payload_elems(width), dtype=torch.int8 if width == 8 else torch.int32,
                         device=self.device)  # absent tensors: any level times their zero norm adds +0
        nd = torch.from_numpy(norms).to(self.device)
        hostio.bytes_to_device(items, qd, isz * self.plan.payload_elems(width), key="ps_decode", check=check)
        total = self.total_samples + int(number_samples)
        if self.avg is None:
            self.avg = torch.empty_like(self.acc)
        s = compressor.s
        _, q, norms_out = self.plan.ps_accumulate_apply_encode(
            self.acc, qd, width, level, nd, float(total), s, acc_out=self.acc if keep_sum else None, avg_out=self.avg,
            seed=compressor.philox_key(), offset=compressor._next_call())
        self.update_count += 1
        self.total_samples = total
        if not keep_sum:
            self._stale = True
        avg = {n: self._avg_slice(n).view(self.shapes[n]) for n in self.names}
        got = qsgd_layers_from_arena(self.plan, q, norms_out, self.names, [self.shapes[n] for n in self.names], 2**s,
                                     compressor.packed_wire)
        out = []
        for n, L in zip(self.names, got):
            out.append(L if L is not None and int(np.prod(self.shapes[n])) > 0 else _encode_dense_layer(n, avg[n]))
        return avg, out

    def apply(self, total_samples: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """_apply_model_updates (global_grpc_server.py:155-171): acc / total_samples per tensor."""
        self._check_fresh()
        total = self.total_samples if total_samples is None else int(total_samples)
        if self.compute_mean:
            codec.div_(self.acc, float(total))
        return {n: self._slice(n).view(self.shapes[n]) for n in self.names}


def weighted_sum_error_bound(abs_sum: torch.Tensor, exact: torch.Tensor, n_terms: int, total: float) -> torch.Tensor:
    """Element-wise bound on ``|reduce(SUM)/total − exact|`` for a sum of ``n_terms`` fp32 terms
    added in ANY order (an RCCL ring or tree reduce picks its own), then one fp32 division.

    ``abs_sum`` = Σ_i |x_i| and ``exact`` = (Σ_i x_i)/total, both in fp64.  Every order of
    N−1 fp32 additions errs by at most γ_{N−1}·Σ|x_i| (γ_m = m·u/(1 − m·u), u = 2⁻²⁴; Higham,
    *Accuracy and Stability of Numerical Algorithms*, §4.2), and the division adds u·|result|;
    N·2⁻¹⁴⁹ covers subnormal rounding.  The reference PS sums in nondeterministic gRPC arrival
    order (global_grpc_server.py:147-153), so this bound — not bit equality — is the parity bar
    of the ``reduce`` mode; the ``gather`` mode is bit-exact in rank order."""
    u = 2.0**-24
    m = max(int(n_terms) - 1, 0)
    gamma = m * u / (1.0 - m * u)
    w = abs(float(total))
    err_sum = gamma * abs_sum.double() / w
    return err_sum + u * (exact.double().abs() + err_sum) + n_terms * 2.0**-149 / min(w, 1.0)


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


def total_weight(weight: float, device, group=None) -> float:
    """Σ_i w_i over the ranks (the PS's total_samples, global_grpc_server.py:107)."""
    t = torch.tensor([float(weight)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item())


def _agree_encoded(ops, device, group=None) -> None:
    """Every rank learns whether any rank's encode hit an in-kernel timeout (an 8-byte RCCL
    all-reduce of the flags) before the payloads move, and all of them raise together: a
    failed client never ships an invalid payload into the sum, and no rank is left waiting in
    a collective the others abandoned."""
    status = getattr(ops, "encode_status", None)
    flag = torch.tensor([0 if status is None else int(status())], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if int(flag.item()):
        raise codec.CodecError("qsgd_weighted_round: a rank's QSGD encode hit an in-kernel timeout "
                               "(omf_plan_check OMF_ETIMEOUT); the round is abandoned on every rank")


def qsgd_weighted_round(x: torch.Tensor, weight: float, total: float, ops, bit_width: int, call: int,
                        mode: str = "gather", y: Optional[torch.Tensor] = None, acc: Optional[torch.Tensor] = None,
                        q: Optional[torch.Tensor] = None, norms: Optional[torch.Tensor] = None, group=None,
                        dst: int = 0, bufs=None) -> torch.Tensor:
    """One round of the 8-GPU PS weighted sum: this rank's client update ``x`` is encoded as
    Q(fl32(weight·x)) (the weighting fused into the encoder) and the root ends with
    Σ_i decode(Q(w_i x_i)) / total (``total`` = Σ_i w_i, e.g. from ``total_weight``).
    ``mode``: "gather" (payloads to the root, rank-order decode-accumulate: deterministic)
    or "reduce" (decode locally, RCCL reduce of fp32).  Returns the root's result arena."""
    levels = 2**int(bit_width)
    width = 8 if levels <= 127 else 32
    q, norms = ops.encode(x, bit_width, float(weight), call, q, norms)
    _agree_encoded(ops, x.device, group)
    if mode == "reduce":
        y = ops.decode(q, width, levels, norms, y, False)
        return weighted_sum_reduce(y, total, ops, group=group, dst=dst)
    if mode != "gather":
        raise ValueError("mode must be 'gather' or 'reduce'")
    if acc is None:
        acc = torch.empty(x.numel(), dtype=torch.float32, device=x.device)
    return weighted_sum_gather(q, norms, width, levels, acc, total, ops, group=group, dst=dst, bufs=bufs)


def topk_sparse_aggregate(values: torch.Tensor, indices: torch.Tensor, ratio: float, acc: torch.Tensor, ops,
                          client_count: Optional[int] = None, group=None, dst: Optional[int] = None,
                          bufs: Optional[List[Tuple[torch.Tensor, torch.Tensor]]] = None) -> torch.Tensor:
    """Multi-GPU Top-K aggregate (torch_mpi.py:302-359 + core.py:62-71) over whole arenas.

    ``values``/``indices``: this rank's packed selection (``Plan.topk_encode`` at ``ratio``;
    tensor-local indices).  ``dst=None``: all-gather, every rank ends with the aggregate
    (the reference's form); ``dst=r``: gather to rank r only (half the xGMI traffic).  The
    receiving ranks scatter-add the selections in rank order into ``acc`` (zeroed first) and
    divide by ``client_count`` (default: the world size, as sparse_aggregate)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    count = world if client_count is None else int(client_count)
    receive = dst is None or rank == dst
    if receive and bufs is None:
        bufs = [(torch.empty_like(values), torch.empty_like(indices)) for _ in range(world)]
    if dst is None:
        dist.all_gather([b[0] for b in bufs], values, group=group)
        dist.all_gather([b[1] for b in bufs], indices, group=group)
    elif rank == dst:
        dist.gather(values, gather_list=[b[0] for b in bufs], dst=dst, group=group)
        dist.gather(indices, gather_list=[b[1] for b in bufs], dst=dst, group=group)
    else:
        dist.gather(values, dst=dst, group=group)
        dist.gather(indices, dst=dst, group=group)
    if not receive:
        return acc
    acc.zero_()
    for v, ix in bufs:  # rank order: tensor.data[ix] += vals per client, as layerwise_decompress
        ops.topk_decode(v, ix, ratio, acc, 2)
    ops.div_(acc, float(count))
    return acc
