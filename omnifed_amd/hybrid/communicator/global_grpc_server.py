"""Parameter-server servicer on the GPU codec (mirror of ``src/omnifed/hybrid/communicator/global_grpc_server.py``).

Same class, constructor and RPC semantics as the reference's ``CentralServerServicer``
(:20-250): rounds advance on the first update of a higher round (:81-88), an update for another
round is refused (:90-100), every update is decoded and added into the accumulator under the
servicer lock, the last of ``num_clients`` divides by the total sample count and publishes the
round (:108-137), a ``GetUpdatedModel`` for a finished round re-encodes the current parameters
with the compressor — once per request, as the reference (:173-234) — and one for the round in
progress waits up to 10 s for it (:193-205).  Exceptions become ``success=False`` /
``is_ready=False`` answers (:139-145, :207-211).

The difference is where the work runs: the accumulator is a ``DeviceAggregator`` arena on the
GPU, each update's layers are checked, staged and decoded into it in one launch per
(width, level) (QSGD) and one scatter-add (Top-K) — the reference's ``decode_updates_dict`` then
``acc[name] += update`` (:147-153) — and the average is one division launch (:155-171).
``model``'s parameters receive the average (``param.data``, or ``param.grad`` in gradients mode)
on their own device and dtype, as the reference's ``param.data = avg_update``.
"""

from __future__ import annotations

import threading
from typing import Optional

import torch

from . import global_grpc_pb2 as pb
from . import global_grpc_pb2_grpc
from .global_grpc_compression import GlobalHybridCompressor, decode_updates_dict, encode_updates_dict


class CentralServerServicer(global_grpc_pb2_grpc.CentralServerServicer):
    def __init__(self, num_clients: int, model: torch.nn.Module, compressor: Optional[GlobalHybridCompressor] = None,
                 accumulate_updates: bool = True, communicate_params: bool = True, compute_mean: bool = True,
                 device=None):
        from ...ps import DeviceAggregator

        self.num_clients = num_clients
        self.model = model
        self.compressor = compressor
        self.accumulate_updates = accumulate_updates
        self.communicate_params = communicate_params
        self.compute_mean = compute_mean
        self.registered_clients = set()
        self.current_round = -1
        self.lock = threading.Lock()
        self.round_complete_event = threading.Event()
        self.round_in_progress = -1
        self.aggregator = None
        self.accumulated_updates = None
        if accumulate_updates:
            named = [(n, tuple(p.shape)) for n, p in model.named_parameters()]
            self.aggregator = DeviceAggregator(named, device=device, compute_mean=compute_mean)
            self.accumulated_updates = self.aggregator  # (the reference's attribute; non-None when accumulating)

    @property
    def update_count(self) -> int:
        return self.aggregator.update_count if self.aggregator is not None else 0

    @property
    def total_samples(self) -> int:
        return self.aggregator.total_samples if self.aggregator is not None else 0

    def _response(self, success: bool, message: str, received: Optional[int] = None):
        return pb.active_module().UpdateResponse(
            success=success, message=message, clients_registered=len(self.registered_clients),
            updates_received=self.update_count if received is None else received)

    def SendUpdate(self, request, context):
        """Receive one client's update (global_grpc_server.py:76-145)."""
        with self.lock:
            client_id, round_number = request.client_id, request.round_number
            try:
                if round_number > self.round_in_progress:
                    self.round_in_progress = round_number
                    self.round_complete_event.clear()
                    if self.aggregator is not None:
                        self.aggregator.reset()
                if round_number != self.round_in_progress:
                    return self._response(False, f"Round {round_number} is not the current round "
                                                 f"({self.round_in_progress})")
                if self.aggregator is None:
                    decode_updates_dict(request.layers)  # decoded (and checked) but not kept, as the reference
                else:
                    self.aggregator.accumulate_layers(request.layers, request.number_samples)
                    if self.update_count == self.num_clients:
                        self._apply_model_updates()
                        self.current_round = round_number
                        self.round_complete_event.set()
                return self._response(True, "Update received successfully")
            except Exception as e:  # noqa: BLE001 — the reference answers every failure this way
                return self._response(False, f"Error processing update from {client_id}: {e}", received=0)

    def _apply_model_updates(self):
        """acc / total_samples into the model (global_grpc_server.py:155-171)."""
        avg = self.aggregator.apply()
        with torch.no_grad():
            for name, param in self.model.named_parameters():
                if name not in avg:
                    continue
                val = avg[name].to(param.device, param.dtype, copy=True)  # the accumulator is reused
                if self.communicate_params:
                    param.data = val
                else:
                    param.grad = val

    def GetUpdatedModel(self, request, context):
        """The averaged model for a finished round (global_grpc_server.py:173-211)."""
        round_number = request.round_number
        try:
            with self.lock:
                if round_number <= self.current_round:
                    return self._send_current_model(round_number)
                if round_number != self.round_in_progress:
                    return pb.active_module().ModelParameters(round_number=round_number, layers=[], is_ready=False)
            if self.round_complete_event.wait(timeout=10):
                with self.lock:
                    if round_number <= self.current_round:
                        return self._send_current_model(round_number)
            return pb.active_module().ModelParameters(round_number=round_number, layers=[], is_ready=False)
        except Exception:  # noqa: BLE001
            return pb.active_module().ModelParameters(round_number=round_number, layers=[], is_ready=False)

    def _send_current_model(self, round_number):
        """Re-encode the current parameters for this request (global_grpc_server.py:213-234)."""
        if self.accumulated_updates is None:
            return pb.active_module().ModelParameters(round_number=round_number, layers=[], is_ready=False)
        updates = {name: (p.data if self.communicate_params else p.grad) for name, p in self.model.named_parameters()}
        layers = encode_updates_dict(updates, self.compressor)
        return pb.active_module().ModelParameters(round_number=round_number, layers=layers, is_ready=True)

    def RegisterClient(self, request, context):
        """global_grpc_server.py:236-250."""
        with self.lock:
            self.registered_clients.add(request.client_id)
            total = len(self.registered_clients)
            return pb.active_module().RegistrationResponse(
                success=True, message=f"Client {request.client_id} registered successfully", total_clients=total)
