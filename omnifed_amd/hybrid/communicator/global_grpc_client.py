"""Facility-leader client on the GPU codec (mirror of ``src/omnifed/hybrid/communicator/global_grpc_client.py``).

``GrpcClient`` keeps the reference's constructor, registration (:45-60), ``send_update_to_server``
(:68-98) and ``get_averaged_model`` (:113-145).  The update dict goes through
``encode_updates_dict`` (one encode launch per dict, the payload fetched through the chunked
pinned pipeline) instead of a per-layer loop, and the averaged model is decoded into the
parameters by ``decode_updates_into`` (:98-111's ``decode_layer_tensor(layer, base_tensor=...)``
then ``copy_``: QSGD layers in one launch per (width, level), Top-K overlaid in place, dense
copied).  ``weight`` (ours, optional) fuses the client weighting ``param * batch_samples`` of
``GrpcCommunicator.aggregate`` (global_grpc.py:101-123) into the encoder.  ``grpc`` is imported on
use; the reference's progress prints are log records here.
"""

from __future__ import annotations

import logging
from typing import Dict, Optional

import torch

from . import global_grpc_pb2 as pb
from .global_grpc_compression import GlobalHybridCompressor, compression_mode_name, decode_updates_into, \
    encode_updates_dict
from .global_grpc_limits import GRPC_OPTIONS
from .global_grpc_pb2_grpc import CentralServerStub

log = logging.getLogger(__name__)


class GrpcClient:
    def __init__(self, client_id: str, master_addr: str = "127.0.0.1", master_port: int = 50051,
                 compressor: Optional[GlobalHybridCompressor] = None):
        import grpc

        self.client_id = client_id
        self.compressor = compressor
        self.channel = grpc.insecure_channel(f"{master_addr}:{master_port}", options=GRPC_OPTIONS)
        self.stub = CentralServerStub(self.channel)
        self.round_number = 0
        self.last_wire: Dict[str, int] = {}
        log.info("Client %s initialized (%s), connecting to %s:%s", client_id, compression_mode_name(compressor),
                 master_addr, master_port)
        self._register_with_server()

    def _register_with_server(self):
        import grpc

        try:
            resp = self.stub.RegisterClient(pb.active_module().ClientInfo(client_id=self.client_id))
            if not resp.success:
                log.warning("Failed to register with server: %s", resp.message)
        except grpc.RpcError as e:
            log.warning("Failed to connect to server: %s", e)

    def send_update_to_server(self, updates: Dict[str, torch.Tensor], batch_samples: int, weight=None) -> bool:
        import grpc

        try:
            layers = encode_updates_dict(updates, self.compressor, weight=weight, stats=self.last_wire)
            request = pb.active_module().ModelUpdate(client_id=self.client_id, round_number=self.round_number,
                                                     layers=layers, number_samples=batch_samples)
            resp = self.stub.SendUpdate(request)
            if not resp.success:
                log.warning("Failed to send update: %s", resp.message)
            return bool(resp.success)
        except grpc.RpcError as e:
            log.warning("Failed to send update to server: %s", e)
            return False

    def get_averaged_model(self, msg: torch.nn.Module, communicate_params: bool, max_polls: Optional[int] = None):
        """Poll GetUpdatedModel until the round is ready (the reference polls without bound;
        ``max_polls``, ours, bounds it and raises TimeoutError), then decode into ``msg``."""
        import grpc

        polls = 0
        while max_polls is None or polls < max_polls:
            polls += 1
            try:
                resp = self.stub.GetUpdatedModel(pb.active_module().GetModelRequest(client_id=self.client_id,
                                                                                    round_number=self.round_number))
            except grpc.RpcError as e:
                log.warning("Failed to get averaged model (will retry): %s", e)
                continue
            if resp.is_ready:
                with torch.no_grad():
                    targets = {}
                    for name, p in msg.named_parameters():
                        t = p.data if communicate_params else p.grad
                        if t is not None:
                            targets[name] = t
                    decode_updates_into(resp.layers, targets)
                return msg
        raise TimeoutError(f"round {self.round_number}: the averaged model was not ready after {polls} polls")
