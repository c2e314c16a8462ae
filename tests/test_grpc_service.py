"""CPU: the CentralServer service glue over a real loopback gRPC channel (no GPU, no codec).

``global_grpc_pb2_grpc`` mirrors the reference's generated module (stub, servicer base,
``add_CentralServerServicer_to_server``) with grpcio's generic handlers; the method paths are
global_grpc.proto's, and the channel options the reference's 2 GiB - 1 limits
(global_grpc.py:44-49, global_grpc_client.py:31-37)."""

from concurrent import futures

import pytest

grpc = pytest.importorskip("grpc")

from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb  # noqa: E402
from omnifed_amd.hybrid.communicator.global_grpc_limits import GRPC_MAX_MESSAGE_BYTES, GRPC_OPTIONS  # noqa: E402
from omnifed_amd.hybrid.communicator.global_grpc_pb2_grpc import (  # noqa: E402
    CentralServerServicer,
    CentralServerStub,
    add_CentralServerServicer_to_server,
    method_path,
)


class Echo(CentralServerServicer):
    def __init__(self):
        self.seen = []

    def RegisterClient(self, request, context):
        self.seen.append(request.client_id)
        return pb.RegistrationResponse(success=True, message="ok", total_clients=len(self.seen))

    def SendUpdate(self, request, context):
        n = sum(len(L.values_data) for L in request.layers)
        return pb.UpdateResponse(success=True, message=str(n), updates_received=len(request.layers))


def test_loopback_service_roundtrip():
    assert GRPC_MAX_MESSAGE_BYTES == 2**31 - 1
    assert method_path("SendUpdate") == "/src.omnifed.hybrid.communicator.CentralServer/SendUpdate"
    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=2), options=GRPC_OPTIONS)
    svc = Echo()
    add_CentralServerServicer_to_server(svc, srv)
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{port}", options=GRPC_OPTIONS)
        stub = CentralServerStub(ch)
        r = stub.RegisterClient(pb.ClientInfo(client_id="client_1"))
        assert r.success and r.total_clients == 1 and svc.seen == ["client_1"]
        big = pb.LayerState(layer_name="w", values_data=b"\x01" * (8 << 20), compression_type="QSGDQuantCompression")
        r = stub.SendUpdate(pb.ModelUpdate(client_id="client_1", layers=[big, big], number_samples=3))
        assert r.success and r.message == str(16 << 20) and r.updates_received == 2  # over grpc's 4 MiB default
        with pytest.raises(grpc.RpcError) as e:  # not overridden: UNIMPLEMENTED, as protoc's base class
            stub.GetUpdatedModel(pb.GetModelRequest(client_id="client_1", round_number=0))
        assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
        ch.close()
    finally:
        srv.stop(grace=0)
