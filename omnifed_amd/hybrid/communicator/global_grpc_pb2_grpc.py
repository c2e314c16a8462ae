"""The ``CentralServer`` service over grpcio (mirror of the reference's generated
``src/omnifed/hybrid/communicator/global_grpc_pb2_grpc.py``; proto: ``global_grpc.proto``).

Same names as protoc's output — ``CentralServerStub``, ``CentralServerServicer``,
``add_CentralServerServicer_to_server`` — built on grpcio's generic handlers and this package's
message classes (``global_grpc_pb2``), so no generated code is needed.  Method paths are the
proto's: ``/src.omnifed.hybrid.communicator.CentralServer/{SendUpdate,GetUpdatedModel,RegisterClient}``,
so either side interoperates with the reference's generated stubs.  ``grpc`` is imported on use.
"""

from __future__ import annotations

from . import global_grpc_pb2 as pb

# (method, request class, response class): global_grpc.proto's service
METHODS = (
    ("SendUpdate", pb.ModelUpdate, pb.UpdateResponse),
    ("GetUpdatedModel", pb.GetModelRequest, pb.ModelParameters),
    ("RegisterClient", pb.ClientInfo, pb.RegistrationResponse),
)


def _serialize(msg) -> bytes:
    """Any generated module's message of the schema (the caller's global_grpc_pb2, or ours)."""
    return msg.SerializeToString()


def method_path(name: str) -> str:
    return f"/{pb.SERVICE_NAME}/{name}"


class CentralServerStub:
    """Client stub: one unary-unary callable per method (as the generated stub)."""

    def __init__(self, channel):
        for name, req, resp in METHODS:
            setattr(self, name, channel.unary_unary(method_path(name), request_serializer=_serialize,
                                                    response_deserializer=resp.FromString))


class CentralServerServicer:
    """Service base class: every method answers UNIMPLEMENTED until overridden."""

    def _unimplemented(self, context):
        import grpc

        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")

    def SendUpdate(self, request, context):
        self._unimplemented(context)

    def GetUpdatedModel(self, request, context):
        self._unimplemented(context)

    def RegisterClient(self, request, context):
        self._unimplemented(context)


def add_CentralServerServicer_to_server(servicer, server) -> None:
    import grpc

    handlers = {
        name: grpc.unary_unary_rpc_method_handler(getattr(servicer, name), request_deserializer=req.FromString,
                                                  response_serializer=_serialize)
        for name, req, resp in METHODS
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(pb.SERVICE_NAME, handlers),))
