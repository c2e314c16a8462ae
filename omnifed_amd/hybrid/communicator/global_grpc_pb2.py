"""Wire schema of the hybrid global gRPC hop, built at import time.

Field numbers and types are the frozen wire contract of
``src/omnifed/hybrid/communicator/global_grpc.proto:16-67`` (reference;
``LayerState`` fields 1-13 at :23-39).  No generated code is needed: the
descriptor is assembled with ``descriptor_pb2`` into a private pool (so it can
live in one process beside the reference's own generated module) and the
message classes come from ``message_factory``.  Serialised bytes are identical
to protoc-generated classes for the same schema (checked against the
reference's own ``SerializeToString`` output in ``tests/test_wire_host.py``).

Interop with the caller's generated module: protobuf refuses a message from another
descriptor pool inside a repeated field (``ModelUpdate(layers=...)`` raises
``TypeError``), and the reference's unchanged client and server put the codec's
``LayerState``s into their OWN generated ``ModelUpdate`` / ``ModelParameters``
(global_grpc_client.py:75-80, global_grpc_server.py:226-230).  So every
``LayerState`` the codec builds comes from ``active_module()``: a module injected
with ``set_wire_module``, else the reference's generated module
``src.omnifed.hybrid.communicator.global_grpc_pb2`` when the process has imported
it, else this private schema (standalone use).
"""

from __future__ import annotations

import sys
import types
from typing import Optional

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "src.omnifed.hybrid.communicator"

_F = descriptor_pb2.FieldDescriptorProto
_T = {
    "string": _F.TYPE_STRING,
    "int32": _F.TYPE_INT32,
    "float": _F.TYPE_FLOAT,
    "bytes": _F.TYPE_BYTES,
    "bool": _F.TYPE_BOOL,
}

# (message, [(field, number, type, repeated)])
_SCHEMA = [
    ("LayerState", [
        ("layer_name", 1, "string", False),
        ("param_update", 2, "float", True),
        ("param_shape", 3, "int32", True),
        ("compression_type", 4, "string", False),
        ("values_data", 5, "bytes", False),
        ("indices_data", 6, "bytes", False),
        ("values_dtype", 7, "string", False),
        ("indices_dtype", 8, "string", False),
        ("original_shape", 9, "int32", True),
        ("meta_tensor", 10, "bytes", False),
        ("meta_tensor_dtype", 11, "string", False),
        ("width", 12, "int32", False),
        ("level", 13, "int32", False),
    ]),
    ("ModelUpdate", [
        ("client_id", 1, "string", False),
        ("round_number", 2, "int32", False),
        ("layers", 3, "LayerState", True),
        ("number_samples", 4, "int32", False),
    ]),
    ("ModelParameters", [
        ("round_number", 1, "int32", False),
        ("layers", 2, "LayerState", True),
        ("is_ready", 3, "bool", False),
    ]),
    ("UpdateResponse", [
        ("success", 1, "bool", False),
        ("message", 2, "string", False),
        ("clients_registered", 3, "int32", False),
        ("updates_received", 4, "int32", False),
    ]),
    ("GetModelRequest", [
        ("client_id", 1, "string", False),
        ("round_number", 2, "int32", False),
    ]),
    ("ClientInfo", [
        ("client_id", 1, "string", False),
    ]),
    ("RegistrationResponse", [
        ("success", 1, "bool", False),
        ("message", 2, "string", False),
        ("total_clients", 3, "int32", False),
    ]),
]

_SERVICE = ("CentralServer", [
    ("SendUpdate", "ModelUpdate", "UpdateResponse"),
    ("GetUpdatedModel", "GetModelRequest", "ModelParameters"),
    ("RegisterClient", "ClientInfo", "RegistrationResponse"),
])


def _build(file_name: str = "omnifed_amd/global_grpc.proto"):
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = file_name
    fdp.package = PACKAGE
    fdp.syntax = "proto3"
    for msg_name, fields in _SCHEMA:
        m = fdp.message_type.add()
        m.name = msg_name
        for fname, num, ftype, rep in fields:
            f = m.field.add()
            f.name = fname
            f.number = num
            f.label = _F.LABEL_REPEATED if rep else _F.LABEL_OPTIONAL
            if ftype in _T:
                f.type = _T[ftype]
            else:
                f.type = _F.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{ftype}"
    svc = fdp.service.add()
    svc.name = _SERVICE[0]
    for mname, req, resp in _SERVICE[1]:
        md = svc.method.add()
        md.name = mname
        md.input_type = f".{PACKAGE}.{req}"
        md.output_type = f".{PACKAGE}.{resp}"
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    return pool, fd


POOL, DESCRIPTOR = _build()


def _cls(name, pool=None):
    return message_factory.GetMessageClass((pool or POOL).FindMessageTypeByName(f"{PACKAGE}.{name}"))


LayerState = _cls("LayerState")
ModelUpdate = _cls("ModelUpdate")
ModelParameters = _cls("ModelParameters")
UpdateResponse = _cls("UpdateResponse")
GetModelRequest = _cls("GetModelRequest")
ClientInfo = _cls("ClientInfo")
RegistrationResponse = _cls("RegistrationResponse")

SERVICE_NAME = f"{PACKAGE}.{_SERVICE[0]}"

MESSAGE_NAMES = [m for m, _ in _SCHEMA]

# ---------------------------------------------------------------- caller's module
REFERENCE_MODULE = "src.omnifed.hybrid.communicator.global_grpc_pb2"
_injected: Optional[types.ModuleType] = None


def set_wire_module(module: Optional[types.ModuleType]) -> None:
    """Build every codec ``LayerState`` from ``module`` (a protoc-generated ``global_grpc_pb2``
    or anything with a compatible ``LayerState``); ``None`` restores the automatic choice."""
    global _injected
    if module is not None and getattr(module, "LayerState", None) is None:
        raise TypeError("set_wire_module: the module has no LayerState message class")
    _injected = module


def active_module():
    """The module whose ``LayerState`` the codec instantiates (see the module docstring)."""
    if _injected is not None:
        return _injected
    mod = sys.modules.get(REFERENCE_MODULE)
    if mod is not None and getattr(mod, "LayerState", None) is not None:
        return mod
    return sys.modules[__name__]


def layer_state(**fields):
    """A ``LayerState`` of the active module."""
    return active_module().LayerState(**fields)


def schema_module(name: str) -> types.ModuleType:
    """A fresh module holding this schema in a pool of its own: stands in for another
    generated ``global_grpc_pb2`` (interop tests)."""
    pool, _ = _build(f"{name.replace('.', '/')}.proto")
    mod = types.ModuleType(name)
    for m in MESSAGE_NAMES:
        setattr(mod, m, _cls(m, pool))
    return mod
