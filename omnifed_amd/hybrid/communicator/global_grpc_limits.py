"""gRPC message size limit of the global hop (mirror of ``src/omnifed/hybrid/communicator/global_grpc_limits.py``).

grpcio converts channel arguments through a signed 32-bit integer: 2 GiB - 1 is the largest
accepted value (the reference's comment, :6-8).  Llama-class dense messages exceed the old
100 MiB default."""

GRPC_MAX_MESSAGE_BYTES = 2147483647
GRPC_OPTIONS = [
    ("grpc.max_send_message_length", GRPC_MAX_MESSAGE_BYTES),
    ("grpc.max_receive_message_length", GRPC_MAX_MESSAGE_BYTES),
]
