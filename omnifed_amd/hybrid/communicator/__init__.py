"""Drop-in for ``src.omnifed.hybrid.communicator`` codec surface (global gRPC hop)."""
