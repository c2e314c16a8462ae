"""Opt-in bit-packed QSGD wire, host side: the numpy restatement's known
answers and round trips, the layer builder and the decoder's field checks (no GPU)."""

import numpy as np
import pytest

from oracle import bitpack
from omnifed_amd import codec
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    build_global_compressor,
    decode_layer_tensor,
    hybrid_global_compressor_from_cfg,
    qsgd_packed_layer_from_payload,
)
from omnifed_amd.hybrid.compression import QSGD_PACKED_COMPRESSION_NAME


def test_bits_per_element():
    # ceil(log2(2L + 1)): s = log2(L) -> s + 2 bits
    assert [codec.packed_bits(2**s) for s in range(0, 9)] == [2, 3, 4, 5, 6, 7, 8, 9, 10]
    assert codec.packed_bits(3) == 3 and codec.packed_bits(127) == 8 and codec.packed_bits(2**16) == 18
    assert all(bitpack.packed_bits(L) == codec.packed_bits(L) for L in range(1, 3000))
    with pytest.raises(ValueError):
        codec.packed_bits(0)


def test_known_answer():
    # L = 16 (s = 4): codes 0, 32, 16 in 6 bits each, LSB first -> bits 11 and 16 set
    assert bitpack.pack(np.array([-16, 16, 0]), 16) == bytes([0x00, 0x08, 0x01])
    assert bitpack.unpack(bytes([0x00, 0x08, 0x01]), 3, 16).tolist() == [-16, 16, 0]
    # L = 2 (s = 1): codes 0..4 in 3 bits
    assert bitpack.pack(np.array([-2, -1, 0, 1, 2]), 2) == bytes([0b10001000, 0b01000110])


@pytest.mark.parametrize("L", [1, 2, 4, 16, 64, 128, 256, 1000, 2**16])
def test_round_trip(L):
    rng = np.random.default_rng(L)
    for n in (1, 7, 32, 33, 1000):
        q = rng.integers(-L, L + 1, n)
        q[0] = L
        data = bitpack.pack(q, L)
        assert len(data) == (n * bitpack.packed_bits(L) + 7) // 8
        assert np.array_equal(bitpack.unpack(data, n, L), q)
    with pytest.raises(ValueError):
        bitpack.pack(np.array([L + 1]), L)


def test_layer_builder_and_checks():
    L = 16
    q = np.array([3, -16, 0, 16, 5, -1, 2], dtype=np.int64)
    layer = qsgd_packed_layer_from_payload("w", (7,), bitpack.pack(q, L), 0.5, L)
    assert layer.compression_type == QSGD_PACKED_COMPRESSION_NAME == "QSGDBitPackedCompression"
    assert layer.width == 6 and layer.level == 16 and layer.values_dtype == "packed.u6"
    assert np.frombuffer(layer.meta_tensor, np.float32)[0] == 0.5
    assert len(layer.values_data) == 6  # 7 * 6 bits -> 6 bytes
    wire = pb.LayerState()
    wire.ParseFromString(layer.SerializeToString())
    assert wire == layer
    bad = pb.LayerState()
    bad.CopyFrom(layer)
    bad.width = 8
    with pytest.raises(ValueError, match="unsupported width"):
        decode_layer_tensor(bad)
    bad.CopyFrom(layer)
    bad.values_data = layer.values_data[:-1]
    with pytest.raises(ValueError, match="cannot reshape"):
        decode_layer_tensor(bad)
    bad.CopyFrom(layer)
    bad.level = 0
    with pytest.raises(ValueError, match="invalid level"):
        decode_layer_tensor(bad)


def test_opt_in_only():
    assert build_global_compressor(enabled=True, scheme="qsgd", bit_width=4).packed_wire is False
    assert build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, packed_wire=True).packed_wire
    cfg = {"engine": {"hybrid": {"global_compression": {"enabled": True, "scheme": "qsgd", "bit_width": 4}}}}
    assert hybrid_global_compressor_from_cfg(cfg).packed_wire is False
    cfg["engine"]["hybrid"]["global_compression"]["packed_wire"] = True
    assert hybrid_global_compressor_from_cfg(cfg).packed_wire is True
