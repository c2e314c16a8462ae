"""Opt-in bit-packed QSGD wire on the GPU: omf_qsgd_pack against the numpy restatement
(oracle/bitpack.py), packed decode bit-identical to the int8/int32 decode, and the wire
round trip through encode_updates_dict / decode_updates_dict / decode_layer_tensor."""

import numpy as np
import pytest
import torch

import oracle
from oracle import bitpack
from omnifed_amd import codec
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    build_global_compressor,
    decode_layer_tensor,
    decode_updates_dict,
    decode_updates_into,
    encode_updates_dict,
)
from omnifed_amd.hybrid.compression import QSGD_PACKED_COMPRESSION_NAME

pytestmark = pytest.mark.gpu

SIZES = [5, 64, 1000, 16385, 70001, 3, 1 << 18, 1155]  # ends on a partial group of 32


@pytest.mark.parametrize("s", [0, 1, 2, 3, 4, 6, 7, 8, 12])
def test_pack_matches_oracle_and_decode_is_identical(gpu, s):
    plan = codec.Plan(SIZES, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(s)
    x = torch.randn(plan.arena_end, device=gpu, generator=g)
    q, norms = plan.qsgd_encode(x, s, seed=7, offset=s)
    L = 2**s
    width = codec.storage_width(L)
    packed = plan.qsgd_pack(q, width, L)
    assert packed.numel() == plan.packed_words(L) == -(-plan.arena_end // 32) * codec.packed_bits(L)
    ph = packed.cpu().numpy().view(np.uint8)
    qh = q.cpu().numpy()
    b = codec.packed_bits(L)
    for o, n in zip(plan.offsets, plan.sizes):
        start = o * b // 8
        got = ph[start:start + (n * b + 7) // 8].tobytes()
        assert got == bitpack.pack(qh[o:o + n], L), (s, n)
    y_ref = plan.qsgd_decode(q, width, L, norms)
    y = plan.qsgd_decode_packed(packed, L, norms)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(y[o:o + n], y_ref[o:o + n]), (s, n)
    # accumulate mode (the PS decode-accumulate)
    acc = torch.randn(plan.arena_end, device=gpu, generator=g)
    acc_ref = acc.clone()
    plan.qsgd_decode(q, width, L, norms, y_out=acc_ref, accumulate=True)
    plan.qsgd_decode_packed(packed, L, norms, y_out=acc, accumulate=True)
    for o, n in zip(plan.offsets, plan.sizes):
        assert torch.equal(acc[o:o + n], acc_ref[o:o + n]), (s, n)


@pytest.mark.parametrize("bits", [2, 4, 8])
def test_packed_wire_round_trip(gpu, bits):
    g = torch.Generator().manual_seed(bits)
    named = [("w0", (64, 33)), ("b0", (33,)), ("w1", (1000, 17)), ("z", (7, 5)), ("w2", (3, 5, 7, 11))]
    upd = {n: (torch.zeros(s) if n == "z" else torch.randn(s, generator=g) * 1e-2).to(gpu) for n, s in named}
    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=bits, device=gpu, packed_wire=True)
    layers = encode_updates_dict(upd, comp)
    L = 2**bits
    b = codec.packed_bits(L)
    for layer, (n, s) in zip(layers, named):
        numel = int(np.prod(s))
        if n == "z":  # zero norm: dense, as the reference
            assert layer.compression_type == ""
            continue
        assert layer.compression_type == QSGD_PACKED_COMPRESSION_NAME and layer.width == b and layer.level == L
        assert len(layer.values_data) == (numel * b + 7) // 8
    got = decode_updates_dict(layers)
    got_dev = decode_updates_dict(layers, device=gpu)
    for layer, (n, s) in zip(layers, named):
        if n == "z":
            assert torch.equal(got[n], torch.zeros(s))
            continue
        numel = int(np.prod(s))
        q = bitpack.unpack(layer.values_data, numel, L)
        assert np.all(np.abs(q) <= L)
        norm = float(np.frombuffer(layer.meta_tensor, np.float32)[0])
        want = oracle.qsgd_dequantize(torch.from_numpy(q), norm, L, s)
        assert got[n].numpy().tobytes() == want.numpy().tobytes(), n
        assert torch.equal(got_dev[n].cpu(), got[n])
        assert torch.equal(decode_layer_tensor(layer), got[n])
        # |decode - x| <= norm / L (QSGD's per-element bound)
        assert float((got[n] - upd[n].cpu()).abs().max()) <= norm / L * (1 + 1e-6)
    targets = {n: torch.full(s, 3.0, device=gpu) for n, s in named}
    decode_updates_into(layers, targets)
    for n, _ in named:
        assert torch.equal(targets[n].cpu(), got[n]), n


def test_packed_wire_is_smaller(gpu):
    upd = {"w": torch.randn(1 << 20, device=gpu)}
    for bits, ratio in ((4, 6 / 8), (2, 4 / 8), (8, 10 / 32)):
        plain = encode_updates_dict(upd, build_global_compressor(enabled=True, scheme="qsgd", bit_width=bits,
                                                                 device=gpu))
        packed = encode_updates_dict(upd, build_global_compressor(enabled=True, scheme="qsgd", bit_width=bits,
                                                                  device=gpu, packed_wire=True))
        assert len(packed[0].values_data) == int(len(plain[0].values_data) * ratio)


@pytest.mark.parametrize("levels", [5, 16, 100000])  # non-power-of-two, int8 s = 4, runtime width
def test_packed_decode_many_tensors_keeps_padding(gpu, levels):
    """The arena-indexed packed decoder on many small and ragged tensors (blocks that cross
    tensor boundaries, tensors shorter than a group, a partial last group): bit-identical to
    the int8/int32 decode on every tensor, and the arena padding keeps what y held, plain and
    accumulating."""
    rng = np.random.default_rng(levels)
    sizes = [int(v) for v in rng.integers(1, 300, 150)] + [8192, 8191, 40000, 33, 1 << 16, 97]
    plan = codec.Plan(sizes, device=gpu)
    width = codec.storage_width(levels)
    qt = torch.int8 if width == 8 else torch.int32
    q = torch.from_numpy(rng.integers(-levels, levels + 1, plan.arena_end)).to(qt).to(gpu)
    norms = torch.from_numpy(rng.random(plan.nt, dtype=np.float32) + 0.5).to(gpu)
    packed = plan.qsgd_pack(q, width, levels)
    ph = packed.cpu().numpy().view(np.uint8)
    qh = q.cpu().numpy()
    b = codec.packed_bits(levels)
    for o, n in zip(plan.offsets, plan.sizes):  # the pack against the numpy restatement
        assert ph[o * b // 8:o * b // 8 + (n * b + 7) // 8].tobytes() == bitpack.pack(qh[o:o + n], levels), n
    pad = torch.ones(plan.arena_end, dtype=torch.bool)
    for o, n in zip(plan.offsets, plan.sizes):
        pad[o:o + n] = False
    pad = pad.to(gpu)
    y_ref = plan.qsgd_decode(q, width, levels, norms, y_out=torch.full((plan.arena_end,), 7.0, device=gpu))
    for accumulate in (False, True):
        y = torch.full((plan.arena_end,), 7.0, device=gpu)
        plan.qsgd_decode_packed(packed, levels, norms, y_out=y, accumulate=accumulate)
        want = y_ref + 7.0 if accumulate else y_ref
        for o, n in zip(plan.offsets, plan.sizes):
            assert torch.equal(y[o:o + n], want[o:o + n]), (levels, accumulate, n)
        assert bool((y[pad] == 7.0).all()), (levels, accumulate)


def test_packed_wire_needs_offsets_on_groups_of_32(gpu):
    """Offsets that are multiples of 4 but not of 32 are a valid plan, not a packed arena."""
    plan = codec.Plan([100, 50], offsets=[0, 100], device=gpu)
    q = torch.zeros(plan.arena_end + 12, dtype=torch.int8, device=gpu)
    with pytest.raises(ValueError, match="multiples of 32"):
        plan.qsgd_pack(q, 8, 16)
    with pytest.raises(ValueError, match="multiples of 32"):
        plan.qsgd_decode_packed(torch.zeros(plan.packed_words(16), dtype=torch.int32, device=gpu), 16,
                                torch.ones(2, device=gpu))
