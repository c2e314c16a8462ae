"""INTEGRATION.md §2 exercised as a patch: the re-export stubs it documents are read from
INTEGRATION.md itself, executed as modules registered under the reference's module names
(``src.omnifed.hybrid.compression.{core,qsgd,topk}``, ``src.omnifed.hybrid.communicator.
global_grpc_compression``; ``global_grpc_pb2`` is a generated stand-in of the reference's schema),
and reference-shaped call sites then run THROUGH those names:

* the semantics of the reference's own codec tests (tests/test_hybrid_global_grpc_compression.py:
  16-69: Top-K error-feedback round trip, sparse overlay decode, dense legacy path, QSGD layer
  fields, the factory) — re-expressed, not copied;
* a ``GrpcClient._update_model_from_protobuf``-shaped downlink (global_grpc_client.py:98-111:
  ``decode_layer_tensor(layer, base_tensor=param.data)`` then ``target.copy_``) into a model's
  parameters on the GPU, from a ``ModelParameters`` message of the caller's schema, and the
  one-launch ``decode_updates_into`` replacement INTEGRATION.md offers beside it;
* the ``isinstance`` dispatch (global_grpc_compression.py:28-31, 133-137) against the stubs'
  classes.
No reference file is read or copied; the stubs are this repository's documentation.
"""

import os
import re
import sys
import types

import numpy as np
import pytest
import torch

from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb

HERE = os.path.dirname(os.path.abspath(__file__))
INTEGRATION = os.path.join(os.path.dirname(HERE), "INTEGRATION.md")
STUB_RE = re.compile(r"```python\n# (src/omnifed/[\w/]+\.py)\n(.*?)```", re.S)
PACKAGES = ("src", "src.omnifed", "src.omnifed.hybrid", "src.omnifed.hybrid.compression",
            "src.omnifed.hybrid.communicator")


def _stubs():
    with open(INTEGRATION) as f:
        return dict(STUB_RE.findall(f.read()))


@pytest.fixture
def patched(monkeypatch):
    """The INTEGRATION.md §2 patch installed under the reference's module names."""
    mods = {}
    for name in PACKAGES:
        m = types.ModuleType(name)
        m.__path__ = []
        mods[name] = m
        monkeypatch.setitem(sys.modules, name, m)
    schema = pb.schema_module(pb.REFERENCE_MODULE)  # the caller's generated global_grpc_pb2
    mods[pb.REFERENCE_MODULE] = schema
    monkeypatch.setitem(sys.modules, pb.REFERENCE_MODULE, schema)
    for path, code in _stubs().items():
        name = path[:-3].replace("/", ".")
        m = types.ModuleType(name)
        exec(compile(code, path, "exec"), m.__dict__)
        mods[name] = m
        monkeypatch.setitem(sys.modules, name, m)
    for name, m in mods.items():  # attribute chain for `import src.omnifed....x as y`
        parent, _, leaf = name.rpartition(".")
        if parent:
            setattr(mods[parent], leaf, m)
    comp = mods["src.omnifed.hybrid.compression"]  # the package exports (compression/__init__.py:3-21)
    for sub in ("core", "qsgd", "topk"):
        for k, v in vars(mods[f"src.omnifed.hybrid.compression.{sub}"]).items():
            if not k.startswith("_"):
                setattr(comp, k, v)
    return mods


def test_integration_stubs_cover_the_plugin_surface():
    """CPU: the documented patch names every symbol of SURVEY.md §8b's plugin surface."""
    stubs = _stubs()
    assert set(stubs) == {"src/omnifed/hybrid/compression/qsgd.py", "src/omnifed/hybrid/compression/topk.py",
                          "src/omnifed/hybrid/compression/core.py",
                          "src/omnifed/hybrid/communicator/global_grpc_compression.py"}
    text = "\n".join(stubs.values())
    for sym in ("QSGDQuantCompression", "TopKCompression", "Compression", "ResidualUpdates", "layerwise_decompress",
                "QSGD_COMPRESSION_NAME", "TOPK_COMPRESSION_NAME", "build_global_compressor",
                "hybrid_global_compressor_from_cfg", "encode_layer_state", "decode_layer_tensor",
                "encode_updates_dict", "decode_updates_dict", "compression_mode_name"):
        assert re.search(rf"\b{sym}\b", text), sym


@pytest.mark.gpu
def test_reference_codec_semantics_through_the_patch(gpu, patched):
    import src.omnifed.hybrid.communicator.global_grpc_pb2 as wire  # noqa: F401  (the caller's schema)
    from src.omnifed.hybrid.communicator.global_grpc_compression import (
        build_global_compressor, compression_mode_name, decode_layer_tensor, encode_layer_state)
    from src.omnifed.hybrid.compression.qsgd import QSGD_COMPRESSION_NAME, QSGDQuantCompression
    from src.omnifed.hybrid.compression.topk import TOPK_COMPRESSION_NAME, TopKCompression

    torch.manual_seed(0)
    # Top-K with error feedback: k = max(1, int(n * ratio)) values, decompress restores the shape
    tk = TopKCompression(device="cpu", compress_ratio=0.25)
    x = torch.randn(32)
    (values, indices), ctx = tk.compress(x.clone(), name="layer0")
    assert values.numel() == 8 and indices.numel() == 8
    assert tk.decompress((values, indices), ctx).shape == x.shape
    # sparse LayerState: overlay on the base keeps every unselected entry
    tk = TopKCompression(device="cpu", compress_ratio=0.1)
    base = torch.randn(4, 4)
    layer = encode_layer_state("conv.weight", base, tk)
    assert type(layer) is wire.LayerState  # built from the caller's generated module
    assert layer.compression_type == TOPK_COMPRESSION_NAME and len(layer.param_update) == 0
    assert layer.values_data and layer.indices_data
    dec = decode_layer_tensor(layer, base_tensor=base)
    assert dec.shape == base.shape
    keep = torch.ones(16, dtype=torch.bool)
    keep[np.frombuffer(layer.indices_data, dtype=np.int64)] = False
    assert torch.equal(dec.reshape(-1)[keep], base.reshape(-1)[keep])
    # dense legacy path
    t = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    dl = encode_layer_state("dense", t, None)
    assert dl.compression_type == "" and torch.equal(decode_layer_tensor(dl), t)
    # QSGD LayerState fields
    q = QSGDQuantCompression(bit_width=4, device="cpu")
    ql = encode_layer_state("fc.weight", torch.randn(8), q)
    assert ql.compression_type == QSGD_COMPRESSION_NAME and ql.values_data and ql.meta_tensor
    assert (ql.width, ql.level) == (8, 16)
    assert decode_layer_tensor(ql).shape == (8,)
    # the factory and the isinstance dispatch against the stubs' classes
    c = build_global_compressor(enabled=True, scheme="qsgd", bit_width=3)
    assert isinstance(c, QSGDQuantCompression) and c.s == 3
    assert compression_mode_name(c) == "QSGD" and compression_mode_name(tk) == "TopK"
    assert build_global_compressor(enabled=False) is None


def _update_model_from_protobuf(communicate_params, model, proto_layers, decode_layer_tensor):
    """global_grpc_client.py:98-111, as the unchanged client runs it (re-expressed)."""
    layer_by_name = {layer.layer_name: layer for layer in proto_layers}
    with torch.no_grad():
        for name, param in model.named_parameters():
            layer = layer_by_name.get(name)
            if layer is None:
                continue
            base = param.data if communicate_params else param.grad
            decoded = decode_layer_tensor(layer, base_tensor=base)
            target = param.data if communicate_params else param.grad
            target.copy_(decoded.to(device=target.device, dtype=target.dtype))
    return model


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", ["topk", "qsgd"])
def test_client_downlink_through_the_patch(gpu, patched, scheme):
    """The PS's averaged model in a ModelParameters of the caller's schema, decoded by the
    unchanged client's _update_model_from_protobuf into a GPU model: Top-K overlays the selected
    entries on the client's parameters (the rest keep their values), QSGD replaces them with the
    decoded average; decode_updates_into gives the same parameters bit for bit."""
    import src.omnifed.hybrid.communicator.global_grpc_pb2 as wire
    from src.omnifed.hybrid.communicator.global_grpc_compression import (
        build_global_compressor, decode_layer_tensor, encode_updates_dict)
    from omnifed_amd.hybrid.communicator.global_grpc_compression import decode_updates_into

    torch.manual_seed(4)
    model = torch.nn.Sequential(torch.nn.Linear(64, 32), torch.nn.ReLU(), torch.nn.Linear(32, 10)).to(gpu)
    server = {n: (p.detach() * 0.5 + 0.1).clone() for n, p in model.named_parameters()}  # the PS's average
    comp = build_global_compressor(enabled=True, scheme=scheme, compress_ratio=0.1, bit_width=4, device="cpu")
    layers = encode_updates_dict(server, comp)
    msg = wire.ModelParameters(round_number=3, layers=layers, is_ready=True)
    got = wire.ModelParameters()
    got.ParseFromString(msg.SerializeToString())
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    _update_model_from_protobuf(True, model, got.layers, decode_layer_tensor)
    other = torch.nn.Sequential(torch.nn.Linear(64, 32), torch.nn.ReLU(), torch.nn.Linear(32, 10)).to(gpu)
    other.load_state_dict({k: v for k, v in before.items()})
    decode_updates_into(got.layers, {n: p.data for n, p in other.named_parameters()})
    for (n, p), L in zip(model.named_parameters(), got.layers):
        assert L.layer_name == n
        assert torch.equal(p.data, dict(other.named_parameters())[n].data), n
        if scheme == "topk":
            ix = torch.from_numpy(np.frombuffer(L.indices_data, dtype=np.int64).copy()).to(gpu)
            flat, b0, s0 = p.data.reshape(-1), before[n].reshape(-1), server[n].reshape(-1)
            keep = torch.ones_like(flat, dtype=torch.bool)
            keep[ix] = False
            assert torch.equal(flat[keep], b0[keep]), n  # the overlay leaves the rest alone
            assert torch.equal(flat[ix], s0[ix]), n      # the selected entries are the server's
        else:
            norm = float(np.frombuffer(L.meta_tensor, np.float32)[0])
            assert float((p.data - server[n]).abs().max()) <= norm / L.level * (1 + 1e-6), n
