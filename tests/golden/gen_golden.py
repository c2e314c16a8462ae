#!/usr/bin/env python3
"""Generate golden vectors from the REAL reference codec (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Imports ``/root/reference/src/omnifed/hybrid/{compression,communicator}`` with
two import shims: the ``src.omnifed.hybrid`` package
``__init__`` (which needs hydra) is skipped, and ``omegaconf`` is stubbed with
the two names ``global_grpc_compression.py:11`` imports.  Nothing from the
reference is copied: only inputs and the reference's outputs are written, as
``.npz`` data under ``tests/golden/``.

Inputs are exact by construction (integers scaled by powers of two / float32
casts), so tests regenerate the large ones from their seed and compare a
SHA-256 instead of storing them.
"""

from __future__ import annotations

import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from inputs import exact_input, sha  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _install_shim():
    if not os.path.isdir(REF):
        raise SystemExit("reference tree not present: golden vectors can only be generated in the build container")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    om = types.ModuleType("omegaconf")

    class _OC:
        @staticmethod
        def select(cfg, key, default=None):
            cur = cfg
            for part in key.split("."):
                if isinstance(cur, dict) and part in cur:
                    cur = cur[part]
                else:
                    return default
            return cur

    om.OmegaConf = _OC
    om.DictConfig = dict
    sys.modules["omegaconf"] = om
    import src.omnifed as o  # noqa: F401

    pkg = types.ModuleType("src.omnifed.hybrid")
    pkg.__path__ = [os.path.join(REF, "src/omnifed/hybrid")]
    sys.modules["src.omnifed.hybrid"] = pkg
    o.hybrid = pkg


def b2u8(b: bytes) -> np.ndarray:
    return np.frombuffer(b, dtype=np.uint8).copy()


def main():
    _install_shim()
    from src.omnifed.hybrid.compression.qsgd import QSGDQuantCompression
    from src.omnifed.hybrid.compression.topk import TopKCompression
    from src.omnifed.hybrid.communicator import global_grpc_pb2 as pb
    from src.omnifed.hybrid.communicator.global_grpc_compression import (
        build_global_compressor,
        decode_layer_tensor,
        decode_updates_dict,
        encode_layer_state,
        encode_updates_dict,
    )
    from src.omnifed.hybrid.communicator.global_grpc_server import CentralServerServicer

    torch.set_num_threads(8)
    store = {}
    index = {"qsgd": [], "qsgd_hashed": [], "qsgd_edge": [], "topk": [], "dict": [], "ps": []}

    # ---------------- QSGD single-tensor cases (stored in full) ----------------
    sizes = [1, 7, 8, 9, 15, 16, 17, 100, 1000, 4099]
    bitw = [1, 2, 3, 4, 6, 7, 8]
    scales = [-13, -7, 0, 6]
    cid = 0
    for n in sizes:
        for s in bitw:
            seed = cid
            sc = scales[cid % len(scales)]
            x = exact_input(seed, n, sc)
            shape = (n,) if n % 4 else (n // 4, 4)
            torch.manual_seed(seed)
            comp = QSGDQuantCompression(bit_width=s, device="cpu")
            layer = encode_layer_state(f"t{cid}", torch.from_numpy(x.copy()).reshape(shape), comp)
            y = decode_layer_tensor(layer).numpy().reshape(-1)
            key = f"qsgd/{cid}"
            store[key + "/x"] = x
            store[key + "/q"] = b2u8(layer.values_data)
            store[key + "/y"] = y.astype(np.float32)
            store[key + "/layer"] = b2u8(layer.SerializeToString())
            norm = float(np.frombuffer(layer.meta_tensor, dtype=np.float32)[0])
            index["qsgd"].append(dict(id=cid, n=n, s=s, seed=seed, shape=list(shape), norm=norm,
                                      width=layer.width, level=layer.level, dtype=layer.values_dtype))
            cid += 1

    # ---------------- QSGD larger cases (hashes only) ----------------
    for (n, s, seed, sc) in [(65537, 4, 101, -10), (65537, 8, 102, 0), (1_000_003, 4, 103, -10),
                             (1_000_003, 3, 104, -10), (1_000_003, 8, 105, -10), (2_359_296, 4, 106, -10)]:
        x = exact_input(seed, n, sc)
        torch.manual_seed(seed)
        comp = QSGDQuantCompression(bit_width=s, device="cpu")
        layer = encode_layer_state("big", torch.from_numpy(x.copy()), comp)
        y = decode_layer_tensor(layer).numpy()
        norm = float(np.frombuffer(layer.meta_tensor, dtype=np.float32)[0])
        index["qsgd_hashed"].append(dict(n=n, s=s, seed=seed, scale_log2=sc, norm=norm,
                                         x_sha=sha(x), q_sha=hashlib.sha256(layer.values_data).hexdigest(),
                                         y_sha=sha(y.astype(np.float32)), width=layer.width,
                                         q_head=list(np.frombuffer(layer.values_data[:64], dtype=np.uint8).tolist())))

    # ---------------- QSGD edge cases ----------------
    nan = float("nan")
    inf = float("inf")
    edges = {
        "zeros": torch.zeros(10),
        "single": torch.tensor([0.0, 0.0, 3.5, 0.0]),
        "negzero": torch.tensor([-0.0, 1.0, -0.0, -2.0, 0.0]),
        "int64": torch.arange(6, dtype=torch.int64).reshape(2, 3),
        "empty": torch.zeros(0),
        "tiny": torch.full((12,), 1e-30),
        "denormal": torch.tensor([1e-40, -3e-41, 0.0, 2e-39]),
        "huge": torch.tensor([3e19, -2e19, 1.0]),
        "nan": torch.tensor([1.0, nan, -2.0]),
        "inf": torch.tensor([1.0, inf, -2.0]),
        "equal": torch.full((64,), 0.25),
        "fourd": torch.from_numpy(exact_input(7, 2 * 3 * 5 * 7, -3)).reshape(2, 3, 5, 7),
    }
    for j, (name, t) in enumerate(edges.items()):
        for s in (2, 4, 8):
            torch.manual_seed(500 + j)
            comp = QSGDQuantCompression(bit_width=s, device="cpu")
            layer = encode_layer_state(name, t.clone(), comp)
            y = decode_layer_tensor(layer)
            key = f"edge/{name}/{s}"
            store[key + "/x"] = t.numpy().copy()
            store[key + "/layer"] = b2u8(layer.SerializeToString())
            store[key + "/y"] = y.numpy().copy()
            index["qsgd_edge"].append(dict(name=name, s=s, seed=500 + j, ctype=layer.compression_type,
                                           dtype=str(t.dtype), shape=list(t.shape)))

    # ---------------- dict-level stream continuity ----------------
    for (s, seed) in [(4, 77), (8, 78), (3, 79)]:
        upd = {
            "a.weight": torch.from_numpy(exact_input(seed, 100, -8)).reshape(10, 10),
            "zero.bias": torch.zeros(50),
            "b.bias": torch.from_numpy(exact_input(seed + 1, 7, -8)),
            "steps": torch.arange(5, dtype=torch.int64),
            "c.weight": torch.from_numpy(exact_input(seed + 2, 1000, -5)).reshape(20, 50),
        }
        torch.manual_seed(seed)
        comp = QSGDQuantCompression(bit_width=s, device="cpu")
        layers = encode_updates_dict(upd, comp)
        dec = decode_updates_dict(layers)
        key = f"dict/{s}"
        for name, t in upd.items():
            store[f"{key}/in/{name}"] = t.numpy().copy()
        for lay in layers:
            store[f"{key}/layer/{lay.layer_name}"] = b2u8(lay.SerializeToString())
            store[f"{key}/dec/{lay.layer_name}"] = dec[lay.layer_name].numpy().copy()
        index["dict"].append(dict(s=s, seed=seed, names=list(upd.keys())))

    # ---------------- Top-K with error feedback, 3 successive calls ----------------
    for tcase, (n, ratio, shape) in enumerate([(32, 0.25, (32,)), (1000, 0.01, (10, 100)),
                                               (4099, 0.05, (4099,)), (100, 0.001, (100,)),
                                               (65536, 0.01, (256, 256))]):
        comp = TopKCompression(device="cpu", compress_ratio=ratio)
        calls = []
        for call in range(3):
            x = torch.from_numpy(exact_input(900 + 10 * tcase + call, n, -6)).reshape(shape)
            layer = encode_layer_state("w", x.clone(), comp)
            base = torch.from_numpy(exact_input(950 + 10 * tcase + call, n, -6)).reshape(shape)
            dec_zero = decode_layer_tensor(layer)
            dec_base = decode_layer_tensor(layer, base_tensor=base)
            key = f"topk/{tcase}/{call}"
            store[key + "/x"] = x.numpy().copy()
            store[key + "/base"] = base.numpy().copy()
            store[key + "/layer"] = b2u8(layer.SerializeToString())
            store[key + "/residual"] = comp.residual.residuals["w"].numpy().copy()
            store[key + "/dec_zero"] = dec_zero.numpy().copy()
            store[key + "/dec_base"] = dec_base.numpy().copy()
            calls.append(call)
        index["topk"].append(dict(id=tcase, n=n, ratio=ratio, shape=list(shape), calls=calls))

    # ---------------- PS aggregate-after-decode (servicer driven directly) ----------------
    for pcase, (scheme, s) in enumerate([("qsgd", 4), ("qsgd", 8), ("topk", 0)]):
        model = torch.nn.Sequential(torch.nn.Linear(16, 8), torch.nn.Linear(8, 3))
        names = [n for n, _ in model.named_parameters()]
        comp = build_global_compressor(enabled=True, scheme=scheme, bit_width=s, compress_ratio=0.25)
        servicer = CentralServerServicer(num_clients=3, model=model, compressor=None)
        samples = [5, 11, 3]
        for c in range(3):
            upd = {}
            for k_, (name, p) in enumerate(model.named_parameters()):
                upd[name] = torch.from_numpy(exact_input(1200 + 31 * pcase + 7 * c + k_, p.numel(), -4)).reshape(p.shape)
            torch.manual_seed(1300 + pcase * 10 + c)
            client_comp = build_global_compressor(enabled=True, scheme=scheme, bit_width=s, compress_ratio=0.25)
            layers = encode_updates_dict(upd, client_comp)
            req = pb.ModelUpdate(client_id=f"c{c}", round_number=0, layers=layers, number_samples=samples[c])
            resp = servicer.SendUpdate(req, None)
            assert resp.success, resp.message
            store[f"ps/{pcase}/req/{c}"] = b2u8(req.SerializeToString())
        for name, p in model.named_parameters():
            store[f"ps/{pcase}/out/{name}"] = p.data.numpy().copy()
        index["ps"].append(dict(id=pcase, scheme=scheme, s=s, samples=samples, names=names))
        del comp

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **store)
    with open(os.path.join(HERE, "golden_index.json"), "w") as f:
        json.dump(index, f, indent=1)
    tot = os.path.getsize(os.path.join(HERE, "golden.npz"))
    print(f"wrote {len(store)} arrays, {tot/1e6:.2f} MB")


if __name__ == "__main__":
    main()
