#!/usr/bin/env python3
"""Round-2 golden vectors from the REAL reference codec (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_r2.py

Same import shims as ``gen_golden.py`` (hydra-free package init, stub ``omegaconf``).
Writes ``golden_r2.npz`` + ``golden_r2_index.json`` (inputs and the reference's outputs
only; large outputs as SHA-256):

* ``half/*``  — QSGD on bfloat16 / float16 tensors (the reference quantises in the
  tensor's own dtype, qsgd.py:46-58), with and without the client weighting
  ``torch.mul(param, batch_samples)`` of global_grpc.py:104, plus fp16 edge cases
  (|vn|·L overflowing fp16, a norm overflowing fp16, fp16 subnormal quotients);
* ``lwd/*``   — ``core.layerwise_decompress`` (core.py:62-71) over Top-K selections that
  the reference ``TopKCompression`` made for 2 and 3 clients of a 3-tensor model;
* ``r18/*``   — one ResNet-18 round (BASELINE config 1): 2 clients weight their
  62-tensor update by batch_samples, encode it with the reference QSGD (bit_width 4,
  MT19937 stream from a seed) and send it to the reference ``CentralServerServicer``;
  the norms, the SHA-256 of every payload and of every averaged parameter are stored.
"""

from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from gen_golden import _install_shim, b2u8  # noqa: E402
from inputs import exact_input, sha  # noqa: E402

R18_SAMPLES = (37, 91)
R18_SEEDS = (3000, 3001)


def r18_update(client: int, named):
    """Client ``client``'s unweighted ResNet-18 update (exact fp32 inputs)."""
    out = {}
    for i, (name, shape) in enumerate(named):
        n = int(np.prod(shape))
        out[name] = torch.from_numpy(exact_input(2000 + 100 * client + i, n, -12)).reshape(shape)
    return out


def _nested_model(named):
    """An nn.Module whose named_parameters() are ``named`` (dotted names via submodules)."""
    root = torch.nn.Module()
    for name, shape in named:
        parts = name.split(".")
        mod = root
        for p in parts[:-1]:
            if not hasattr(mod, p):
                mod.add_module(p, torch.nn.Module())
            mod = getattr(mod, p)
        mod.register_parameter(parts[-1], torch.nn.Parameter(torch.zeros(shape)))
    assert [n for n, _ in root.named_parameters()] == [n for n, _ in named]
    return root


def main():
    _install_shim()
    from src.omnifed.hybrid.compression.core import layerwise_decompress
    from src.omnifed.hybrid.compression.qsgd import QSGDQuantCompression
    from src.omnifed.hybrid.compression.topk import TopKCompression
    from src.omnifed.hybrid.communicator import global_grpc_pb2 as pb
    from src.omnifed.hybrid.communicator.global_grpc_compression import (
        decode_layer_tensor,
        encode_layer_state,
        encode_updates_dict,
    )
    from src.omnifed.hybrid.communicator.global_grpc_server import CentralServerServicer
    from omnifed_amd.shapes import resnet18

    torch.set_num_threads(8)
    store = {}
    index = {"half": [], "lwd": [], "r18": {}}

    # ---------------- QSGD in bfloat16 / float16 ----------------
    hid = 0
    dtypes = {"bf16": torch.bfloat16, "fp16": torch.float16}
    for dname, dt in dtypes.items():
        for (n, s, weight) in [(7, 4, None), (100, 2, None), (1000, 4, None), (4099, 8, None), (1000, 3, 37),
                               (4099, 4, 91), (65537, 4, None), (20000, 6, 5)]:
            seed = 700 + hid
            x = torch.from_numpy(exact_input(seed, n, -6)).to(dt)
            upd = x if weight is None else torch.mul(x, weight)  # global_grpc.py:104
            torch.manual_seed(seed)
            layer = encode_layer_state(f"h{hid}", upd.clone(), QSGDQuantCompression(bit_width=s, device="cpu"))
            y = decode_layer_tensor(layer)
            key = f"half/{hid}"
            store[key + "/x"] = x.float().numpy()
            store[key + "/layer"] = b2u8(layer.SerializeToString())
            store[key + "/y"] = y.float().numpy().reshape(-1)
            norm = float(np.frombuffer(layer.meta_tensor, np.float32)[0]) if layer.meta_tensor else None
            index["half"].append(dict(id=hid, dtype=dname, n=n, s=s, seed=seed, weight=weight, norm=norm,
                                      ctype=layer.compression_type, shape=[n]))
            hid += 1
    edges = [
        ("fp16", torch.tensor([1.0, 0.001, -0.002, 0.0005]), 16, None),   # |vn| * 2^16 = inf in fp16 -> 0
        ("fp16", torch.full((16,), 30000.0), 4, None),                    # the fp16 norm overflows to inf
        ("fp16", torch.tensor([1.0, 1e-6, -3e-7, 2e-5, 0.0, -0.5]), 8, None),  # subnormal fp16 quotients
        ("fp16", torch.tensor([0.25, -0.125, 3.0, 1.0 / 3.0]), 4, 3000),  # weighting rounds in fp16
        ("bf16", torch.tensor([1.0, 1e-30, -2e-38, 3e38 / 4, 7.0]), 20, None),
        ("bf16", torch.tensor([0.1, -0.2, 0.3, 1.0 / 7.0]), 4, 1000001),  # weighting rounds in bf16
    ]
    for dname, t, s, weight in edges:
        seed = 700 + hid
        x = t.to(dtypes[dname])
        upd = x if weight is None else torch.mul(x, weight)
        torch.manual_seed(seed)
        layer = encode_layer_state(f"h{hid}", upd.clone(), QSGDQuantCompression(bit_width=s, device="cpu"))
        y = decode_layer_tensor(layer)
        key = f"half/{hid}"
        store[key + "/x"] = x.float().numpy()
        store[key + "/layer"] = b2u8(layer.SerializeToString())
        store[key + "/y"] = y.float().numpy().reshape(-1)
        norm = float(np.frombuffer(layer.meta_tensor, np.float32)[0]) if layer.meta_tensor else None
        index["half"].append(dict(id=hid, dtype=dname, n=int(t.numel()), s=s, seed=seed, weight=weight, norm=norm,
                                  ctype=layer.compression_type, shape=[int(t.numel())]))
        hid += 1

    # ---------------- layerwise_decompress over reference Top-K selections ----------------
    lwd_shapes = [(10, 100), (37,), (64, 64)]
    for cid, clients in enumerate((2, 3)):
        ratio = 0.05
        sel = []
        for c in range(clients):
            comp = TopKCompression(device="cpu", compress_ratio=ratio)
            per = []
            for t, shape in enumerate(lwd_shapes):
                x = torch.from_numpy(exact_input(4000 + 50 * cid + 10 * c + t, int(np.prod(shape)), -5)).reshape(shape)
                (v, ix), _ = comp.compress(x, name=f"p{t}")
                per.append((v.clone(), ix.clone()))
            sel.append(per)
        for t, shape in enumerate(lwd_shapes):
            out = layerwise_decompress(collected_vals=[sel[c][t][0] for c in range(clients)],
                                       collected_ix=[sel[c][t][1] for c in range(clients)],
                                       tensor_shape=shape, client_count=clients, device="cpu")
            store[f"lwd/{cid}/out/{t}"] = out.numpy().reshape(-1).copy()
            for c in range(clients):
                store[f"lwd/{cid}/vals/{c}/{t}"] = sel[c][t][0].numpy().copy()
                store[f"lwd/{cid}/idx/{c}/{t}"] = sel[c][t][1].numpy().copy()
        index["lwd"].append(dict(id=cid, clients=clients, ratio=ratio, shapes=[list(s) for s in lwd_shapes]))

    # ---------------- one ResNet-18 round through the reference servicer ----------------
    named = resnet18(10)
    model = _nested_model(named)
    servicer = CentralServerServicer(num_clients=2, model=model, compressor=None)
    r18 = {"samples": list(R18_SAMPLES), "seeds": list(R18_SEEDS), "bit_width": 4, "clients": []}
    for c in range(2):
        upd = {k: torch.mul(v, R18_SAMPLES[c]) for k, v in r18_update(c, named).items()}  # global_grpc.py:104
        torch.manual_seed(R18_SEEDS[c])
        comp = QSGDQuantCompression(bit_width=4, device="cpu")
        layers = encode_updates_dict(upd, comp)
        rec = []
        for L in layers:
            rec.append(dict(name=L.layer_name, ctype=L.compression_type,
                            norm_bits=int(np.frombuffer(L.meta_tensor, np.uint32)[0]) if L.meta_tensor else None,
                            q_sha=hashlib.sha256(L.values_data).hexdigest() if L.values_data else None,
                            layer_sha=hashlib.sha256(L.SerializeToString()).hexdigest()))
        r18["clients"].append(rec)
        req = pb.ModelUpdate(client_id=f"c{c}", round_number=0, layers=layers, number_samples=R18_SAMPLES[c])
        resp = servicer.SendUpdate(req, None)
        assert resp.success, resp.message
    r18["out_sha"] = {n: sha(p.data.numpy()) for n, p in model.named_parameters()}
    r18["out_head"] = {n: p.data.numpy().reshape(-1)[:4].tolist() for n, p in model.named_parameters()}
    index["r18"] = r18

    np.savez_compressed(os.path.join(HERE, "golden_r2.npz"), **store)
    with open(os.path.join(HERE, "golden_r2_index.json"), "w") as f:
        json.dump(index, f, indent=1)
    print(f"wrote {len(store)} arrays, {os.path.getsize(os.path.join(HERE, 'golden_r2.npz')) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
