#!/usr/bin/env python3
"""Round-6 golden vectors from the REAL reference codec: Top-K where magnitudes tie (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_r6.py

Same import shims as ``gen_golden.py``.  Writes ``golden_r6.npz`` + ``golden_r6_index.json``
(the reference's outputs; inputs are regenerated from ``inputs.py``'s recipes, outputs of
more than 100 000 elements are stored as SHA-256).  The reference selects with
``torch.topk(|t'|, k, sorted=False)`` on the CPU (topk.py:13), so among equal magnitudes both
the members taken at rank k and their order are torch's CPU algorithm's; these cases make that
visible:

* ``zero/*``  — fewer than k non-zeros (nnz in {0, 0.3 k, k - 1}) at n in {70 000, 1 000 003},
  ratio 0.01: the selection is completed with zeros (signed zeros are one magnitude).  Two calls
  of one ``TopKCompression`` (error feedback: the second call's t' is the residual plus a second
  sparse input), each call's ``LayerState`` from ``_encode_topk_layer``
  (global_grpc_compression.py:84-98), and the overlay decode of the first call's layer onto a base
  tensor (``_decode_topk_layer(base_tensor=...)``, :153-156: the client downlink);
* ``tied/*``  — a tensor whose k-th magnitude is shared across rank k (both signs), and 24-bit
  integer inputs whose top 1 % holds many equal magnitudes (order inside the selection);
* ``nth/*``   — k * 64 > n (torch's nth_element regime; the reference's own test uses ratio 0.25,
  tests/test_hybrid_global_grpc_compression.py:17), tied and untied;
* ``dict/*``  — ``encode_updates_dict`` of a 4-tensor dict through two error-feedback calls.
"""

from __future__ import annotations

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
from inputs import exact_input, ints, sha, sparse_input, tied_kth  # noqa: E402


def main():
    _install_shim()
    from src.omnifed.hybrid.compression.topk import TopKCompression
    from src.omnifed.hybrid.communicator.global_grpc_compression import (
        _decode_topk_layer,
        _encode_topk_layer,
        encode_updates_dict,
    )

    torch.set_num_threads(8)
    store = {}
    index = {"zero": [], "tied": [], "nth": [], "dict": {}, "layer_sha": {}}

    def layer_arrays(key, layer):
        store[key + "/values"] = np.frombuffer(layer.values_data, np.float32).copy()
        store[key + "/indices"] = np.frombuffer(layer.indices_data, np.int64).copy()
        index["layer_sha"][key] = sha(b2u8(layer.SerializeToString()))

    # ---------------- fewer than k non-zeros: the zero fill ----------------
    cid = 0
    for n in (70000, 1000003):
        k = max(1, int(n * 0.01))
        for nnz in (0, int(0.3 * k), k - 1):
            comp = TopKCompression(device="cpu", compress_ratio=0.01)
            x1 = sparse_input(100 + cid, n, nnz)
            x2 = sparse_input(200 + cid, n, nnz)
            base = exact_input(300 + cid, n, -3)
            key = f"zero/{cid}"
            L1 = _encode_topk_layer("w", torch.from_numpy(x1.copy()), comp)
            layer_arrays(key + "/call0", L1)
            L2 = _encode_topk_layer("w", torch.from_numpy(x2.copy()), comp)
            layer_arrays(key + "/call1", L2)
            res = comp.residual.residuals["w"].numpy().reshape(-1)
            over = _decode_topk_layer(L1, base_tensor=torch.from_numpy(base.copy())).numpy().reshape(-1)
            small = n <= 100000
            if small:
                store[key + "/residual"], store[key + "/overlay0"] = res.copy(), over.copy()
            index["zero"].append(dict(id=cid, n=n, k=k, nnz=nnz, ratio=0.01, seeds=[100 + cid, 200 + cid, 300 + cid],
                                      residual_sha=sha(res), overlay0_sha=sha(over)))
            cid += 1

    # ---------------- ties across rank k, ties inside the selection ----------------
    tid = 0
    for n, kind in ((70000, "kth"), (1000003, "kth"), (200003, "ints"), (1 << 20, "exact")):
        k = max(1, int(n * 0.01))
        x = tied_kth(tid, n, k) if kind == "kth" else ints(tid, n, 3000) if kind == "ints" else exact_input(
            500 + tid, n, -7)
        comp = TopKCompression(device="cpu", compress_ratio=0.01)
        key = f"tied/{tid}"
        L = _encode_topk_layer("w", torch.from_numpy(x.copy()), comp)
        layer_arrays(key, L)
        res = comp.residual.residuals["w"].numpy().reshape(-1)
        index["tied"].append(dict(id=tid, n=n, k=k, kind=kind, ratio=0.01, x_sha=sha(x), residual_sha=sha(res)))
        tid += 1

    # ---------------- k * 64 > n: nth_element's order ----------------
    nid = 0
    for n, ratio, kind in ((1000, 0.25, "exact"), (4099, 0.05, "ints"), (64, 0.5, "ints"), (5000, 0.02, "exact"),
                           (37, 0.1, "ints")):
        x = exact_input(600 + nid, n, -1) if kind == "exact" else ints(600 + nid, n, 7)
        comp = TopKCompression(device="cpu", compress_ratio=ratio)
        key = f"nth/{nid}"
        L = _encode_topk_layer("w", torch.from_numpy(x.copy()), comp)
        layer_arrays(key, L)
        index["nth"].append(dict(id=nid, n=n, k=max(1, int(n * ratio)), ratio=ratio, kind=kind))
        nid += 1

    # ---------------- a dict through encode_updates_dict, two EF calls ----------------
    shapes = [("emb", (1000, 70)), ("w", (300, 300)), ("b", (300,)), ("z", (1200, 64))]
    comp = TopKCompression(device="cpu", compress_ratio=0.01)
    for call in range(2):
        upd = {}
        for t, (name, shape) in enumerate(shapes):
            n = int(np.prod(shape))
            if name == "z":
                x = sparse_input(700 + 10 * call + t, n, 100)
            elif name == "w":
                x = ints(700 + 10 * call + t, n, 200)
            else:
                x = exact_input(700 + 10 * call + t, n, -5)
            upd[name] = torch.from_numpy(x.copy()).reshape(shape)
        layers = encode_updates_dict(upd, comp)
        for L in layers:
            layer_arrays(f"dict/out/{call}/{L.layer_name}", L)
    for name, _ in shapes:
        store[f"dict/residual/{name}"] = comp.residual.residuals[name].numpy().reshape(-1).copy()
    # inputs: dict/x/{call}/{name} = sparse_input(700 + 10 call + t, n, 100) for "z",
    # ints(700 + 10 call + t, n, 200) for "w", exact_input(700 + 10 call + t, n, -5) otherwise
    index["dict"] = dict(shapes=[[n, list(s)] for n, s in shapes], ratio=0.01, calls=2)

    np.savez_compressed(os.path.join(HERE, "golden_r6.npz"), **store)
    with open(os.path.join(HERE, "golden_r6_index.json"), "w") as f:
        json.dump(index, f, indent=1)
    print(f"wrote {len(store)} arrays, {os.path.getsize(os.path.join(HERE, 'golden_r6.npz')) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
