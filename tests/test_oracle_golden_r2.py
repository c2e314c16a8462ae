"""The oracle pinned on the round-2 reference fixtures (CPU; tests/golden/gen_golden_r2.py).

* bf16/fp16 QSGD (the reference quantises in the tensor's own dtype, qsgd.py:46-58): the
  oracle's op sequence on the half tensor, with the reference's norm and MT19937 draws,
  reproduces the payload and the decoded floats;
* ``layerwise_decompress`` (core.py:62-71): the oracle equals the reference on Top-K
  selections the reference TopKCompression made;
* one ResNet-18 round through the reference CentralServerServicer: the oracle re-encodes
  both weighted clients (payload SHA-256 per layer) and aggregates them (SHA-256 per
  averaged parameter).
"""

import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

import oracle
from inputs import sha
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb

HERE = os.path.dirname(os.path.abspath(__file__))
DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16}


@pytest.fixture(scope="module")
def g2():
    return np.load(os.path.join(HERE, "golden", "golden_r2.npz"))


@pytest.fixture(scope="module")
def g2i():
    with open(os.path.join(HERE, "golden", "golden_r2_index.json")) as f:
        return json.load(f)


def _same_floats(a, b) -> bool:
    a, b = np.asarray(a, np.float32).reshape(-1), np.asarray(b, np.float32).reshape(-1)
    return a.shape == b.shape and bool(np.all((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))))


def test_half_precision_qsgd(g2, g2i):
    for c in g2i["half"]:
        key = f"half/{c['id']}"
        L = pb.LayerState()
        L.ParseFromString(g2[key + "/layer"].tobytes())
        x = torch.from_numpy(g2[key + "/x"]).to(DTYPES[c["dtype"]])
        if c["weight"] is not None:
            x = torch.mul(x, c["weight"])  # global_grpc.py:104, in the tensor's dtype
        norm = float(np.frombuffer(L.meta_tensor, np.float32)[0])
        u = torch.from_numpy(oracle.mt19937_uniforms(c["seed"], c["n"]))
        q, nv, width, levels = oracle.qsgd_quantize(x, c["s"], norm=norm, u=u)
        assert q.numpy().tobytes() == L.values_data, key
        assert (width, levels) == (L.width, L.level)
        y = oracle.qsgd_dequantize(q, nv, levels, (c["n"],))
        assert y.dtype == torch.float32 and _same_floats(y.numpy(), g2[key + "/y"]), key
        # the oracle's own norm (torch.norm on the half tensor) is the reference's here
        _, own, _, _ = oracle.qsgd_quantize(x, c["s"], u=u)
        assert np.float32(own).tobytes() == L.meta_tensor, key


def test_layerwise_decompress_pinned(g2, g2i):
    for case in g2i["lwd"]:
        cid, clients = case["id"], case["clients"]
        for t, shape in enumerate(case["shapes"]):
            vals = [torch.from_numpy(g2[f"lwd/{cid}/vals/{c}/{t}"]) for c in range(clients)]
            idx = [torch.from_numpy(g2[f"lwd/{cid}/idx/{c}/{t}"]) for c in range(clients)]
            got = oracle.layerwise_decompress(vals, idx, tuple(shape), clients)
            assert got.numpy().reshape(-1).tobytes() == g2[f"lwd/{cid}/out/{t}"].tobytes(), (cid, t)
            # the selections are the oracle's Top-K of the same inputs (k, order)
            assert all(v.numel() == oracle.topk_k(int(np.prod(shape)), case["ratio"]) for v in vals)


def test_resnet18_round_pinned(g2i):
    """Weighted encode of both clients + the servicer's aggregate, all in the oracle."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from gen_golden_r2 import r18_update

    from omnifed_amd.shapes import resnet18

    r18 = g2i["r18"]
    named = resnet18(10)
    decoded = []
    for c, (ns, seed, rec) in enumerate(zip(r18["samples"], r18["seeds"], r18["clients"])):
        upd = {k: torch.mul(v, ns) for k, v in r18_update(c, named).items()}
        torch.manual_seed(seed)
        stream = oracle.MTStream(seed)
        dec = {}
        for (name, shape), r in zip(named, rec):
            flat = upd[name].reshape(-1)
            norm = float(np.uint32(r["norm_bits"]).view(np.float32))
            q, nv, width, levels = oracle.qsgd_quantize(flat, r18["bit_width"], norm=norm,
                                                        u=torch.from_numpy(stream.draw(flat.numel())))
            assert hashlib.sha256(q.numpy().tobytes()).hexdigest() == r["q_sha"], (c, name)
            dec[name] = oracle.qsgd_dequantize(q, nv, levels, shape)
        decoded.append(dec)
    total = sum(r18["samples"])
    for name, _ in named:
        out = oracle.ps_aggregate([d[name] for d in decoded], total)
        assert sha(out.numpy()) == r18["out_sha"][name], name
