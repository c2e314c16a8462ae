"""A 2-client loopback gRPC round on the GPU (BASELINE config 1's flow).

``scripts/grpc_loopback.run_round``: a ``grpc.server`` on 127.0.0.1 with the reference's options
serves this package's ``CentralServerServicer`` (PS on a DeviceAggregator); 2 client threads
(``GrpcClient``) send weighted ResNet-18 QSGD updates (bit_width 4, the reference's MT19937 stream)
through ``encode_updates_dict`` and ``SendUpdate``, then poll ``GetUpdatedModel``.  The averaged
parameters equal the REAL reference servicer's (golden_r2 ``r18``, SHA-256 per parameter), and both
clients end with the server's parameters."""

import json
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_two_client_loopback_round_equals_reference_servicer(gpu):
    pytest.importorskip("grpc")
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scripts"))
    from grpc_loopback import run_round, sha

    with open(os.path.join(HERE, "golden", "golden_r2_index.json")) as f:
        r18 = json.load(f)["r18"]
    server_model, servicer, out = run_round(r18, gpu)
    assert servicer.current_round == 0 and servicer.total_samples == sum(r18["samples"])
    assert servicer.registered_clients == {"client_1", "client_2"}
    for name, p in server_model.named_parameters():
        assert sha(p.data.cpu().numpy()) == r18["out_sha"][name], name
    for model, *_ in out:
        for (n, pc), (_, ps) in zip(model.named_parameters(), server_model.named_parameters()):
            assert torch.equal(pc.data, ps.data), n
