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


def test_two_round_topk_hop_equals_the_reference_op_sequence(gpu):
    """Two rounds of the reference's default scheme (Top-K both ways, error feedback on every
    client and on the server's downlink compressor, shared by the GetUpdatedModel requests as in
    global_grpc_server.py:213-234) over the loopback channel, uplinks and downlinks in client order:
    the server's averaged parameters and each client's overlaid parameters equal the reference's op
    sequence replayed with the oracle (torch.topk on the CPU, numpy overlay), byte for byte."""
    pytest.importorskip("grpc")
    import numpy as np

    import oracle

    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scripts"))
    from grpc_loopback import run_rounds

    from omnifed_amd.hybrid.compression import TopKCompression

    named = [("emb.weight", (3000, 64)), ("blk.w", (256, 256)), ("blk.b", (256,)), ("head.w", (1000, 70))]
    samples = [37, 91]
    ratio = 0.02
    g = torch.Generator().manual_seed(21)
    updates = [[{n: torch.randn(s, generator=g) * 1e-2 for n, s in named} for _ in samples] for _ in range(2)]
    dev_updates = [[{n: t.to(gpu) for n, t in u.items()} for u in rnd] for rnd in updates]
    out, servicer = run_rounds(named, dev_updates, samples, gpu,
                               client_comp=lambda: TopKCompression(device=gpu, compress_ratio=ratio),
                               server_comp=TopKCompression(device=gpu, compress_ratio=ratio), rounds=2)
    assert servicer.current_round == 1
    # the reference's op sequence on the CPU
    cl_orc = [oracle.TopKOracle(ratio) for _ in samples]
    srv_orc = oracle.TopKOracle(ratio)
    client_params = [{n: torch.zeros(s) for n, s in named} for _ in samples]
    for r in range(2):
        acc = {n: torch.zeros(s) for n, s in named}
        for c in range(len(samples)):
            for n, s in named:
                (v, i), ctx = cl_orc[c].compress(updates[r][c][n], n)
                acc[n] += oracle.topk_desparse(v, i, int(np.prod(s))).view(s)
        avg = {n: acc[n] / sum(samples) for n, _ in named}
        for n, _ in named:
            assert out["server"][r][n].numpy().tobytes() == avg[n].numpy().tobytes(), (r, n)
        for c in range(len(samples)):
            for n, s in named:
                (v, i), _ = srv_orc.compress(avg[n], n)
                base = client_params[c][n].numpy().reshape(-1).copy()
                base[i.numpy()] = v.numpy()
                client_params[c][n] = torch.from_numpy(base.reshape(s))
                assert out["clients"][r][c][n].numpy().tobytes() == client_params[c][n].numpy().tobytes(), (r, c, n)


def test_servicer_refuses_an_update_of_another_round(gpu):
    """global_grpc_server.py:90-100: an update for a round other than the one in progress answers
    success=False and leaves the accumulator alone; decoding errors answer success=False too."""
    from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
    from omnifed_amd.hybrid.communicator.global_grpc_compression import encode_updates_dict
    from omnifed_amd.hybrid.communicator.global_grpc_server import CentralServerServicer

    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scripts"))
    from grpc_loopback import nested_model

    named = [("a", (100, 10)), ("b", (7,))]
    model = nested_model(named, gpu)
    srv = CentralServerServicer(num_clients=2, model=model, device=gpu)
    upd = {n: torch.randn(s, device=gpu) for n, s in named}
    layers = encode_updates_dict(upd, None)
    r = srv.SendUpdate(pb.ModelUpdate(client_id="c1", round_number=3, layers=layers, number_samples=5), None)
    assert r.success and r.updates_received == 1
    r = srv.SendUpdate(pb.ModelUpdate(client_id="c2", round_number=2, layers=layers, number_samples=5), None)
    assert not r.success and "not the current round" in r.message and srv.update_count == 1
    bad = pb.LayerState(layer_name="a", compression_type="QSGDQuantCompression", values_data=b"\x01")
    r = srv.SendUpdate(pb.ModelUpdate(client_id="c2", round_number=3, layers=[bad], number_samples=5), None)
    assert not r.success and r.updates_received == 0 and srv.update_count == 1
    got = srv.GetUpdatedModel(pb.GetModelRequest(client_id="c1", round_number=7), None)
    assert not got.is_ready
