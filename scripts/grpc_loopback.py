#!/usr/bin/env python3
"""A loopback gRPC round of the hybrid hop on one GPU (BASELINE config 1's flow).

    python scripts/grpc_loopback.py [out.json]

A ``grpc.server`` on 127.0.0.1 (ThreadPoolExecutor(10), the reference's 2 GiB - 1 message limits,
global_grpc.py:44-49) serves this package's ``CentralServerServicer`` (the PS on a
``DeviceAggregator``) for 2 clients; 2 client threads (``GrpcClient``) each weight their
ResNet-18 update by ``batch_samples`` (global_grpc.py:104), encode it with QSGD (bit_width 4, the
reference's MT19937 stream from a seed: parity mode) through ``encode_updates_dict``, send it
with ``SendUpdate`` and poll ``GetUpdatedModel`` for the averaged model, decoded into their own
model's parameters (dense downlink: the reference servicer of the fixture had no compressor).
The inputs, seeds and sample counts are golden_r2's ``r18`` round, which the REAL reference
servicer produced (tests/golden/gen_golden_r2.py), so the averaged parameters can be compared
with its SHA-256s.  Client sends are serialised (one MT19937 generator per process, seeded per
client, as the fixture's clients ran in turn); the polls run concurrently.
"""

from __future__ import annotations

import hashlib
import json
import os
import sys
import threading
import time
from concurrent import futures

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from omnifed_amd import shapes  # noqa: E402


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def nested_model(named, device):
    """An nn.Module whose named_parameters() are ``named`` (dotted names via submodules)."""
    root = torch.nn.Module()
    for name, shape in named:
        parts = name.split(".")
        mod = root
        for p in parts[:-1]:
            if not hasattr(mod, p):
                mod.add_module(p, torch.nn.Module())
            mod = getattr(mod, p)
        mod.register_parameter(parts[-1], torch.nn.Parameter(torch.zeros(shape, device=device)))
    return root


def run_round(r18, device, compressor_factory=None):
    """One round; returns (server model, client models, per-client timings, wire sizes)."""
    import grpc

    from gen_golden_r2 import r18_update
    from omnifed_amd.hybrid.communicator.global_grpc_client import GrpcClient
    from omnifed_amd.hybrid.communicator.global_grpc_limits import GRPC_OPTIONS
    from omnifed_amd.hybrid.communicator.global_grpc_pb2_grpc import add_CentralServerServicer_to_server
    from omnifed_amd.hybrid.communicator.global_grpc_server import CentralServerServicer
    from omnifed_amd.hybrid.compression import QSGDQuantCompression

    named = shapes.model_shapes("resnet18")
    server_model = nested_model(named, device)
    servicer = CentralServerServicer(num_clients=2, model=server_model, compressor=None, device=device)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=10), options=GRPC_OPTIONS)
    add_CentralServerServicer_to_server(servicer, server)
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    send_lock = threading.Lock()
    turn = [threading.Event(), threading.Event()]
    turn[0].set()
    out = [None, None]
    errors = []

    def client(c):
        try:
            model = nested_model(named, device)
            comp = (compressor_factory or (lambda: QSGDQuantCompression(bit_width=r18["bit_width"], device=device,
                                                                        rng="mt19937")))()
            cl = GrpcClient(client_id=f"client_{c + 1}", master_addr="127.0.0.1", master_port=port, compressor=comp)
            upd = {k: v.to(device) for k, v in r18_update(c, named).items()}
            samples = r18["samples"][c]
            turn[c].wait(60)
            with send_lock:  # one MT19937 generator per process: the clients draw in turn
                torch.manual_seed(r18["seeds"][c])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ok = cl.send_update_to_server({k: torch.mul(v, samples) for k, v in upd.items()}, samples)
                t_up = time.perf_counter() - t0
            if c + 1 < len(turn):
                turn[c + 1].set()
            assert ok, "SendUpdate failed"
            t0 = time.perf_counter()
            cl.get_averaged_model(model, communicate_params=True, max_polls=20)
            torch.cuda.synchronize()
            t_down = time.perf_counter() - t0
            out[c] = (model, t_up, t_down, dict(cl.last_wire))
            cl.channel.close()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            for ev in turn:
                ev.set()

    threads = [threading.Thread(target=client, args=(c,)) for c in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(300)
    server.stop(grace=1)
    if errors:
        raise RuntimeError("; ".join(errors))
    return server_model, servicer, out


class Turns:
    """Serialises one phase of the clients in a fixed order (the reference's server state depends
    on the order of its requests: arrival order of the sum, and a Top-K server compressor's error
    feedback shared by the GetUpdatedModel requests)."""

    def __init__(self, n):
        self.n, self.next = n, 0
        self.cv = threading.Condition()

    def wait(self, c, timeout=120):
        with self.cv:
            if not self.cv.wait_for(lambda: self.next % self.n == c, timeout):
                raise TimeoutError(f"client {c} never got its turn")

    def done(self):
        with self.cv:
            self.next += 1
            self.cv.notify_all()


def run_rounds(named, updates, samples, device, client_comp, server_comp=None, rounds=1):
    """``rounds`` rounds of ``len(samples)`` clients over a loopback gRPC server.  ``updates[r][c]``:
    client c's update dict of round r (sent as is, with ``number_samples = samples[c]``);
    ``client_comp()`` builds a client's compressor, ``server_comp`` is the servicer's (None:
    dense downlink).  Uplinks and downlinks run in client order (Turns).  Returns per round the
    server's parameters and each client's parameters after its downlink (CPU copies)."""
    import grpc

    from omnifed_amd.hybrid.communicator.global_grpc_client import GrpcClient
    from omnifed_amd.hybrid.communicator.global_grpc_limits import GRPC_OPTIONS
    from omnifed_amd.hybrid.communicator.global_grpc_pb2_grpc import add_CentralServerServicer_to_server
    from omnifed_amd.hybrid.communicator.global_grpc_server import CentralServerServicer

    C = len(samples)
    server_model = nested_model(named, device)
    servicer = CentralServerServicer(num_clients=C, model=server_model, compressor=server_comp, device=device)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=10), options=GRPC_OPTIONS)
    add_CentralServerServicer_to_server(servicer, server)
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    up, down = Turns(C), Turns(C)
    out = {"server": [None] * rounds, "clients": [[None] * C for _ in range(rounds)]}
    lock = threading.Lock()
    errors = []

    def client(c):
        try:
            model = nested_model(named, device)
            cl = GrpcClient(client_id=f"client_{c + 1}", master_addr="127.0.0.1", master_port=port,
                            compressor=client_comp())
            for r in range(rounds):
                up.wait(c)
                ok = cl.send_update_to_server(updates[r][c], samples[c])
                up.done()
                assert ok, "SendUpdate failed"
                down.wait(c)
                cl.get_averaged_model(model, communicate_params=True, max_polls=20)
                with lock:
                    if out["server"][r] is None:
                        out["server"][r] = {n: p.data.detach().cpu().clone() for n, p in server_model.named_parameters()}
                out["clients"][r][c] = {n: p.data.detach().cpu().clone() for n, p in model.named_parameters()}
                down.done()
                cl.round_number += 1
            cl.channel.close()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=client, args=(c,)) for c in range(C)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(600)
    server.stop(grace=1)
    if errors:
        raise RuntimeError("; ".join(errors))
    return out, servicer


def main():
    dev = torch.device("cuda", 0)
    with open(os.path.join(ROOT, "tests", "golden", "golden_r2_index.json")) as f:
        r18 = json.load(f)["r18"]
    t0 = time.perf_counter()
    server_model, servicer, out = run_round(r18, dev)
    wall = time.perf_counter() - t0
    mism = [n for n, p in server_model.named_parameters() if sha(p.data.cpu().numpy()) != r18["out_sha"][n]]
    client_eq = all(torch.equal(pc.data, ps.data) for m, *_ in out
                    for (_, pc), (_, ps) in zip(m.named_parameters(), server_model.named_parameters()))
    res = {
        "round": "resnet18, 2 clients, QSGD s=4 MT19937 uplink, dense downlink, loopback gRPC 127.0.0.1",
        "wall_s": round(wall, 3),
        "uplink_ms": [round(o[1] * 1e3, 2) for o in out],
        "downlink_ms": [round(o[2] * 1e3, 2) for o in out],
        "uplink_wire_bytes": [o[3].get("wire_bytes") for o in out],
        "server_params_sha_mismatched": mism,
        "clients_equal_server": client_eq,
    }
    print(json.dumps(res))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
