"""A received Top-K layer that repeats an index with k <= n (a malformed message; no
encoder produces one).  The reference decodes every layer as ``dense[indices] = values`` on numpy
(global_grpc_compression.py:140-160 of the reference), which keeps the LAST value of a repeated
index, and the PS adds that dense tensor to its accumulator (global_grpc_server.py:108-111,
147-153); the client overlays ``param.data`` the same way (global_grpc_client.py:98-111).  The
batched device decodes scatter — a repeated index would keep an arbitrary value (zero fill,
overlay) or every value summed (the PS's scatter-add) — so ``omf_topk_check_duplicates`` flags
such a layer and the Python layer decodes it alone with numpy's rule.  Checked here on all three
paths, with negative indices (numpy wraps them) among the repeats."""

import numpy as np
import pytest
import torch

from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import decode_updates_dict, decode_updates_into
from omnifed_amd.ps import DeviceAggregator

pytestmark = pytest.mark.gpu


def _topk_layer(name, shape, values, indices):
    L = pb.LayerState()
    L.layer_name = name
    L.compression_type = "TopKCompression"
    L.values_data = np.asarray(values, np.float32).tobytes()
    L.values_dtype = "float32"
    L.indices_data = np.asarray(indices, np.int64).tobytes()
    L.indices_dtype = "int64"
    L.original_shape.extend(list(shape))
    return L


def _layers():
    rng = np.random.default_rng(3)
    shapes = {"a": (64, 32), "b": (1000,), "c": (3, 5, 7)}
    msgs = {}
    # a: duplicates (incl. a negative alias of a positive index); b: clean; c: duplicates only
    ia = np.array([5, 17, 5, 2047, -1, 100, 17, 5], np.int64)
    msgs["a"] = (rng.standard_normal(ia.size).astype(np.float32), ia)
    ib = rng.choice(1000, 10, replace=False).astype(np.int64)
    msgs["b"] = (rng.standard_normal(10).astype(np.float32), ib)
    ic = np.array([0, 104, 0, 0], np.int64)
    msgs["c"] = (rng.standard_normal(4).astype(np.float32), ic)
    layers = [_topk_layer(n, shapes[n], v, i) for n, (v, i) in msgs.items()]
    return shapes, msgs, layers


def _dense(shape, v, i, base=None):
    n = int(np.prod(shape))
    d = np.zeros(n, np.float32) if base is None else base.reshape(-1).copy()
    d[i] = v  # numpy: wraps negatives, the last value per index wins
    return d


def test_decode_updates_dict_last_value_wins(gpu):
    shapes, msgs, layers = _layers()
    for device in (None, "cuda"):
        out = decode_updates_dict(layers, device=device)
        for n, (v, i) in msgs.items():
            got = out[n].cpu().numpy().reshape(-1)
            assert got.tobytes() == _dense(shapes[n], v, i).tobytes(), (device, n)


def test_decode_updates_into_overlay_last_value_wins(gpu):
    shapes, msgs, layers = _layers()
    g = torch.Generator().manual_seed(1)
    bases = {n: torch.randn(shapes[n], generator=g) for n in shapes}
    targets = {n: b.clone().to(gpu) for n, b in bases.items()}
    decode_updates_into(layers, targets)
    for n, (v, i) in msgs.items():
        want = _dense(shapes[n], v, i, base=bases[n].numpy())
        assert targets[n].cpu().numpy().reshape(-1).tobytes() == want.tobytes(), n


def test_ps_accumulate_last_value_wins(gpu):
    shapes, msgs, layers = _layers()
    named = [(n, shapes[n]) for n in shapes]
    agg = DeviceAggregator(named, device=gpu)
    agg.accumulate_layers(layers, number_samples=3)
    agg.accumulate_layers(layers, number_samples=1)  # a second client with the same message
    acc = agg.acc.cpu().numpy()
    for t, (n, _s) in enumerate(named):
        v, i = msgs[n]
        d = _dense(shapes[n], v, i)
        want = (np.zeros_like(d) + d) + d  # acc += dense per client, fp32
        o = agg.plan.offsets[t]
        assert acc[o:o + d.size].tobytes() == want.tobytes(), n


def test_check_duplicates_ordered_across_streams(gpu):
    """The duplicate check marks and clears a plan-owned bitmap, so it is one of the plan's stateful
    launches (include/omf_codec.h): a call on another stream waits for the plan's previous one.
    Stream A queues ~200 ms of spin before its check; stream B's check, issued right after, must
    complete after A's (not beside it), and both report the same flags."""
    import time
    from omnifed_amd import codec

    shapes, msgs, _ = _layers()
    names = list(shapes)
    sizes = [int(np.prod(shapes[n])) for n in names]
    plan = codec.Plan.get(sizes, device=gpu)
    counts = [msgs[n][1].size for n in names]
    idx = np.concatenate([np.where(msgs[n][1] < 0, msgs[n][1] + s, msgs[n][1]) for n, s in zip(names, sizes)])
    indices = torch.from_numpy(idx.astype(np.int64)).to(gpu)
    want = [1, 0, 1]
    assert plan.topk_check_duplicates(counts, indices).cpu().tolist() == want  # bitmap made
    # spin calibration (torch's sleep kernel: cycles per ms)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    torch.cuda._sleep(10_000_000)
    b.record()
    torch.cuda.synchronize()
    cycles_per_ms = 10_000_000 / max(a.elapsed_time(b), 1e-3)
    sa, sb = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    with torch.cuda.stream(sa):
        torch.cuda._sleep(int(200 * cycles_per_ms))
        fa = plan.topk_check_duplicates(counts, indices, stream=sa.cuda_stream)
    fb = plan.topk_check_duplicates(counts, indices, stream=sb.cuda_stream)
    t0 = time.perf_counter()
    sb.synchronize()
    wait_ms = (time.perf_counter() - t0) * 1e3
    t1 = time.perf_counter()
    sa.synchronize()  # A's spin and check ended before B's check did: nothing left to wait for
    rest_ms = (time.perf_counter() - t1) * 1e3
    torch.cuda.synchronize()
    assert wait_ms > 100.0 and rest_ms < 50.0, (wait_ms, rest_ms)
    assert fa.cpu().tolist() == want and fb.cpu().tolist() == want
    # and back on A with nothing pending: no wait, same flags
    fc = plan.topk_check_duplicates(counts, indices, stream=sa.cuda_stream)
    sa.synchronize()
    assert fc.cpu().tolist() == want
