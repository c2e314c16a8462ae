"""The codec on gRPC worker threads (round 4).

The reference PS serves SendUpdate / GetUpdatedModel from ``grpc.server(ThreadPoolExecutor(
max_workers=10))`` (global_grpc.py:44-45): each request runs on whichever worker is free, under
the servicer's ``self.lock`` (global_grpc_server.py:78, 181, 198); a client and the PS may also
share a process.  Per-thread state the codec meets there: torch's current stream and device,
the Top-K encoder's per-thread verdict word (omf_topk.hip), and the pinned staging buffers
(omnifed_amd.hostio: leased per call).  Both tests compare bytes with a single-thread run.
"""

import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    build_global_compressor,
    decode_updates_dict,
    decode_updates_into,
    encode_updates_dict,
)
from omnifed_amd.ps import DeviceAggregator

pytestmark = pytest.mark.gpu

# ~37.6 M elements: the int8 payload spans two 32 MiB staging chunks
SHAPES = [("emb", (16384, 1024)), ("w1", (2048, 1024)), ("b1", (2048,)), ("w2", (1024, 2048)), ("n", (7,)),
          ("head", (16000, 1024))]
SAMPLES = [5, 11, 3, 8]


def _updates(gpu, c):
    g = torch.Generator(device=gpu).manual_seed(100 + c)
    return {n: torch.randn(*s, device=gpu, generator=g) * 1e-3 for n, s in SHAPES}


def _compressor(scheme, gpu, instance):
    comp = build_global_compressor(enabled=True, scheme=scheme, bit_width=4, compress_ratio=0.01, device=gpu)
    if scheme == "qsgd":
        comp._instance = instance  # a fixed Philox key across the runs (key = f(seed, instance, client))
        comp.client_id = instance
    return comp


def _round(gpu, scheme, run):
    """One PS round: 4 clients encode (``run(fn)`` decides the thread of each call), the PS
    accumulates each SendUpdate under its lock in a fixed order, applies and re-encodes
    (GetUpdatedModel), and every client decodes the downlink into its model."""
    clients = [_compressor(scheme, gpu, c) for c in range(len(SAMPLES))]
    msgs = [None] * len(SAMPLES)

    def client_encode(c):
        msgs[c] = encode_updates_dict(_updates(gpu, c), clients[c], weight=float(SAMPLES[c]))

    run([lambda c=c: client_encode(c) for c in range(len(SAMPLES))], ordered=False)
    agg = DeviceAggregator(SHAPES, device=gpu)
    lock = threading.Lock()

    def send_update(c):
        with lock:
            agg.accumulate_layers(msgs[c], SAMPLES[c])

    run([lambda c=c: send_update(c) for c in range(len(SAMPLES))], ordered=True)
    server = _compressor(scheme, gpu, 99)
    down = {}

    def get_updated_model():
        with lock:
            down["avg"], down["layers"] = agg.apply_and_encode(server)

    run([get_updated_model], ordered=True)
    models = [{n: torch.zeros(*s, device=gpu) for n, s in SHAPES} for _ in SAMPLES]
    run([lambda c=c: decode_updates_into(down["layers"], models[c]) for c in range(len(SAMPLES))], ordered=False)
    torch.cuda.synchronize()
    return ([[L.SerializeToString() for L in m] for m in msgs], agg.acc.cpu(),
            [L.SerializeToString() for L in down["layers"]], [{n: t.cpu() for n, t in m.items()} for m in models])


def _inline(fns, ordered):
    for f in fns:
        f()


def _workers(pool, seen):
    """Unordered calls all at once on the pool's workers; ordered calls one after another, each on a
    thread of its own."""

    def run(fns, ordered):
        if not ordered:
            for f in [pool.submit(lambda f=f: (seen.add(threading.get_ident()), f())) for f in fns]:
                f.result()
            return
        # each call on a new thread that stays alive until the round's calls are done, so every
        # call runs on a thread no earlier call ran on
        alive, errors = [], []
        for f in fns:
            finished, release = threading.Event(), threading.Event()

            def body(f=f, finished=finished, release=release):
                seen.add(threading.get_ident())
                try:
                    f()
                except BaseException as e:  # re-raised on the calling thread
                    errors.append(e)
                finally:
                    finished.set()
                    release.wait()

            t = threading.Thread(target=body)
            t.start()
            finished.wait()
            alive.append((t, release))
        for t, release in alive:
            release.set()
            t.join()
        if errors:
            raise errors[0]

    return run


@pytest.mark.parametrize("scheme", ["qsgd", "topk"])
def test_servicer_calls_from_worker_threads_equal_single_thread(gpu, scheme):
    want = _round(gpu, scheme, _inline)
    seen = set()
    with ThreadPoolExecutor(max_workers=10) as pool:
        got = _round(gpu, scheme, _workers(pool, seen))
    assert len(seen) >= 3
    assert got[0] == want[0]  # every client's LayerStates
    assert torch.equal(got[1], want[1])  # the PS accumulator
    assert got[2] == want[2]  # the downlink
    for a, b in zip(got[3], want[3]):
        for n in a:
            assert torch.equal(a[n], b[n]), n


def test_client_and_ps_threads_unlocked_on_different_plans(gpu):
    """A client thread (QSGD and Top-K encodes of its own model, its own plans) and a PS thread
    (accumulate + apply_and_encode of another model) run at once, without a shared lock, three
    rounds each: every result equals the same work done on one thread."""
    ps_shapes = [("a", (3000, 2000)), ("b", (4099,)), ("c", (1 << 22,))]

    def ps_work():
        out = []
        agg = DeviceAggregator(ps_shapes, device=gpu)
        for r in range(3):
            comp = _compressor("topk" if r % 2 else "qsgd", gpu, 50 + r)
            g = torch.Generator(device=gpu).manual_seed(7 + r)
            upd = {n: torch.randn(*s, device=gpu, generator=g) for n, s in ps_shapes}
            layers = encode_updates_dict(upd, comp, weight=2.0)
            agg.reset()
            agg.accumulate_layers(layers, 2)
            _, down = agg.apply_and_encode(_compressor("qsgd", gpu, 60 + r))
            out.append(([L.SerializeToString() for L in layers], [L.SerializeToString() for L in down]))
        torch.cuda.synchronize()
        return out

    def client_work():
        out = []
        q, t = _compressor("qsgd", gpu, 70), _compressor("topk", gpu, 71)
        for r in range(3):
            upd = _updates(gpu, 20 + r)
            out.append([L.SerializeToString() for L in encode_updates_dict(upd, q)]
                       + [L.SerializeToString() for L in encode_updates_dict(upd, t)])
        torch.cuda.synchronize()
        return out

    want = (ps_work(), client_work())
    res = {}
    threads = [threading.Thread(target=lambda: res.__setitem__("ps", ps_work())),
               threading.Thread(target=lambda: res.__setitem__("client", client_work()))]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert res["ps"] == want[0]
    assert res["client"] == want[1]


@pytest.mark.parametrize("dtype", [torch.float32, torch.int8])
def test_device_to_host_ring_equals_cpu(gpu, dtype):
    """hostio.device_to_host (the CPU placement's D2H): same bytes as .cpu() for empty, odd-sized
    and many-chunk tensors — through the D2HRing into pageable memory (the ring wrapping several
    times: small chunks, 3 slots; from the main thread and from concurrent threads, each call
    leasing its own ring), into the pooled pageable arenas and, with a budget, the page-locked ones."""
    from omnifed_amd import hostio

    g = torch.Generator(device=gpu).manual_seed(5)
    srcs = [torch.empty(0, device=gpu, dtype=dtype)]
    for n in (1, 4099, 3 * (1 << 20) + 5):
        t = torch.randn(n, device=gpu, generator=g) * 100
        srcs.append(t.to(dtype))
    for s in srcs:
        out = hostio.device_to_host(s, limit=1 << 16, slots=3, pool_memory=False)  # the D2HRing
        assert out.device.type == "cpu" and out.dtype == dtype and not out.is_pinned()
        assert torch.equal(out, s.cpu())
        pooled = hostio.device_to_host(s)  # a pooled pageable arena from 1 MiB up (page-locked: opt-in)
        assert pooled.dtype == dtype and torch.equal(pooled, s.cpu()) and not pooled.is_pinned()
        hostio.set_pinned_arenas(64 << 20)
        try:
            pinned = hostio.device_to_host(s)  # with a budget: a page-locked arena from 1 MiB up
        finally:
            hostio.set_pinned_arenas(0)
        assert pinned.dtype == dtype and torch.equal(pinned, s.cpu())
        assert pinned.is_pinned() == (s.numel() * s.element_size() >= hostio.HostArenaPool.MIN_BYTES)
    with ThreadPoolExecutor(4) as ex:
        outs = list(ex.map(lambda s: hostio.device_to_host(s, limit=1 << 16, slots=3, pool_memory=False), srcs * 2))
    for o, s in zip(outs, srcs * 2):
        assert torch.equal(o, s.cpu())


@pytest.mark.parametrize("bits", [4, 8])
def test_qsgd_cpu_placement_pipeline_equals_device_decode(gpu, bits):
    """decode_updates_dict() on the CPU (the reference's placement) decodes chunk by chunk as the
    payloads arrive and copies the decoded chunks out on a second stream: bit-identical to the
    device decode copied afterwards, for a message of several staging chunks (int8 and int32
    wire), padding between tensors included."""
    g = torch.Generator(device=gpu).manual_seed(40 + bits)
    sizes = {"a": (4099,), "b": (3, 7), "c": (9 << 20,), "d": (1,), "e": (12 << 20,), "f": (1000, 1001)}
    upd = {n: torch.randn(*s, device=gpu, generator=g) * 1e-2 for n, s in sizes.items()}
    comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=bits, device=gpu)
    layers = encode_updates_dict(upd, comp)
    on_cpu = decode_updates_dict(layers)
    on_gpu = decode_updates_dict(layers, device="cuda")
    for L in layers:
        a, b = on_cpu[L.layer_name], on_gpu[L.layer_name]
        assert a.device.type == "cpu" and a.dtype == torch.float32 and a.shape == b.shape
        assert np.array_equal(a.numpy().view(np.int32), b.cpu().numpy().view(np.int32)), L.layer_name


def test_pinned_arena_pool_tensors_are_page_locked(gpu):
    """Page-locked arenas are opt-in and bounded (round 5): the product pool has no budget unless
    OMF_PIN_HOST_ARENAS gives it one; a pinned pool's tensors are seen by torch as pinned (the
    copies into them are asynchronous DMAs); every page-locked byte, handed out or free, counts
    against the budget (a request beyond it gets None); a trimmed buffer is unregistered."""
    import gc
    import os

    from omnifed_amd import hostio

    if not os.environ.get("OMF_PIN_HOST_ARENAS"):
        assert hostio.PINNED_ARENAS.max_bytes == 0 and hostio.pinned_arena(4 << 20) is None
    MiB = 1 << 20
    P = hostio.HostArenaPool(max_bytes=8 * MiB, pinned=True)
    t = P.empty(4 * MiB)
    assert t.is_pinned() and P.live_bytes == 4 * MiB
    src = torch.arange(1 << 20, device=gpu, dtype=torch.float32)
    t.view(torch.float32).copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    assert torch.equal(t.view(torch.float32), src.cpu())
    u = P.empty(4 * MiB)
    assert u is not None and P.live_bytes == 8 * MiB
    assert P.empty(2 * MiB) is None  # over the budget: the caller takes the pageable path
    del u
    gc.collect()
    w = P.empty(2 * MiB)  # the free 4 MiB buffer serves it (no new page-locked memory)
    assert w is not None and P.live_bytes == 8 * MiB
    del t, w
    gc.collect()
    P.set_max_bytes(0)  # trims every free buffer: unregistered, memory released
    assert P.free_bytes() == 0 and P.live_bytes == 0


def test_cpu_placement_returns_pageable_memory_by_default(gpu):
    """decode_updates_dict's CPU placement hands the caller pageable (pooled) memory unless pinned
    arenas were asked for; with a budget (hostio.set_pinned_arenas) the same bytes come back
    page-locked."""
    import os

    from omnifed_amd import hostio
    from omnifed_amd.hybrid.communicator.global_grpc_compression import (
        build_global_compressor, decode_updates_dict, encode_updates_dict)

    if os.environ.get("OMF_PIN_HOST_ARENAS"):
        pytest.skip("pinned arenas enabled by the environment")
    g = torch.Generator(device=gpu).manual_seed(5)
    upd = {f"w{i}": torch.randn(n, device=gpu, generator=g) for i, n in enumerate((1 << 20, 700_001, 3000))}
    for scheme in ("qsgd", "topk"):
        comp = build_global_compressor(enabled=True, scheme=scheme, bit_width=4, compress_ratio=0.05, device=gpu)
        layers = encode_updates_dict(upd, comp)
        a = decode_updates_dict(layers)
        assert not any(t.is_pinned() for t in a.values()), scheme
        hostio.set_pinned_arenas(256 << 20)
        try:
            b = decode_updates_dict(layers)
            assert a["w0"].numel() * 4 < hostio.HostArenaPool.MIN_BYTES or b["w0"].is_pinned(), scheme
        finally:
            hostio.set_pinned_arenas(0)
        for n in upd:
            assert a[n].numpy().tobytes() == b[n].numpy().tobytes(), (scheme, n)
