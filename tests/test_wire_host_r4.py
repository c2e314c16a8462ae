"""Host logic of the round-4 wire path (no GPU): Top-K layer validation in the reference's order,
the rules that send a message to the batched Top-K decoder, the LayerState built from payload
bytes, the leased pinned staging (concurrent callers never share a buffer), and the detection of
tensors that already form a plan's arena."""

import threading

import numpy as np
import pytest
import torch

from omnifed_amd import hostio
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as pb
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    _scan_layers,
    _topk_batch_ok,
    decode_updates_dict,
    read_topk_layer,
    topk_layer_from_bytes,
    topk_layer_from_payload,
)
from omnifed_amd.hybrid.compression.core import shared_arena


def _topk(name, n, k, seed=0):
    rng = np.random.default_rng(seed)
    return topk_layer_from_payload(name, (n,), rng.standard_normal(k).astype(np.float32),
                                   rng.permutation(n)[:k].astype(np.int64))


def test_topk_layer_from_bytes_equals_payload_form(golden, golden_index):
    for c in golden_index["topk"]:
        G = pb.LayerState()
        G.ParseFromString(golden[f"topk/{c['id']}/0/layer"].tobytes())
        L = topk_layer_from_bytes("w", tuple(c["shape"]), G.values_data, G.indices_data)
        assert L.SerializeToString() == G.SerializeToString()


def test_read_topk_layer_errors_like_the_reference():
    """global_grpc_compression.py:145-158: missing payloads, a payload that is not a whole number of
    elements (np.frombuffer), a values / indices length mismatch (the fancy assignment)."""
    L = pb.LayerState(layer_name="w", compression_type="TopKCompression")
    with pytest.raises(ValueError, match="missing values/indices"):
        read_topk_layer(L)
    L.values_data = np.ones(3, np.float32).tobytes()
    with pytest.raises(ValueError, match="missing values/indices"):
        read_topk_layer(L)
    L.indices_data = np.arange(3, dtype=np.int64).tobytes()[:-1]
    with pytest.raises(ValueError, match="multiple of element size"):
        read_topk_layer(L)
    L.indices_data = np.arange(2, dtype=np.int64).tobytes()
    with pytest.raises(ValueError, match="3 values, 2 indices"):
        read_topk_layer(L)
    L.indices_data = np.arange(3, dtype=np.int64).tobytes()
    v, i, k = read_topk_layer(L)
    assert k == 3 and len(v) == 12 and len(i) == 24


def test_scan_raises_the_first_bad_layer_in_message_order():
    """A batched decode validates every layer in message order before any work, so it raises the
    reference's first error — here before any GPU is touched."""
    good = _topk("a", 100, 3)
    bad_topk = pb.LayerState(layer_name="b", compression_type="TopKCompression")
    bad_qsgd = pb.LayerState(layer_name="c", compression_type="QSGDQuantCompression", values_data=b"\x01",
                             meta_tensor=np.float32(1).tobytes(), width=16, level=4)
    with pytest.raises(ValueError, match="'b' missing values/indices"):
        decode_updates_dict([good, bad_topk, bad_qsgd])
    with pytest.raises(ValueError, match="unsupported width"):
        decode_updates_dict([good, bad_qsgd, bad_topk])
    groups, topk = _scan_layers([good, _topk("d", 50, 2)])
    assert not groups and [e[0].layer_name for e in topk] == ["a", "d"] and [e[3] for e in topk] == [3, 2]


def test_topk_batch_rules():
    a, b = _topk("a", 100, 3), _topk("b", 10, 10)
    assert _topk_batch_ok(_scan_layers([a, b])[1])
    assert not _topk_batch_ok(_scan_layers([a, _topk("a", 100, 3, 1)])[1])  # a repeated name: per layer
    over = topk_layer_from_payload("o", (4,), np.ones(5, np.float32), np.array([0, 1, 2, 3, 0], np.int64))
    assert not _topk_batch_ok(_scan_layers([a, over])[1])  # more values than elements (duplicates)


@pytest.fixture
def unpinned(monkeypatch):
    """Leases on a CPU-only host: pinned allocations become plain ones (the pool logic is what is tested)."""
    real = torch.empty

    def empty(*args, pin_memory=False, **kw):
        return real(*args, **kw)

    monkeypatch.setattr(hostio.torch, "empty", empty)
    return hostio.PinnedStaging()


def test_staging_leases_are_exclusive_and_reused(unpinned):
    st = unpinned
    with st.lease("k", 100) as a:
        with st.lease("k", 100) as b:  # a concurrent caller: its own buffer
            assert a.buf.data_ptr() != b.buf.data_ptr()
        pa = a.buf.data_ptr()
    with st.lease("k", 50) as c:  # both free again: the smallest that fits
        assert c.buf.numel() == 50 and c.buf.data_ptr() in (pa, b.buf.data_ptr())
    with st.lease("k", 1 << 20) as d:  # grown
        assert d.buf.numel() == 1 << 20


def test_staging_lease_waits_for_the_previous_holders_event(unpinned):
    st = unpinned

    class Ev:
        waited = 0

        def synchronize(self):
            Ev.waited += 1

    with st.lease("k", 64) as a:
        a.event = Ev()
    with st.lease("k", 64):
        pass
    assert Ev.waited == 1


def test_staging_leases_from_threads(unpinned):
    st = unpinned
    held, errors = set(), []
    lock = threading.Lock()

    def work():
        try:
            for _ in range(20):
                with st.lease("t", 4096) as h:
                    p = h.buf.data_ptr()
                    with lock:
                        assert p not in held
                        held.add(p)
                    with lock:
                        held.discard(p)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ts = [threading.Thread(target=work) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors


def test_shared_arena_detection():
    class P:
        offsets = [0, 64, 192]
        sizes = [10, 100, 3]
        arena_end = 195

    buf = torch.zeros(300)
    dev = torch.device("cpu")
    views = [buf[0:10], buf[64:164], buf[192:195]]
    x = shared_arena(views, dev, P)
    assert x is not None and x.data_ptr() == buf.data_ptr() and x.numel() == 195
    shifted = [buf[4:14], buf[68:168], buf[196:199]]  # 16-byte aligned base 4 elements in
    x = shared_arena(shifted, dev, P)
    assert x is not None and x.data_ptr() - buf.data_ptr() == 16
    assert shared_arena([buf[1:11], buf[65:165], buf[193:196]], dev, P) is None  # misaligned base
    assert shared_arena([buf[0:10], buf[64:164], buf[190:193]], dev, P) is None  # wrong offset
    assert shared_arena([buf[0:10], torch.zeros(100), buf[192:195]], dev, P) is None  # another storage
    assert shared_arena([buf[0:10].double(), buf[64:164], buf[192:195]], dev, P) is None  # not fp32
    assert shared_arena([buf[0:10], buf[64:164], buf[192:195]], dev, type("Q", (), {
        "offsets": [0, 64, 192], "sizes": [10, 100, 200], "arena_end": 392})) is None  # storage too short


def test_host_arena_pool_reuses_pages_and_honours_its_budget():
    """Pooled pageable arenas (hostio.HostArenaPool): ordinary writable CPU tensors; the memory of a
    dropped arena (every view gone) serves the next one of a similar size; free arenas above the
    budget are released; small ones are not pooled."""
    import gc

    MiB = 1 << 20
    P = hostio.HostArenaPool(max_bytes=200 * MiB)
    t = P.empty(3 * MiB + 8).view(torch.float32)
    assert t.numel() == (3 * MiB + 8) // 4 and not t.is_pinned()
    t.fill_(2.0)
    view = t[10:20]
    p = t.data_ptr()
    del t
    gc.collect()
    assert P.free_bytes() == 0  # a view still holds the arena
    assert float(view.sum()) == 20.0
    del view
    gc.collect()
    assert P.free_bytes() == 4 * MiB  # rounded up to 1 MiB below the 64 MiB grain
    u = P.empty(3 * MiB)
    assert u.data_ptr() == p and P.free_bytes() == 0
    a, b = P.empty(100 * MiB), P.empty(100 * MiB)  # 128 MiB each (64 MiB grain)
    del u, a, b
    gc.collect()
    assert P.free_bytes() == 4 * MiB + 128 * MiB  # 4 + 128 + 128 MiB freed, 200 MiB kept at most
    big = P.empty(120 * MiB)  # the free 128 MiB arena serves it
    assert P.free_bytes() == 4 * MiB
    del big
    small = P.empty(1000)
    assert small.numel() == 1000 and P.empty(0).numel() == 0
    gc.collect()


def test_host_arena_pool_threads_never_share_live_memory():
    """Concurrent callers (gRPC worker threads) take and drop arenas: two live arenas never overlap,
    and every returned arena is reusable."""
    import gc

    P = hostio.HostArenaPool(max_bytes=1 << 30)
    errors = []
    live = {}
    lock = threading.Lock()

    def work(seed):
        try:
            for i in range(30):
                n = (1 << 20) + 99991 * ((seed * 31 + i) % 50)
                t = P.empty(n)
                a, b = t.data_ptr(), t.data_ptr() + n
                with lock:
                    for (x, y) in live.values():
                        assert b <= x or y <= a, "two live arenas overlap"
                    live[id(t)] = (a, b)
                t.fill_(seed)
                assert int(t.min()) == seed and int(t.max()) == seed
                with lock:
                    del live[id(t)]
                del t
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ts = [threading.Thread(target=work, args=(s,)) for s in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    gc.collect()
    assert not errors, errors
    assert P.free_bytes() > 0
