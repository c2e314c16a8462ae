"""CPU tests of the wire path's host pipeline (omnifed_amd/hostio.py): chunked, threaded copies
between host memory and protobuf-style ``bytes`` give the same bytes in the same order, with and
without worker threads, including empty spans, one-byte spans and chunk-sized spans."""

import ctypes

import numpy as np
import pytest

from omnifed_amd import hostio


def _spans(rng, n):
    sizes = rng.integers(0, 3 << 20, n)
    sizes[::5] = 0
    sizes[1::7] = 1
    offs, cur = [], 0
    for s in sizes:
        cur = (cur + 63) // 64 * 64
        offs.append(cur)
        cur += int(s)
    return list(zip(offs, [int(s) for s in sizes])), cur


@pytest.mark.parametrize("threads", [0, 3])
def test_fill_bytes_and_stage_payloads_roundtrip(threads):
    rng = np.random.default_rng(5)
    spans, total = _spans(rng, 40)
    src = rng.integers(0, 256, total, dtype=np.uint8)
    hostio.set_workers(threads)
    try:
        landed, got = [], {}
        for i, b in hostio.fill_bytes(src.ctypes.data, spans, landed.append, limit=4 << 20):
            assert isinstance(b, bytes)
            got[i] = b
        assert landed == list(range(len(landed))) and len(landed) > 2
        assert sorted(got) == [i for i, (_, n) in enumerate(spans) if n > 0]
        for i, (o, n) in enumerate(spans):
            if n:
                assert got[i] == src[o:o + n].tobytes()
        dst = np.zeros(total, np.uint8)
        flushed = []
        items = [(o, (lambda b=got.get(i, b""): b)) for i, (o, _) in enumerate(spans)]
        hostio.stage_payloads(items, dst.ctypes.data, total, lambda a, b: flushed.append((a, b)), limit=4 << 20)
        for o, n in spans:
            assert dst[o:o + n].tobytes() == src[o:o + n].tobytes()
        assert flushed[0][0] == spans[0][0] and all(a < b for a, b in flushed)
        assert all(flushed[k][1] <= flushed[k + 1][0] for k in range(len(flushed) - 1))
        with pytest.raises(ValueError, match="bad"):
            def check(i, p):
                if i == 17:
                    raise ValueError("bad payload")
            hostio.stage_payloads(items, dst.ctypes.data, total, lambda a, b: None, limit=4 << 20, check=check)
    finally:
        hostio.set_workers(None)


def test_wire_host_memory_policy_once_and_opt_out(monkeypatch):
    """The wire path sets the host-memory policy once per process; OMF_RETAIN_HOST_MEMORY=0
    leaves glibc's defaults alone (hostio.retain_host_memory is never called)."""
    from omnifed_amd.hybrid.communicator import global_grpc_compression as ggc

    calls = []
    monkeypatch.setattr(hostio, "retain_host_memory", lambda: calls.append(1) or True)
    monkeypatch.setattr(ggc, "_HOST_POLICY", None)
    monkeypatch.setenv("OMF_RETAIN_HOST_MEMORY", "0")
    assert ggc._host_memory_policy() is False and calls == []
    monkeypatch.setattr(ggc, "_HOST_POLICY", None)
    monkeypatch.delenv("OMF_RETAIN_HOST_MEMORY")
    assert ggc._host_memory_policy() is True and ggc._host_memory_policy() is True
    assert calls == [1]


def test_retain_host_memory_sets_mallopt():
    assert hostio.retain_host_memory() in (True, False)  # False only without glibc


def test_pinned_leases_returned_after_the_budget_is_removed_are_released(monkeypatch):
    """A page-locked arena handed out while the budget allowed it, dropped after set_pinned_arenas(0):
    the next pinned_arena call (which returns None) unlocks and frees it, so no page-locked memory
    outlives the budget (the early return used to skip the drain)."""
    import gc

    from omnifed_amd import hostio

    locked = {}
    monkeypatch.setattr(hostio, "_register", lambda ptr, n: locked.__setitem__(ptr, n) or True)
    monkeypatch.setattr(hostio, "_unregister", lambda ptr: locked.pop(ptr))
    pool = hostio.HostArenaPool(max_bytes=0, pinned=True)
    monkeypatch.setattr(hostio, "PINNED_ARENAS", pool)
    hostio.set_pinned_arenas(64 << 20)
    a = hostio.pinned_arena(8 << 20)
    assert a is not None and len(locked) == 1 and pool.live_bytes > 0
    hostio.set_pinned_arenas(0)  # the lease is still out: nothing to drain yet
    assert len(locked) == 1
    del a
    gc.collect()
    assert hostio.pinned_arena(8 << 20) is None
    assert not locked and pool.live_bytes == 0
