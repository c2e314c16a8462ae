"""Host side of the wire path: pinned staging and chunked PCIe copies, overlapped with the host
copies into and out of protobuf ``bytes``.

The drop-in's wire path starts and ends in gRPC host buffers (``LayerState.values_data``,
global_grpc_compression.py:101-123, 163-182).  With the payload arena on the GPU, what is left
on the host per message is: one DMA of the payload through page-locked staging, one copy
between the staging and Python ``bytes`` objects, and protobuf's own copy into / out of its
message arena (upb copies on every set and every get of a bytes field, holding the GIL).
This module overlaps the first two with the third:

* ``device_to_bytes``: the payload arena is copied device-to-host in ~32 MiB chunks, each
  followed by an event; as soon as a chunk lands, its tensors' ``bytes`` objects are
  allocated (uninitialised, ``PyBytes_FromStringAndSize(NULL, n)``) and filled by worker
  threads (``memmove`` through ctypes releases the GIL), while the caller assigns the
  previous chunk's ``bytes`` to its messages.
* ``bytes_to_device``: each message's bytes (protobuf's get-copy) are copied into the staging
  by the workers, and every finished chunk goes host-to-device while the next chunk's
  messages are read.
* ``device_to_host``: a decoded arena into an ordinary (pageable) CPU tensor — the reference's
  CPU placement — through a ring of pinned chunks, each drained by a worker thread's memmove
  while the next chunks' DMAs run, into pooled pages the next round reuses: 56 ms for
  Llama-400M's 1.6 GB into fresh memory against 126 ms for a plain ``.cpu()``.  Page-locked
  result arenas (one DMA each) are opt-in and bounded (``set_pinned_arenas``).

Nothing here changes bytes: the payload is the encoder's, byte for byte.
"""

from __future__ import annotations

import ctypes
import os
import threading
from concurrent.futures import ThreadPoolExecutor
from contextlib import contextmanager
from typing import Callable, Dict, Iterator, List, Optional, Sequence, Tuple

import torch

CHUNK_BYTES = 32 << 20
INLINE_BYTES = 1 << 20  # a copy this small is done on the calling thread (a pool hand-off costs more)

_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
_bytes_addr = ctypes.pythonapi.PyBytes_AsString
_bytes_addr.restype = ctypes.c_void_p
_bytes_addr.argtypes = [ctypes.py_object]

_pool = None
_pool_lock = threading.Lock()
_workers: Optional[int] = None


class _Inline:
    """Executor of ``workers() == 0``: every copy runs at once on the calling thread."""

    class _Done:
        def __init__(self, value):
            self._value = value

        def result(self):
            return self._value

    def submit(self, fn, *args):
        return self._Done(fn(*args))


def workers() -> int:
    """Copy threads: ``OMF_WIRE_THREADS`` (0 = copy on the calling thread), else half the CPUs
    this process may run on, 2..8."""
    if _workers is not None:
        return _workers
    env = os.environ.get("OMF_WIRE_THREADS")
    if env is not None and env.strip().isdigit():
        return int(env)
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        n = os.cpu_count() or 4
    return max(2, min(8, n // 2))


def set_workers(n: Optional[int]) -> None:
    """Override the copy-thread count (None: back to ``workers()``'s default); tuning hook."""
    global _workers, _pool
    with _pool_lock:
        _workers = None if n is None else max(0, int(n))
        old, _pool = _pool, None
    if isinstance(old, ThreadPoolExecutor):
        old.shutdown(wait=True)


def pool():
    global _pool
    if _pool is None:
        with _pool_lock:
            if _pool is None:
                n = workers()
                _pool = ThreadPoolExecutor(max_workers=n, thread_name_prefix="omf-wire") if n > 0 else _Inline()
    return _pool


def retain_host_memory(mmap_threshold: int = 32 << 20, trim_threshold: int = 1 << 30) -> bool:
    """Process-wide (glibc ``mallopt``): serve allocations below ``mmap_threshold`` from
    the heap and keep up to ``trim_threshold`` of freed heap memory instead of returning it to
    the OS.  The wire path's host cost is dominated by page faults: every round, protobuf
    allocates ~w·N bytes of fresh message memory for the payloads (the previous round's was
    unmapped when its messages were freed), and each first touch of a 4 KiB page faults.  With
    the memory retained, a round reuses the previous round's pages.  Returns False where glibc
    is not available.  The wire path calls it once (global_grpc_compression._host_memory_policy)
    unless OMF_RETAIN_HOST_MEMORY=0."""
    try:
        libc = ctypes.CDLL("libc.so.6")
    except OSError:
        return False
    M_TRIM_THRESHOLD, M_MMAP_THRESHOLD = -1, -3
    return bool(libc.mallopt(M_MMAP_THRESHOLD, int(mmap_threshold))) and bool(
        libc.mallopt(M_TRIM_THRESHOLD, int(trim_threshold)))


class PinnedStaging:
    """Reusable page-locked host buffers, per purpose (``key``), grown on demand.

    ``lease(key, nbytes)`` hands out a buffer no other caller holds until the lease ends: the
    reference PS runs the codec on gRPC worker threads (``ThreadPoolExecutor(max_workers=10)``,
    global_grpc.py:44-45), and a client and the PS may share one process, so two calls may stage
    at once — each gets its own buffer (a key's pool grows to the number of concurrent users:
    one under the servicer's lock).  A caller finishes with a buffer (its copies have landed)
    before its lease ends."""

    def __init__(self):
        self._free: Dict[str, List[tuple]] = {}  # key -> [(buffer, event its last copies completed by)]
        self._lock = threading.Lock()

    @contextmanager
    def lease(self, key: str, nbytes: int) -> Iterator["Lease"]:
        nbytes = max(int(nbytes), 1)
        with self._lock:
            pool = self._free.setdefault(key, [])
            pick = None
            for i, (c, _) in enumerate(pool):  # the smallest free buffer that fits, else the largest (regrown)
                if c.numel() >= nbytes and (pick is None or c.numel() < pool[pick][0].numel()):
                    pick = i
            buf, ev = pool.pop(pick) if pick is not None else (pool.pop() if pool else (None, None))
        if ev is not None:
            ev.synchronize()  # the previous holder's copies out of the buffer have landed
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 4096), dtype=torch.uint8, pin_memory=True)
        h = Lease(buf[:nbytes])
        try:
            yield h
        finally:
            with self._lock:
                self._free.setdefault(key, []).append((buf, h.event))
                self._free[key].sort(key=lambda e: e[0].numel())

    def get(self, key: str, nbytes: int) -> torch.Tensor:
        """A buffer for single-threaded callers that finish with it before their next call (tests,
        tools); product paths take a ``lease``."""
        with self.lease(key, nbytes) as h:
            return h.buf


class Lease:
    """A leased staging buffer; ``event``: set by a holder whose copies out of the buffer are
    still queued when the lease ends (the next holder waits for it)."""

    __slots__ = ("buf", "event")

    def __init__(self, buf: torch.Tensor):
        self.buf = buf
        self.event = None


STAGING = PinnedStaging()


def _groups(spans: Sequence[Tuple[int, int]], limit: int) -> List[Tuple[int, int, List[int]]]:
    """Consecutive spans (byte offset, length; ascending offsets) grouped into chunks of about
    ``limit`` bytes: (first byte, end byte, span indices)."""
    out: List[Tuple[int, int, List[int]]] = []
    cur: List[int] = []
    a = b = 0
    for i, (off, n) in enumerate(spans):
        if cur and off + n - a > limit:
            out.append((a, b, cur))
            cur = []
        if not cur:
            a = off
        cur.append(i)
        b = max(b, off + n)
    if cur:
        out.append((a, b, cur))
    return out


def fill_bytes(base: int, spans: Sequence[Tuple[int, int]], landed: Callable[[int], None],
               limit: int = CHUNK_BYTES) -> Iterator[Tuple[int, bytes]]:
    """Yield ``(i, bytes)`` copies of the host spans i = (byte offset from ``base``, length) in
    order (length 0 skipped).  Chunk g's ``bytes`` objects are allocated once ``landed(g)``
    returns and filled by the worker threads while the caller consumes chunk g - 1; at most two
    chunks of ``bytes`` are alive at a time, so their memory is recycled from one chunk to the
    next instead of being faulted in fresh."""
    ex = pool()
    pending: List[Tuple[int, bytes, object]] = []
    for g, (a, b, idx) in enumerate(_groups(spans, limit)):
        landed(g)
        filled = []
        for i in idx:
            off, n = spans[i]
            if n <= 0:
                continue
            obj = _new_bytes(None, n)
            if n < INLINE_BYTES:
                ctypes.memmove(_bytes_addr(obj), base + off, n)
                filled.append((i, obj, _Inline._Done(None)))
            else:
                filled.append((i, obj, ex.submit(ctypes.memmove, _bytes_addr(obj), base + off, n)))
        for item in pending:  # the previous chunk, while this one is copied
            item[2].result()
            yield item[0], item[1]
        pending = filled
    for item in pending:
        item[2].result()
        yield item[0], item[1]


def device_to_bytes(src: torch.Tensor, spans: Sequence[Tuple[int, int]], stream=None, key: str = "encode",
                    limit: int = CHUNK_BYTES) -> Iterator[Tuple[int, bytes]]:
    """Yield ``(i, bytes)`` for every span i = (byte offset, length) of the device buffer ``src``
    (ascending offsets; length 0 is skipped), in order, each as soon as its bytes are filled.
    The device-to-host copies (one per ~``limit`` bytes, each followed by an event) are queued on
    ``stream`` (default: the current stream of ``src``'s device) behind the work already there."""
    if stream is None:
        stream = torch.cuda.current_stream(src.device)
    raw = src.reshape(-1).view(torch.uint8)
    total = max((off + n for off, n in spans), default=0)
    with STAGING.lease(key, max(total, 1)) as h:
        staged = h.buf
        events = []
        with torch.cuda.stream(stream):
            for a, b, _ in _groups(spans, limit):
                if b > a:
                    staged[a:b].copy_(raw[a:b], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                events.append(ev)
        try:
            yield from fill_bytes(staged.data_ptr(), spans, lambda g: events[g].synchronize(), limit)
        finally:
            events[-1].synchronize() if events else None  # an abandoned generator: the copies land first


def _nbytes(m) -> int:
    return m.numel() * m.element_size() if isinstance(m, torch.Tensor) else m.nbytes


class _HostLease:
    """The owner of one hand-out of a pooled host buffer: numpy arrays made from it (through
    ``__array_interface__``) keep it as their base, torch tensors made from those keep the arrays,
    so it dies with the last tensor that uses the memory — and gives the buffer back to its pool."""

    __slots__ = ("mem", "pool", "__array_interface__")

    def __init__(self, mem, nbytes: int, pool: "HostArenaPool"):
        self.mem = mem
        self.pool = pool
        ptr = mem.data_ptr() if isinstance(mem, torch.Tensor) else mem.ctypes.data
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}

    def __del__(self):
        self.pool._returned.append(self.mem)  # list.append is atomic: no lock in a finaliser


def _register(ptr: int, nbytes: int) -> bool:
    """Page-lock host memory in place (hipHostRegister through torch's runtime binding)."""
    try:
        return int(torch._C._cudart.cudaHostRegister(ptr, nbytes, 0)) == 0
    except Exception:  # pragma: no cover - no HIP runtime
        return False


def _unregister(ptr: int) -> None:
    try:
        torch._C._cudart.cudaHostUnregister(ptr)
    except Exception:  # pragma: no cover
        pass


def _pin_budget_from_env() -> int:
    """``OMF_PIN_HOST_ARENAS``: unset or 0 = no page-locked arenas (the default); 1 = up to 4 GiB;
    any other number = that many MiB."""
    v = os.environ.get("OMF_PIN_HOST_ARENAS", "0").strip()
    if not v.isdigit() or int(v) == 0:
        return 0
    return (4 << 30) if int(v) == 1 else int(v) << 20


class HostArenaPool:
    """Host buffers for decoded arenas returned to the caller (the CPU placement).

    A fresh 1.6 GB ``torch.empty`` every round is mmap'd, its 400 K pages faulted in by the copy and
    unmapped again when the caller drops the tensors (glibc serves blocks above 32 MiB by mmap, and
    ``M_MMAP_THRESHOLD`` cannot go higher): most of the CPU placement's cost.  Here the memory of a
    dropped arena goes back to a pool and the next round's arena reuses its pages.  The tensors
    handed out are ordinary, writable CPU tensors (numpy-backed storage); the pool keeps at most
    ``max_bytes`` of free buffers (the rest goes back to the OS).

    ``pinned``: the buffers are page-locked in place (hipHostRegister on numpy memory), so a DMA
    lands in them directly — opt-in (``OMF_PIN_HOST_ARENAS`` / ``set_pinned_arenas``), because
    page-locking gigabytes on a PS host is a resource-policy change the reference never makes.
    Every page-locked byte, handed out or pooled, counts against ``max_bytes``: ``empty`` returns
    None when a new buffer would exceed it (the caller then takes the pageable path), and a buffer
    trimmed from the pool is unregistered before its memory goes back to the OS."""

    GRAIN = 64 << 20      # sizes rounded up to this above it (to 1 MiB below)
    MIN_BYTES = 1 << 20   # smaller arenas are not pooled

    def __init__(self, max_bytes: int = 8 << 30, pinned: bool = False):
        import numpy as np

        self._np = np
        self.max_bytes = int(max_bytes)
        self.pinned = bool(pinned)
        self.live_bytes = 0  # pinned pools: page-locked bytes, handed out or free
        self._free: List[object] = []
        self._returned: List[object] = []
        self._lock = threading.Lock()

    def _release(self, m) -> None:
        if self.pinned:
            _unregister(m.ctypes.data)
            self.live_bytes -= _nbytes(m)

    def _drain(self) -> None:
        while self._returned:
            self._free.append(self._returned.pop())
        self._free.sort(key=_nbytes)
        kept, total = [], 0
        for m in self._free:  # the smallest first: drop what exceeds the budget
            if total + _nbytes(m) <= self.max_bytes:
                kept.append(m)
                total += _nbytes(m)
            else:
                self._release(m)
        self._free = kept

    def set_max_bytes(self, max_bytes: int) -> None:
        with self._lock:
            self.max_bytes = int(max_bytes)
            self._drain()

    def empty(self, nbytes: int) -> Optional[torch.Tensor]:
        """An uninitialised uint8 CPU tensor of ``nbytes`` backed by pooled memory (a pinned pool:
        None when its budget cannot hold a new buffer)."""
        nbytes = int(nbytes)
        if nbytes < self.MIN_BYTES and not self.pinned:  # small: malloc's own free lists serve it
            return torch.empty(nbytes, dtype=torch.uint8)
        with self._lock:
            self._drain()
            pick = next((i for i, m in enumerate(self._free) if nbytes <= _nbytes(m) <= 2 * nbytes + self.GRAIN), None)
            mem = self._free.pop(pick) if pick is not None else None
            if mem is None:
                grain = self.GRAIN if nbytes >= self.GRAIN else self.MIN_BYTES
                size = -(-nbytes // grain) * grain
                if self.pinned:
                    while self._free and self.live_bytes + size > self.max_bytes:  # make room: drop free ones
                        self._release(self._free.pop())
                    if self.live_bytes + size > self.max_bytes:
                        return None
                mem = self._np.empty(size, dtype=self._np.uint8)
                if self.pinned:
                    if not _register(mem.ctypes.data, size):
                        return None
                    self.live_bytes += size
        return torch.from_numpy(self._np.asarray(_HostLease(mem, nbytes, self)))

    def free_bytes(self) -> int:
        with self._lock:
            self._drain()
            return sum(_nbytes(m) for m in self._free)


HOST_ARENAS = HostArenaPool()
# page-locked arenas: off unless OMF_PIN_HOST_ARENAS / set_pinned_arenas gives them a budget
PINNED_ARENAS = HostArenaPool(max_bytes=_pin_budget_from_env(), pinned=True)


def set_pinned_arenas(max_bytes: int) -> None:
    """Budget of page-locked decoded arenas (0 = off, the default): the CPU
    placement's results then land by one DMA each instead of through the pinned chunk ring."""
    PINNED_ARENAS.set_max_bytes(max(0, int(max_bytes)))


def pinned_arena(nbytes: int) -> Optional[torch.Tensor]:
    """A page-locked pooled arena of ``nbytes`` if the budget allows, else None.  With no budget,
    the buffers of leases handed out before it was removed are unlocked and freed here as they come
    back (their finalisers only queue them)."""
    if PINNED_ARENAS.max_bytes <= 0:
        if PINNED_ARENAS._returned:
            with PINNED_ARENAS._lock:
                PINNED_ARENAS._drain()
        return None
    return PINNED_ARENAS.empty(nbytes)


# 32 MiB chunks x max(4, workers()) slots (256 MiB of staging at 8 copy threads): the pageable CPU
# placement of a Llama-400M QSGD decode took 56.7 / 52.8 / 47.6-54.6 / 45.8 ms at 8 / 16 / 32 / 64 MiB
# chunks on one box (scripts/exp/host_decode_sweep.py; fewer, larger chunks cost the feeder thread
# fewer Python round trips), 16 slots no better than 8.
RING_CHUNK_BYTES = 32 << 20


class D2HRing:
    """Device-to-host copies into a host destination (``dst_ptr``) through a ring of ``slots``
    pinned chunks of ``limit`` bytes, fed by a thread of its own: ``submit(src, dst_off, after)``
    returns at once; the feeder makes ``stream`` wait for the event ``after`` (work queued on
    another stream), queues each chunk's DMA on ``stream`` once its slot is free and hands the
    landed chunk to a worker thread's memmove.  So a caller can keep queueing host-to-device work
    on its own stream while earlier results flow out (PCIe is full duplex).  ``close()`` (or the
    context's exit) returns when every byte has landed; a failure in the feeder is raised there."""

    def __init__(self, dst_ptr: int, stream, key: str = "d2h", limit: Optional[int] = None,
                 slots: Optional[int] = None):
        import queue

        self.dst, self.stream, self.limit = int(dst_ptr), stream, int(limit or RING_CHUNK_BYTES)
        self.n_slots = slots or max(4, workers())
        self._cm = STAGING.lease(key, self.n_slots * self.limit)
        self._lease = self._cm.__enter__()
        self._base = self._lease.buf.data_ptr()
        self._busy: List[Optional[object]] = [None] * self.n_slots
        self._g = 0
        self._q = queue.Queue()
        self._err: Optional[BaseException] = None
        self._t = threading.Thread(target=self._feed, name="omf-d2h", daemon=True)
        self._t.start()

    @staticmethod
    def _land(ev, d, s, n):
        ev.synchronize()
        ctypes.memmove(d, s, n)

    def _feed(self) -> None:
        ex = pool()
        while True:
            req = self._q.get()
            if req is None:
                break
            if self._err is not None:
                continue
            src, off, after = req
            try:
                with torch.cuda.device(self.stream.device), torch.cuda.stream(self.stream):
                    if after is not None:
                        self.stream.wait_event(after)
                    total = src.numel()
                    for a in range(0, total, self.limit):
                        b = min(a + self.limit, total)
                        s = self._g % self.n_slots
                        self._g += 1
                        if self._busy[s] is not None:
                            self._busy[s].result()  # the slot's previous chunk is out
                        self._lease.buf[s * self.limit:s * self.limit + (b - a)].copy_(src[a:b], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                        self._busy[s] = ex.submit(self._land, ev, self.dst + off + a, self._base + s * self.limit, b - a)
            except BaseException as e:  # reported by close()
                self._err = e

    def submit(self, src: torch.Tensor, dst_off: int, after=None) -> None:
        """Copy the bytes of the device tensor ``src`` (a uint8 view) to ``dst_ptr + dst_off``
        once the event ``after`` (if any) has completed."""
        self._q.put((src, int(dst_off), after))

    def close(self) -> None:
        self._q.put(None)
        self._t.join()
        try:
            for f in self._busy:
                if f is not None:
                    f.result()
        finally:
            self._cm.__exit__(None, None, None)
        if self._err is not None:
            raise self._err

    def __enter__(self) -> "D2HRing":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def device_to_host(src: torch.Tensor, stream=None, key: str = "d2h", limit: Optional[int] = None,
                   slots: Optional[int] = None, pool_memory: bool = True) -> torch.Tensor:
    """A CPU copy of the device tensor ``src`` (1-D, same dtype), queued on ``stream`` (default the
    current stream of ``src``'s device) behind the work already there.  Into a page-locked pooled
    arena when ``set_pinned_arenas`` / ``OMF_PIN_HOST_ARENAS`` gave them a budget that holds it
    (one DMA at the link's rate); otherwise through a ``D2HRing`` (``slots`` pinned chunks of
    ``limit`` bytes) into pageable memory — pooled (``HOST_ARENAS``: the pages reused round after
    round) with ``pool_memory``, else a fresh tensor.  Returns when every byte has landed."""
    if stream is None:
        stream = torch.cuda.current_stream(src.device)
    raw = src.reshape(-1).view(torch.uint8)
    big = raw.numel() >= HostArenaPool.MIN_BYTES
    out = pinned_arena(raw.numel()) if pool_memory and big else None
    if out is not None:  # page-locked: one DMA
        with torch.cuda.stream(stream):
            out.copy_(raw, non_blocking=True)
        stream.synchronize()
        return out.view(src.dtype)
    out = (HOST_ARENAS.empty(raw.numel()) if pool_memory and big else torch.empty(raw.numel(), dtype=torch.uint8))
    out = out.view(src.dtype)
    if raw.numel() == 0:
        return out
    with D2HRing(out.data_ptr(), stream, key, limit, slots) as ring:
        ring.submit(raw, 0)
    return out


def stage_payloads(items: Sequence[Tuple[int, Callable[[], bytes]]], base: int, total_bytes: int,
                   flush: Callable[[int, int], None], limit: int = CHUNK_BYTES,
                   check: Optional[Callable[[int, bytes], None]] = None) -> None:
    """Copy the payloads ``getter()`` of ``items`` = (byte offset from ``base``, getter) —
    ascending offsets, all below ``total_bytes`` — into host memory at ``base``: each payload is
    handed to a worker thread as soon as it is read (protobuf's get-copy, on this thread), and
    once a ~``limit``-byte chunk [a, b) is complete ``flush(a, b)`` runs (the caller queues its
    host-to-device copy) while the next chunk is read.  At most two chunks of payloads are alive
    at a time (their memory is recycled).  ``check(i, payload)`` may raise before item i is
    copied; copies already started are waited for first."""
    ex = pool()
    started: List[object] = []
    prev = None  # (a, b, futures, payloads) of the chunk being copied
    ga, gb, futs, held = -1, 0, [], []

    def close(chunk) -> None:
        a, b, fs, _ = chunk
        for f in fs:
            f.result()
        if b > a:
            flush(a, b)

    try:
        for i, (off, get) in enumerate(items):
            p = get()
            if check is not None:
                check(i, p)
            n = len(p)
            if off + n > total_bytes:
                raise ValueError("payload past the end of the staging arena")
            if ga < 0:
                ga = off
            if futs and off + n - ga > limit:  # this chunk is complete: the previous one goes out
                if prev is not None:
                    close(prev)
                prev, ga, gb, futs, held = (ga, gb, futs, held), off, off, [], []
            if 0 < n < INLINE_BYTES:
                ctypes.memmove(base + off, _bytes_addr(p), n)
            elif n:
                f = ex.submit(ctypes.memmove, base + off, _bytes_addr(p), n)
                futs.append(f)
                started.append(f)
                held.append(p)
            gb = max(gb, off + n)
        if prev is not None:
            close(prev)
            prev = None
        if ga >= 0:
            close((ga, gb, futs, held))
    finally:
        for f in started:
            f.result()


def bytes_to_device(items: Sequence[Tuple[int, Callable[[], bytes]]], dst: torch.Tensor, total_bytes: int,
                    stream=None, key: str = "decode", limit: int = CHUNK_BYTES,
                    check: Optional[Callable[[int, bytes], None]] = None,
                    after_flush: Optional[Callable[[int, int], None]] = None) -> None:
    """``stage_payloads`` into pinned staging (a lease), each chunk's host-to-device copy into the
    device buffer ``dst`` queued on ``stream`` as soon as the chunk is complete, then
    ``after_flush(a, b)`` (optional) with the chunk's byte range.  Returns once the
    last copy is queued (the staging goes back to its pool with an event the next holder waits for)."""
    if stream is None:
        stream = torch.cuda.current_stream(dst.device)
    raw = dst.reshape(-1).view(torch.uint8)
    with STAGING.lease(key, max(int(total_bytes), 1)) as h:
        staged = h.buf

        def flush(a: int, b: int) -> None:
            with torch.cuda.stream(stream):
                raw[a:b].copy_(staged[a:b], non_blocking=True)
            if after_flush is not None:  # e.g. decode what has arrived (queued behind this copy)
                after_flush(a, b)

        try:
            stage_payloads(items, staged.data_ptr(), total_bytes, flush, limit, check)
        finally:
            h.event = torch.cuda.Event()  # the next holder waits for these copies
            h.event.record(stream)
