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

Nothing here changes bytes: the payload is the encoder's, byte for byte.
"""

from __future__ import annotations

import ctypes
import os
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, Iterator, List, Optional, Sequence, Tuple

import torch

CHUNK_BYTES = 32 << 20

_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
_bytes_addr = ctypes.pythonapi.PyBytes_AsString
_bytes_addr.restype = ctypes.c_void_p
_bytes_addr.argtypes = [ctypes.py_object]

_pool: Optional[ThreadPoolExecutor] = None
_pool_lock = threading.Lock()


def workers() -> int:
    """Copy threads: half the CPUs this process may run on, 2..8."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        n = os.cpu_count() or 4
    return max(2, min(8, n // 2))


def pool() -> ThreadPoolExecutor:
    global _pool
    if _pool is None:
        with _pool_lock:
            if _pool is None:
                _pool = ThreadPoolExecutor(max_workers=workers(), thread_name_prefix="omf-wire")
    return _pool


class PinnedStaging:
    """Reusable page-locked host buffers (one per purpose), grown on demand.  A caller finishes
    with a buffer (its copies have landed) before the next call reuses it."""

    def __init__(self):
        self._bufs: Dict[str, torch.Tensor] = {}
        self._lock = threading.Lock()

    def get(self, key: str, nbytes: int) -> torch.Tensor:
        with self._lock:
            b = self._bufs.get(key)
            if b is None or b.numel() < nbytes:
                b = torch.empty(max(int(nbytes), 4096), dtype=torch.uint8, pin_memory=True)
                self._bufs[key] = b
            return b[:nbytes]


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


def device_to_bytes(src: torch.Tensor, spans: Sequence[Tuple[int, int]], stream=None, key: str = "encode",
                    limit: int = CHUNK_BYTES) -> Iterator[Tuple[int, bytes]]:
    """Yield ``(i, bytes)`` for every span i = (byte offset, length) of the device buffer ``src``
    (ascending offsets; length 0 is skipped), in order, each as soon as its bytes are filled.
    The device-to-host copies are queued on ``stream`` (default: the current stream of ``src``'s
    device) behind the work already there."""
    if stream is None:
        stream = torch.cuda.current_stream(src.device)
    raw = src.reshape(-1).view(torch.uint8)
    total = max((off + n for off, n in spans), default=0)
    staged = STAGING.get(key, total)
    groups = _groups(spans, limit)
    events = []
    with torch.cuda.stream(stream):
        for a, b, _ in groups:
            if b > a:
                staged[a:b].copy_(raw[a:b], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            events.append(ev)
    base = staged.data_ptr()
    ex = pool()
    pending: List[Tuple[int, bytes, object]] = []
    for (a, b, idx), ev in zip(groups, events):
        ev.synchronize()
        filled = []
        for i in idx:
            off, n = spans[i]
            if n <= 0:
                continue
            obj = _new_bytes(None, n)
            filled.append((i, obj, ex.submit(ctypes.memmove, _bytes_addr(obj), base + off, n)))
        for i, obj, fut in pending:  # the previous chunk, while this one is copied
            fut.result()
            yield i, obj
        pending = filled
    for i, obj, fut in pending:
        fut.result()
        yield i, obj


def bytes_to_device(items: Sequence[Tuple[int, Callable[[], bytes]]], dst: torch.Tensor, total_bytes: int,
                    stream=None, key: str = "decode", limit: int = CHUNK_BYTES,
                    check: Optional[Callable[[int, bytes], None]] = None) -> None:
    """Copy the payloads ``getter()`` of ``items`` = (byte offset in ``dst``, getter) — ascending
    offsets, all below ``total_bytes`` — into the device buffer ``dst`` through pinned staging:
    each payload is handed to a worker thread as soon as it is read, and every ~``limit``-byte
    chunk goes host-to-device (queued on ``stream``) while the next chunk's payloads are read.
    ``check(i, payload)`` may raise before item i is copied (copies already started are waited
    for first).  Returns once the last copy is queued; the caller synchronises the stream before
    the staging is reused (the next call)."""
    if stream is None:
        stream = torch.cuda.current_stream(dst.device)
    raw = dst.reshape(-1).view(torch.uint8)
    staged = STAGING.get(key, max(int(total_bytes), 1))
    base = staged.data_ptr()
    ex = pool()
    keep: List[bytes] = []  # alive until their copies are done
    every: List[object] = []

    def flush(a: int, b: int, futs: List[object]) -> None:
        for f in futs:
            f.result()
        if b > a:
            with torch.cuda.stream(stream):
                raw[a:b].copy_(staged[a:b], non_blocking=True)

    prev = None
    ga, gb, futs = -1, 0, []
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
            if futs and off + n - ga > limit:  # close the chunk: copy the previous one to the GPU
                if prev is not None:
                    flush(*prev)
                prev, ga, futs = (ga, gb, futs), off, []
            if n:
                f = ex.submit(ctypes.memmove, base + off, _bytes_addr(p), n)
                futs.append(f)
                every.append(f)
                keep.append(p)
            gb = max(gb, off + n)
        if prev is not None:
            flush(*prev)
        if ga >= 0:
            flush(ga, gb, futs)
    finally:
        for f in every:
            f.result()
