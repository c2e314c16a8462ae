"""Device codec: the Python face of ``libomf_codec.so`` over torch device tensors.

An *update arena* is one fp32 device buffer holding every named tensor of a
client, tensor t at ``[offsets[t], offsets[t] + sizes[t])`` (``arena_layout``
pads every start to a multiple of 64 elements = 256 B).  All kernels process a
whole arena per launch; payload arenas (int8/int32 levels, decoded fp32) share
the element offsets.  Every function validates shapes, dtypes, devices and
alignment on the host before anything is launched: a kernel never sees a
buffer shorter than the plan assumes.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ._lib import CodecError, check, lib  # noqa: F401  (CodecError: raised by check())

ALIGN_ELEMS = 64


def arena_layout(sizes: Sequence[int], align: int = ALIGN_ELEMS) -> Tuple[List[int], int]:
    """Offsets (multiples of ``align``) and total length of an arena holding ``sizes``."""
    offs, cur = [], 0
    for n in sizes:
        offs.append(cur)
        cur += (int(n) + align - 1) // align * align
    return offs, max(cur, align)


def storage_width(levels: int) -> int:
    """qsgd.py:18-21: payload bits per element (8 while levels <= 127, else 32)."""
    return 8 if levels <= 127 else 32


def packed_bits(levels: int) -> int:
    """Bits per element of the opt-in packed wire: ceil(log2(2 L + 1)) (omf_qsgd_packed_bits)."""
    levels = int(levels)
    if levels <= 0 or levels >= 2**31 - 1:
        raise ValueError(f"invalid level={levels}")
    return (2 * levels).bit_length()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device: torch.device) -> int:
    """The current stream's handle (the raw getter: ~0.1 us per call against ~2 us for
    ``torch.cuda.current_stream(device).cuda_stream``, which builds a Stream object)."""
    if _raw_stream is not None:
        return _raw_stream(device.index)
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _need(t: torch.Tensor, name: str, dtype, device, numel: int, align: int):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.numel() < numel:
        raise ValueError(f"{name}: {t.numel()} elements, plan needs {numel}")
    if t.data_ptr() % align:
        raise ValueError(f"{name} must be {align}-byte aligned")


# encoder strategies by omf_plan_set_encode_strategy code (include/omf_codec.h)
STRATEGIES = ("resident", "ordered", "ring", "bracket", "grid")


DECODE_BLOCK = 4096  # elements per decode block (omf_qsgd_decode_range granularity)


class Plan:
    """An ``omf_plan`` over fixed tensor sizes/offsets on one device (cached, reusable)."""

    _cache: Dict[tuple, "Plan"] = {}
    _cache_lock = threading.Lock()

    def __init__(self, sizes: Sequence[int], offsets: Optional[Sequence[int]] = None,
                 device: Optional[torch.device] = None, chunk: int = 0):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("the codec runs on a GPU device")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.sizes = [int(n) for n in sizes]
        if offsets is None:
            offsets, _ = arena_layout(self.sizes)
        self.offsets = [int(o) for o in offsets]
        if len(self.sizes) != len(self.offsets) or not self.sizes:
            raise ValueError("sizes and offsets must be non-empty and of equal length")
        self.nt = len(self.sizes)
        self.device = device
        self.chunk = int(chunk)
        self.arena_end = self.offsets[-1] + self.sizes[-1]
        L = lib()
        n = self.nt
        szs = (ctypes.c_int64 * n)(*self.sizes)
        ofs = (ctypes.c_int64 * n)(*self.offsets)
        h = ctypes.c_void_p()
        check(L.omf_plan_create(szs, ofs, n, self.chunk, device.index, ctypes.byref(h)), "omf_plan_create")
        self._h = h
        self._lock = threading.Lock()
        self._topk_ws: Dict[int, torch.Tensor] = {}  # per stream: launches on two streams never share one
        self._dec_ws: Dict[int, torch.Tensor] = {}   # tiled Top-K decode workspace, per stream
        self._dec_need: Dict[float, int] = {}
        self._counts_cache: Dict[tuple, tuple] = {}
        self._topk_cache: Dict[float, tuple] = {}
        self.topk_reordered = 0  # tensors the latest tie_order="torch" encode rewrote (diagnostics)
        # the library's choice (by arena size, or OMF_ENCODE_STRATEGY)
        self.strategy = STRATEGIES[int(L.omf_plan_encode_strategy(h))]

    @classmethod
    def get(cls, sizes, offsets=None, device=None, chunk: int = 0) -> "Plan":
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if offsets is None:
            offsets, _ = arena_layout(sizes)
        key = (tuple(int(s) for s in sizes), tuple(int(o) for o in offsets), str(device), int(chunk))
        with cls._cache_lock:
            p = cls._cache.get(key)
            if p is None:
                p = cls(sizes, offsets, device, chunk)
                cls._cache[key] = p
            return p

    @property
    def handle(self):
        return self._h

    def payload_elems(self, width: int) -> int:
        """Elements a payload arena must hold: an int8 payload is stored in whole dwords, so the
        last tensor's partial dword may be written (as zero levels) up to ``arena_end`` rounded
        up to 4 (include/omf_codec.h, data layout)."""
        return self.arena_end if int(width) == 32 else (self.arena_end + 3) & ~3

    @property
    def encode_items(self) -> int:
        return int(lib().omf_plan_encode_items(self._h))

    def check(self, stream: Optional[int] = None) -> bool:
        """Synchronise; raise ``CodecError`` (a ``RuntimeError``) on an in-kernel timeout (the
        payload of that launch is invalid).  Returns False if an encoder had to recompute a
        norm (results exact, but the grid was not co-resident).  Every product entry point
        calls it at the synchronisation it already makes."""
        with self._lock:  # the plan's host state (its last stream, the flags it clears) is shared by threads
            rc = lib().omf_plan_check(self._h, ctypes.c_void_p(stream if stream is not None else _stream(self.device)))
        if rc == 1:
            return False
        check(rc, "omf_plan_check")
        return True

    def set_topk(self, groups: int = -1, fallback: int = -1, sample_runs: int = -1, sure=None) -> None:
        """Test / experiment hook of the Top-K encoder (omf_plan_set_topk): the group pipeline,
        the forced fallback (1: the exact tail's radix sort; 2: the same with a forced barrier
        expiry, the test of its bound), the sample size (0 = default), the sure margin (z, c).
        None of them changes the selection (fallback 2 invalidates it and makes ``check`` raise);
        -1 / None keeps a setting."""
        z, c = (-1.0, -1.0) if sure is None else (float(sure[0]), float(sure[1]))
        with self._lock:
            check(lib().omf_plan_set_topk(self._h, int(groups), int(fallback), int(sample_runs), z, c),
                  "omf_plan_set_topk")

    def topk_stats(self, reset: bool = False) -> dict:
        """The plan's Top-K encoder counters (omf_topk_stats): sampled-path calls, bucket-sort fast
        path, zero fills (tensors completed with their lowest-index zeros), radix-sort fallbacks,
        exact redos, exact-path calls."""
        out = (ctypes.c_int64 * 6)()
        with self._lock:
            check(lib().omf_topk_stats(self._h, out, 1 if reset else 0), "omf_topk_stats")
        return dict(zip(("calls", "fast", "zero_fill", "fallback", "redo", "exact"), (int(v) for v in out)))

    def set_debug(self, ring: int = 0, spec: int = 0, lds_wait_us: int = 0) -> None:
        """Test / experiment hook (omf_plan_set_debug): switches that change what an encode
        writes (never set in production); all zero restores the production behaviour."""
        check(lib().omf_plan_set_debug(self._h, int(ring), int(spec), int(lds_wait_us)), "omf_plan_set_debug")

    @property
    def resident_capacity(self) -> int:
        return int(lib().omf_plan_resident_capacity(self._h))

    def set_resident_capacity(self, cap: int = 0, wait_us: int = 0) -> None:
        """Tuning / test hook: see omf_plan_set_resident_capacity."""
        check(lib().omf_plan_set_resident_capacity(self._h, int(cap), int(wait_us)), "omf_plan_set_resident_capacity")

    def set_encode_strategy(self, strategy: str) -> None:
        """'grid' (one-launch encoder of small arenas: registers + one grid-wide barrier), 'bracket'
        (bracketed single-read encoder), 'ring' (single-read ring encoder), 'ordered' (two-pass
        everywhere) or 'resident' (register-resident small tensors + two-pass)."""
        code = STRATEGIES.index(strategy)
        check(lib().omf_plan_set_encode_strategy(self._h, code), "omf_plan_set_encode_strategy")
        self.strategy = strategy

    def set_wide_levels(self, on: bool) -> None:
        """Bit widths 5-8 (fp32) through the bracketed encoder (True, the default) or the ring /
        two-pass encoders (omf_plan_set_wide_levels); identical payloads."""
        with self._lock:
            check(lib().omf_plan_set_wide_levels(self._h, 1 if on else 0), "omf_plan_set_wide_levels")

    def set_fused_bracket(self, on: bool) -> None:
        """The bracketed encoder's bracket folded into its pass (omf_plan_set_fused_bracket: bit
        widths 1-4, and 5-8 with wide levels); identical payloads."""
        with self._lock:
            check(lib().omf_plan_set_fused_bracket(self._h, 1 if on else 0), "omf_plan_set_fused_bracket")

    @property
    def last_encoder(self) -> str:
        """The encoder the latest encode launched (omf_plan_last_encoder): one of STRATEGIES,
        "norm_in" (levels with caller norms) or "none"."""
        code = int(lib().omf_plan_last_encoder(self._h))
        return STRATEGIES[code] if 0 <= code < len(STRATEGIES) else ("norm_in" if code == 5 else "none")

    @property
    def encoder_kernel(self) -> str:
        """Name of the kernel one encode launch runs (profiling / roofline bookkeeping)."""
        return self.encoder_kernel_for(4)

    @property
    def last_encoder_kernel(self) -> str:
        """The kernel name (or "qsgd_spec_all" for the bracketed encoder's three launches) of the
        latest encode — what a profile of it shows."""
        return {"bracket": "qsgd_spec_all", "ring": "qsgd_encode_pc", "grid": "qsgd_encode_grid",
                "norm_in": "qsgd_quant_sub"}.get(self.last_encoder, "qsgd_encode_ordered")

    def encoder_kernel_for(self, bit_width: int) -> str:
        """The kernel an fp32, on-device-draw encode at ``bit_width`` runs by default: the bracketed
        encoder (three launches: "qsgd_spec_all") serves bit widths 1-8 (5-8 with its wide-level
        list, omf_plan_set_wide_levels), wider int32 payloads take the ring (omf_plan_encode_strategy).
        ``last_encoder_kernel`` reports what a call actually launched."""
        if self.strategy == "bracket" and not 1 <= int(bit_width) <= 8:
            return "qsgd_encode_pc" if storage_width(2 ** int(bit_width)) == 32 else "qsgd_encode_ordered"
        return {"ring": "qsgd_encode_pc", "bracket": "qsgd_spec_all", "grid": "qsgd_encode_grid"}.get(
            self.strategy, "qsgd_encode_ordered")

    def set_ring(self, cfg: int = -1, big_mode: int = -1, gap: int = -2, hold_max: int = -1) -> None:
        """Tuning / test hook of the ring encoder: see omf_plan_set_ring."""
        check(lib().omf_plan_set_ring(self._h, int(cfg), int(big_mode), int(gap), int(hold_max)), "omf_plan_set_ring")

    def ring_profile(self) -> List[int]:
        """Experiment hook: per-phase cycle totals (set_debug ring bit 4), read and reset."""
        out = (ctypes.c_int64 * 16)()
        check(lib().omf_plan_ring_profile(self._h, out), "omf_plan_ring_profile")
        return [int(v) for v in out]

    def spec_stats(self, stream: Optional[int] = None) -> Dict[str, int]:
        """Diagnostics of the last bracketed encode (omf_plan_spec_stats; synchronises)."""
        out = (ctypes.c_int64 * 4)()
        st = stream if stream is not None else _stream(self.device)
        with self._lock:
            check(lib().omf_plan_spec_stats(self._h, ctypes.c_void_p(st), out), "omf_plan_spec_stats")
        return dict(zip(("whole", "deferred", "listed", "full_slots"), (int(v) for v in out)))

    @property
    def ring_info(self) -> Dict[str, int]:
        out = (ctypes.c_int64 * 6)()
        check(lib().omf_plan_ring_info(self._h, out), "omf_plan_ring_info")
        keys = ("grid", "chunk", "items", "hold_max", "two_pass_tensors", "cfg")
        return dict(zip(keys, (int(v) for v in out)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().omf_plan_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------ QSGD
    def qsgd_encode(self, x: torch.Tensor, bit_width: int, q_out: Optional[torch.Tensor] = None,
                    norm_out: Optional[torch.Tensor] = None, alpha: float = 1.0,
                    u: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0,
                    norm_in: Optional[torch.Tensor] = None, stream: Optional[int] = None, value_format: int = 0):
        """Encode the whole arena ``x``; returns ``(q, norms)`` (device tensors).

        ``value_format``: 0 fp32, 1 bf16, 2 fp16 — the dtype the tensors had (x holds their exact
        fp32 upcast; omf_qsgd_encode_ex rounds where the reference's reduced-precision ops do)."""
        s = int(bit_width)
        if not 0 <= s <= 30:
            raise ValueError("bit_width must be in [0, 30]")
        width = storage_width(2 ** s)
        qdt = torch.int8 if width == 8 else torch.int32
        dev = self.device
        _need(x, "x", torch.float32, dev, self.arena_end, 16)
        if q_out is None:
            q_out = torch.empty(self.payload_elems(width), dtype=qdt, device=dev)
        _need(q_out, "q_out", qdt, dev, self.payload_elems(width), 4 if width == 8 else 16)
        if norm_out is None:
            norm_out = torch.empty(self.nt, dtype=torch.float32, device=dev)
        _need(norm_out, "norm_out", torch.float32, dev, self.nt, 4)
        if u is not None:
            _need(u, "u", torch.float32, dev, self.arena_end, 16)
        if norm_in is not None:
            _need(norm_in, "norm_in", torch.float32, dev, self.nt, 4)
        st = stream if stream is not None else _stream(dev)
        with self._lock:
            check(lib().omf_qsgd_encode_ex(self._h, _ptr(x), float(alpha), s, int(value_format), _ptr(u),
                                           int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset) & 0xFFFFFFFFFFFFFFFF,
                                           _ptr(norm_in), _ptr(q_out), _ptr(norm_out), ctypes.c_void_p(st)),
                  "omf_qsgd_encode_ex")
        return q_out, norm_out

    def ps_apply_encode(self, acc: torch.Tensor, divisor: float, bit_width: int,
                        avg_out: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None, seed: int = 0,
                        offset: int = 0, q_out: Optional[torch.Tensor] = None,
                        norm_out: Optional[torch.Tensor] = None, stream: Optional[int] = None):
        """Fused PS step (omf_ps_apply_encode): ``avg = acc / divisor`` and its QSGD payload.

        Returns ``(avg, q, norms)``; ``avg_out`` may be ``acc`` itself (in place).
        """
        s = int(bit_width)
        if not 0 <= s <= 30:
            raise ValueError("bit_width must be in [0, 30]")
        if not float(divisor) != 0.0:
            raise ValueError("divisor must be non-zero")
        width = storage_width(2 ** s)
        qdt = torch.int8 if width == 8 else torch.int32
        dev = self.device
        _need(acc, "acc", torch.float32, dev, self.arena_end, 16)
        if avg_out is None:
            avg_out = torch.empty(self.arena_end, dtype=torch.float32, device=dev)
        _need(avg_out, "avg_out", torch.float32, dev, self.arena_end, 16)
        if q_out is None:
            q_out = torch.empty(self.payload_elems(width), dtype=qdt, device=dev)
        _need(q_out, "q_out", qdt, dev, self.payload_elems(width), 4 if width == 8 else 16)
        if norm_out is None:
            norm_out = torch.empty(self.nt, dtype=torch.float32, device=dev)
        _need(norm_out, "norm_out", torch.float32, dev, self.nt, 4)
        if u is not None:
            _need(u, "u", torch.float32, dev, self.arena_end, 16)
        st = stream if stream is not None else _stream(dev)
        with self._lock:
            check(lib().omf_ps_apply_encode(self._h, _ptr(acc), float(divisor), _ptr(avg_out), s, _ptr(u),
                                            int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset) & 0xFFFFFFFFFFFFFFFF,
                                            _ptr(q_out), _ptr(norm_out), ctypes.c_void_p(st)),
                  "omf_ps_apply_encode")
        return avg_out, q_out, norm_out

    def ps_accumulate_apply_encode(self, acc: torch.Tensor, q_in: torch.Tensor, width_in: int, levels_in: int,
                                   norm_in: torch.Tensor, divisor: float, bit_width: int,
                                   acc_out: Optional[torch.Tensor] = None, avg_out: Optional[torch.Tensor] = None,
                                   u: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0,
                                   q_out: Optional[torch.Tensor] = None, norm_out: Optional[torch.Tensor] = None,
                                   stream: Optional[int] = None):
        """The PS round's last step (omf_ps_accumulate_apply_encode): ``sum = acc + decode(q_in)`` (the
        last client's payload), ``avg = sum / divisor`` and its QSGD payload, acc and q_in read once.
        ``acc_out``: where ``sum`` is stored (``acc`` itself, another arena, or None: not stored).
        Returns ``(avg, q, norms)``."""
        s = int(bit_width)
        if not 0 <= s <= 30:
            raise ValueError("bit_width must be in [0, 30]")
        if not float(divisor) != 0.0:
            raise ValueError("divisor must be non-zero")
        width = storage_width(2 ** s)
        qdt = torch.int8 if width == 8 else torch.int32
        dev = self.device
        wi = int(width_in)
        _need(acc, "acc", torch.float32, dev, self.arena_end, 16)
        _need(q_in, "q_in", torch.int8 if wi == 8 else torch.int32, dev, self.arena_end, 4 if wi == 8 else 16)
        _need(norm_in, "norm_in", torch.float32, dev, self.nt, 4)
        if acc_out is not None:
            _need(acc_out, "acc_out", torch.float32, dev, self.arena_end, 16)
        if avg_out is None:
            avg_out = torch.empty(self.arena_end, dtype=torch.float32, device=dev)
        _need(avg_out, "avg_out", torch.float32, dev, self.arena_end, 16)
        if q_out is None:
            q_out = torch.empty(self.payload_elems(width), dtype=qdt, device=dev)
        _need(q_out, "q_out", qdt, dev, self.payload_elems(width), 4 if width == 8 else 16)
        if norm_out is None:
            norm_out = torch.empty(self.nt, dtype=torch.float32, device=dev)
        _need(norm_out, "norm_out", torch.float32, dev, self.nt, 4)
        if u is not None:
            _need(u, "u", torch.float32, dev, self.arena_end, 16)
        st = stream if stream is not None else _stream(dev)
        with self._lock:
            check(lib().omf_ps_accumulate_apply_encode(
                self._h, _ptr(acc), _ptr(q_in), wi, int(levels_in), _ptr(norm_in), _ptr(acc_out), float(divisor),
                _ptr(avg_out), s, _ptr(u), int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset) & 0xFFFFFFFFFFFFFFFF,
                _ptr(q_out), _ptr(norm_out), ctypes.c_void_p(st)), "omf_ps_accumulate_apply_encode")
        return avg_out, q_out, norm_out

    def qsgd_norms(self, x: torch.Tensor, alpha: float = 1.0, norm_out: Optional[torch.Tensor] = None,
                   stream: Optional[int] = None, value_format: int = 0) -> torch.Tensor:
        dev = self.device
        _need(x, "x", torch.float32, dev, self.arena_end, 16)
        if norm_out is None:
            norm_out = torch.empty(self.nt, dtype=torch.float32, device=dev)
        _need(norm_out, "norm_out", torch.float32, dev, self.nt, 4)
        st = stream if stream is not None else _stream(dev)
        with self._lock:
            check(lib().omf_qsgd_norms_ex(self._h, _ptr(x), float(alpha), int(value_format), _ptr(norm_out),
                                          ctypes.c_void_p(st)), "omf_qsgd_norms_ex")
        return norm_out

    def qsgd_decode(self, q: torch.Tensor, width: int, levels: int, norm: torch.Tensor,
                    y_out: Optional[torch.Tensor] = None, accumulate: bool = False,
                    stream: Optional[int] = None, elems: Optional[Tuple[int, int]] = None) -> torch.Tensor:
        """omf_qsgd_decode; ``elems=(begin, end)``: omf_qsgd_decode_range (only the decode blocks
        of ``DECODE_BLOCK`` elements overlapping that arena range are decoded)."""
        width, levels = int(width), int(levels)
        if width not in (8, 32):
            raise ValueError(f"unsupported width={width}")
        if levels <= 0:
            raise ValueError(f"invalid level={levels}")
        dev = self.device
        qdt = torch.int8 if width == 8 else torch.int32
        _need(q, "q", qdt, dev, self.arena_end, 4 if width == 8 else 16)
        _need(norm, "norm", torch.float32, dev, self.nt, 4)
        if y_out is None:
            if accumulate:
                raise ValueError("accumulate=True needs y_out")
            y_out = torch.empty(self.arena_end, dtype=torch.float32, device=dev)
        _need(y_out, "y_out", torch.float32, dev, self.arena_end, 16)
        st = stream if stream is not None else _stream(dev)
        if elems is not None:
            check(lib().omf_qsgd_decode_range(self._h, _ptr(q), width, levels, _ptr(norm), _ptr(y_out),
                                              1 if accumulate else 0, int(elems[0]), int(elems[1]),
                                              ctypes.c_void_p(st)), "omf_qsgd_decode_range")
            return y_out
        check(lib().omf_qsgd_decode(self._h, _ptr(q), width, levels, _ptr(norm), _ptr(y_out),
                                    1 if accumulate else 0, ctypes.c_void_p(st)), "omf_qsgd_decode")
        return y_out

    # ------------------------------------------------------------ bit-packed wire (opt-in)
    def packed_words(self, levels: int) -> int:
        """32-bit words of the packed arena: ceil(arena_end / 32) groups of 32 elements, b words
        each (tensor t at word ``offsets[t] * b // 32``; the last tensor's partial group too)."""
        return -(-self.arena_end // 32) * packed_bits(levels)

    def qsgd_pack(self, q: torch.Tensor, width: int, levels: int, packed_out: Optional[torch.Tensor] = None,
                  stream: Optional[int] = None) -> torch.Tensor:
        """Levels (int8/int32 payload arena) -> codes ``q + L`` in ``packed_bits(L)`` bits (an int32
        tensor holding the packed words)."""
        width, levels = int(width), int(levels)
        if width not in (8, 32):
            raise ValueError(f"unsupported width={width}")
        dev = self.device
        _need(q, "q", torch.int8 if width == 8 else torch.int32, dev, self.arena_end, 16)
        words = self.packed_words(levels)
        if packed_out is None:
            packed_out = torch.empty(max(words, 1), dtype=torch.int32, device=dev)
        _need(packed_out, "packed_out", torch.int32, dev, words, 8)  # 8-byte word-pair stores
        st = stream if stream is not None else _stream(dev)
        check(lib().omf_qsgd_pack(self._h, _ptr(q), width, levels, _ptr(packed_out), ctypes.c_void_p(st)),
              "omf_qsgd_pack")
        return packed_out

    def qsgd_decode_packed(self, packed: torch.Tensor, levels: int, norm: torch.Tensor,
                           y_out: Optional[torch.Tensor] = None, accumulate: bool = False,
                           stream: Optional[int] = None) -> torch.Tensor:
        levels = int(levels)
        dev = self.device
        _need(packed, "packed", torch.int32, dev, self.packed_words(levels), 4)
        _need(norm, "norm", torch.float32, dev, self.nt, 4)
        if y_out is None:
            if accumulate:
                raise ValueError("accumulate=True needs y_out")
            y_out = torch.empty(self.arena_end, dtype=torch.float32, device=dev)
        _need(y_out, "y_out", torch.float32, dev, self.arena_end, 16)
        st = stream if stream is not None else _stream(dev)
        check(lib().omf_qsgd_decode_packed(self._h, _ptr(packed), levels, _ptr(norm), _ptr(y_out),
                                           1 if accumulate else 0, ctypes.c_void_p(st)), "omf_qsgd_decode_packed")
        return y_out

    # ------------------------------------------------------------ Top-K
    def topk_ks(self, ratio: float) -> List[int]:
        return list(self._topk_geom(ratio)[0])

    def _topk_geom(self, ratio: float):
        """(ks, K, workspace bytes) of one ratio, cached: the per-call host path stays short
        (the library's sizing runs once per ratio, not once per tensor per call)."""
        key = float(ratio)
        g = self._topk_cache.get(key)
        if g is None:
            L = lib()
            ks = tuple(int(L.omf_topk_k(n, key)) for n in self.sizes)
            for n, k in zip(self.sizes, ks):
                if k > n:
                    raise ValueError("selected index k out of range: compress_ratio too large")
            g = (ks, sum(ks), int(L.omf_topk_workspace_bytes(self._h, key)))
            self._topk_cache[key] = g
        return g

    def topk_encode(self, x: torch.Tensor, ratio: float, residual: Optional[torch.Tensor] = None,
                    residual_mode: int = 0, values: Optional[torch.Tensor] = None,
                    indices: Optional[torch.Tensor] = None, stream: Optional[int] = None, alpha: float = 1.0,
                    tie_order: str = "index"):
        """Returns ``(values, indices, ks)``; tensor t's selection at ``[sum(ks[:t]), +ks[t])``.

        ``alpha``: the client weighting (t' = residual + fl32(alpha * x)), fused in.
        ``tie_order``: "index" — the device selection alone, (|t'| descending, index ascending),
        asynchronous on the stream (the fallback too: ``omf_plan_check`` reports an exact-tail
        barrier expiry, never expected); "torch" — then ``omf_topk_torch_order``: where magnitudes
        tie, which of them are selected and their order are torch's CPU ``topk`` (the reference's
        bytes; synchronises the stream, then checks the plan).  Without ties the two are the same
        bytes."""
        if tie_order not in ("index", "torch"):
            raise ValueError(f"tie_order must be 'index' or 'torch', not {tie_order!r}")
        dev = self.device
        ks, K, need = self._topk_geom(ratio)
        ks = list(ks)
        _need(x, "x", torch.float32, dev, self.arena_end, 16)
        if residual_mode not in (0, 1, 2):
            raise ValueError("residual_mode must be 0, 1 or 2")
        if residual_mode:
            if residual is None:
                raise ValueError("residual_mode != 0 needs a residual buffer")
            _need(residual, "residual", torch.float32, dev, self.arena_end, 16)
        if values is None:
            values = torch.empty(K, dtype=torch.float32, device=dev)
        if indices is None:
            indices = torch.empty(K, dtype=torch.int64, device=dev)
        _need(values, "values", torch.float32, dev, K, 4)
        _need(indices, "indices", torch.int64, dev, K, 8)
        L = lib()
        st = stream if stream is not None else _stream(dev)
        with self._lock:
            ws = self._topk_ws.get(st)
            if ws is None or ws.numel() < need:
                ws = torch.empty(need, dtype=torch.uint8, device=dev)
                self._topk_ws[st] = ws
            check(L.omf_topk_encode(self._h, _ptr(x), _ptr(residual) if residual_mode else None, int(residual_mode),
                                    float(ratio), float(alpha), _ptr(values), _ptr(indices), _ptr(ws),
                                    ctypes.c_size_t(ws.numel()), ctypes.c_void_p(st)),
                  "omf_topk_encode")
            if tie_order == "torch":
                nre = ctypes.c_int64(0)
                check(L.omf_topk_torch_order(self._h, _ptr(x), _ptr(residual) if residual_mode else None,
                                             int(residual_mode), float(ratio), float(alpha), _ptr(values),
                                             _ptr(indices), _ptr(ws), ctypes.c_size_t(ws.numel()),
                                             ctypes.c_void_p(st), ctypes.byref(nre)),
                      "omf_topk_torch_order")
                self.topk_reordered = int(nre.value)
        if tie_order == "torch":  # (the stream is synchronised already) an exact-tail barrier expiry raises
            self.check(st)
        return values, indices, ks


    def topk_decode_arena(self, values: torch.Tensor, indices: torch.Tensor, ratio: float,
                          y: Optional[torch.Tensor] = None, mode: int = 0, stream: Optional[int] = None) -> torch.Tensor:
        """Decode one client's whole Top-K selection (topk_encode's packed layout at ``ratio``)
        into the arena ``y``: mode 0 zeros + set, 1 overlay, 2 scatter-add (one launch)."""
        dev = self.device
        K = self._topk_geom(ratio)[1]
        _need(values, "values", torch.float32, dev, K, 4)
        _need(indices, "indices", torch.int64, dev, K, 8)
        if mode not in (0, 1, 2):
            raise ValueError("mode must be 0, 1 or 2")
        if y is None:
            if mode != 0:
                raise ValueError("mode 1/2 need y")
            y = torch.empty(self.arena_end, dtype=torch.float32, device=dev)
        _need(y, "y", torch.float32, dev, self.arena_end, 4)
        st = stream if stream is not None else _stream(dev)
        L = lib()
        if mode == 0 and y.data_ptr() % 16 == 0:  # one streaming write of the arena (tiled decode)
            key = float(ratio)
            need = self._dec_need.get(key)
            if need is None:
                need = self._dec_need[key] = int(L.omf_topk_decode_workspace_bytes(self._h, key))
            with self._lock:
                ws = self._dec_workspace(st, need)
                rc = L.omf_topk_decode_arena_ws(self._h, float(ratio), _ptr(values), _ptr(indices), _ptr(y), 0,
                                                _ptr(ws), ctypes.c_size_t(ws.numel()), ctypes.c_void_p(st))
                if rc != 0:
                    self._dec_ws.pop(st, None)  # its counters may be left non-zero: start afresh
                check(rc, "omf_topk_decode_arena_ws")
            return y
        with self._lock:
            check(L.omf_topk_decode_arena(self._h, float(ratio), _ptr(values), _ptr(indices), _ptr(y), int(mode),
                                          ctypes.c_void_p(st)), "omf_topk_decode_arena")
        return y

    def _dec_workspace(self, st: int, need: int) -> torch.Tensor:
        """The tiled decode's workspace of stream ``st`` (caller holds ``self._lock``): zero-filled
        once (every call leaves its counters zero), the fill ordered before its first use on ``st``."""
        ws = self._dec_ws.get(st)
        if ws is None or ws.numel() < need:
            ws = torch.zeros(max(need, 256), dtype=torch.uint8, device=self.device)
            torch.cuda.current_stream(self.device).synchronize()  # the fill ran on the current stream
            self._dec_ws[st] = ws
        return ws

    def _counts(self, counts: Sequence[int]):
        """(ctypes int64 array, total) of a per-tensor count vector (cached: a message layout
        repeats every round)."""
        key = tuple(int(c) for c in counts)
        with self._lock:  # plans are shared by threads (gRPC workers, a client and the PS)
            c = self._counts_cache.get(key)
        if c is None:
            if len(key) != self.nt:
                raise ValueError(f"counts: {len(key)} entries, plan has {self.nt} tensors")
            arr = (ctypes.c_int64 * self.nt)(*key)
            need = int(lib().omf_topk_decode_counts_workspace_bytes(self._h, arr))
            if need == 0:
                raise ValueError("counts must satisfy 0 <= counts[t] <= sizes[t]")
            c = (arr, sum(key), need)
            with self._lock:
                while len(self._counts_cache) >= 16:
                    self._counts_cache.pop(next(iter(self._counts_cache)))
                self._counts_cache[key] = c
        return c

    def topk_check_indices(self, counts: Sequence[int], indices: torch.Tensor,
                           stream: Optional[int] = None) -> torch.Tensor:
        """omf_topk_check_indices: wrap indices in [-n_t, 0) in place (numpy's negative indexing of the
        reference decoder) and return a device int32 holding the lowest tensor with an index outside
        [-n_t, n_t) (>= nt when there is none).  Asynchronous."""
        arr, ktot, _ = self._counts(counts)
        dev = self.device
        _need(indices, "indices", torch.int64, dev, ktot, 8)
        bad = torch.empty(1, dtype=torch.int32, device=dev)
        st = stream if stream is not None else _stream(dev)
        with self._lock:
            check(lib().omf_topk_check_indices(self._h, arr, _ptr(indices), _ptr(bad), ctypes.c_void_p(st)),
                  "omf_topk_check_indices")
        return bad

    def topk_check_duplicates(self, counts: Sequence[int], indices: torch.Tensor,
                              stream: Optional[int] = None) -> torch.Tensor:
        """omf_topk_check_duplicates: a device int32 per tensor, 1 where an (in-range) index of the
        message repeats (run after ``topk_check_indices``).  Asynchronous."""
        arr, ktot, _ = self._counts(counts)
        dev = self.device
        _need(indices, "indices", torch.int64, dev, ktot, 8)
        flags = torch.empty(self.nt, dtype=torch.int32, device=dev)
        st = stream if stream is not None else _stream(dev)
        with self._lock:
            check(lib().omf_topk_check_duplicates(self._h, arr, _ptr(indices), _ptr(flags), ctypes.c_void_p(st)),
                  "omf_topk_check_duplicates")
        return flags

    def topk_decode_counts(self, counts: Sequence[int], values: torch.Tensor, indices: torch.Tensor,
                           y: Optional[torch.Tensor] = None, mode: int = 0, stream: Optional[int] = None) -> torch.Tensor:
        """Decode one received message's Top-K selection (per-tensor sizes ``counts``, packed in plan
        order) into the arena ``y``: mode 0 zeros + set (tiled), 1 overlay, 2 scatter-add; one call."""
        arr, ktot, need = self._counts(counts)
        dev = self.device
        _need(values, "values", torch.float32, dev, ktot, 4)
        _need(indices, "indices", torch.int64, dev, ktot, 8)
        if mode not in (0, 1, 2):
            raise ValueError("mode must be 0, 1 or 2")
        if y is None:
            if mode != 0:
                raise ValueError("mode 1/2 need y")
            y = torch.empty(self.arena_end, dtype=torch.float32, device=dev)
        _need(y, "y", torch.float32, dev, self.arena_end, 16 if mode == 0 else 4)
        st = stream if stream is not None else _stream(dev)
        L = lib()
        with self._lock:
            ws = self._dec_workspace(st, need) if mode == 0 else None
            rc = L.omf_topk_decode_counts(self._h, arr, _ptr(values), _ptr(indices), _ptr(y), int(mode), _ptr(ws),
                                          ctypes.c_size_t(0 if ws is None else ws.numel()), ctypes.c_void_p(st))
            if rc != 0 and ws is not None:
                self._dec_ws.pop(st, None)
            check(rc, "omf_topk_decode_counts")
        return y


def div_(y: torch.Tensor, divisor: float, stream: Optional[int] = None) -> torch.Tensor:
    """In-place ``y /= divisor`` (fp32 IEEE division) on the GPU."""
    if y.dtype != torch.float32 or not y.is_cuda or not y.is_contiguous() or y.data_ptr() % 16:
        raise ValueError("div_: y must be a contiguous, 16-byte aligned fp32 CUDA tensor")
    st = stream if stream is not None else _stream(y.device)
    check(lib().omf_div_f32(_ptr(y), y.numel(), float(divisor), ctypes.c_void_p(st)), "omf_div_f32")
    return y


def topk_decode(values: torch.Tensor, indices: torch.Tensor, n: int, y: Optional[torch.Tensor] = None,
                mode: int = 0, stream: Optional[int] = None) -> torch.Tensor:
    """Scatter decode of one tensor: mode 0 zeros+set, 1 overlay on ``y``, 2 scatter-add into ``y``."""
    dev = values.device
    if not dev.type == "cuda":
        raise ValueError("topk_decode runs on a GPU device")
    if values.dtype != torch.float32 or indices.dtype != torch.int64:
        raise ValueError("values must be fp32 and indices int64")
    values = values.contiguous()
    indices = indices.to(dev).contiguous()
    if values.numel() != indices.numel():
        raise ValueError("values and indices differ in length")
    if y is None:
        if mode != 0:
            raise ValueError("mode 1/2 need y")
        y = torch.empty(int(n), dtype=torch.float32, device=dev)
    _need(y, "y", torch.float32, dev, int(n), 4)
    st = stream if stream is not None else _stream(dev)
    check(lib().omf_topk_decode(_ptr(values), _ptr(indices), values.numel(), _ptr(y), int(n), int(mode),
                                ctypes.c_void_p(st)), "omf_topk_decode")
    return y
