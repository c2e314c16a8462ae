"""ctypes binding of ``libomf_codec.so`` (declarations: ``include/omf_codec.h``, and the test /
experiment hooks of ``include/omf_codec_experimental.h``).

There is no CPU fallback: if the library is missing, ``lib()`` raises.  The
library is built in-tree by ``omnifed_amd.build`` and loaded from
``omnifed_amd/libomf_codec.so`` so that the driver can see which native code
ran.  ctypes releases the GIL for the duration of every call.
"""

from __future__ import annotations

import ctypes
import os
import threading

from .build import LIB as LIB_PATH

OMF_OK = 0
OMF_EINVAL = -1
OMF_EHIP = -2
OMF_ETIMEOUT = -3
OMF_ENOMEM = -4

_c_i32 = ctypes.c_int32
_c_i64 = ctypes.c_int64
_c_u64 = ctypes.c_uint64
_c_f32 = ctypes.c_float
_c_f64 = ctypes.c_double
_c_p = ctypes.c_void_p
_c_size = ctypes.c_size_t

# name -> (restype, argtypes); every symbol include/omf_codec.h and omf_codec_experimental.h declare.
SIGNATURES = {
    "omf_abi_version": (ctypes.c_int, []),
    "omf_last_error": (ctypes.c_char_p, []),
    "omf_plan_create": (ctypes.c_int, [ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64), _c_i32, _c_i64,
                                        ctypes.c_int, ctypes.POINTER(_c_p)]),
    "omf_plan_destroy": (ctypes.c_int, [_c_p]),
    "omf_plan_encode_items": (_c_i64, [_c_p]),
    "omf_plan_check": (ctypes.c_int, [_c_p, _c_p]),
    "omf_plan_set_encode_strategy": (ctypes.c_int, [_c_p, _c_i32]),
    "omf_plan_encode_strategy": (_c_i32, [_c_p]),
    "omf_plan_last_encoder": (_c_i32, [_c_p]),
    "omf_plan_set_wide_levels": (ctypes.c_int, [_c_p, _c_i32]),
    "omf_plan_set_fused_bracket": (ctypes.c_int, [_c_p, _c_i32]),
    "omf_plan_resident_capacity": (_c_i64, [_c_p]),
    "omf_plan_set_resident_capacity": (ctypes.c_int, [_c_p, _c_i64, _c_i64]),
    "omf_plan_set_ring": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i64, _c_i64]),
    "omf_plan_set_debug": (ctypes.c_int, [_c_p, ctypes.c_uint32, ctypes.c_uint32, _c_i64]),
    "omf_plan_ring_info": (ctypes.c_int, [_c_p, ctypes.POINTER(_c_i64)]),
    "omf_plan_spec_stats": (ctypes.c_int, [_c_p, _c_p, ctypes.POINTER(_c_i64)]),
    "omf_plan_ring_profile": (ctypes.c_int, [_c_p, ctypes.POINTER(_c_i64)]),
    "omf_qsgd_encode": (ctypes.c_int, [_c_p, _c_p, _c_f32, _c_i32, _c_p, _c_u64, _c_u64, _c_p, _c_p, _c_p, _c_p]),
    "omf_qsgd_norms": (ctypes.c_int, [_c_p, _c_p, _c_f32, _c_p, _c_p]),
    "omf_qsgd_encode_ex": (ctypes.c_int, [_c_p, _c_p, _c_f32, _c_i32, _c_i32, _c_p, _c_u64, _c_u64, _c_p, _c_p, _c_p,
                                          _c_p]),
    "omf_qsgd_norms_ex": (ctypes.c_int, [_c_p, _c_p, _c_f32, _c_i32, _c_p, _c_p]),
    "omf_ps_apply_encode": (ctypes.c_int, [_c_p, _c_p, _c_f32, _c_p, _c_i32, _c_p, _c_u64, _c_u64, _c_p, _c_p,
                                           _c_p]),
    "omf_ps_accumulate_apply_encode": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_f32, _c_p,
                                                      _c_i32, _c_p, _c_u64, _c_u64, _c_p, _c_p, _c_p]),
    "omf_qsgd_decode": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_p]),
    "omf_qsgd_decode_range": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_i64, _c_i64, _c_p]),
    "omf_div_f32": (ctypes.c_int, [_c_p, _c_i64, _c_f32, _c_p]),
    "omf_qsgd_packed_bits": (_c_i32, [_c_i32]),
    "omf_qsgd_pack": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p]),
    "omf_qsgd_decode_packed": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_p, _c_p, _c_i32, _c_p]),
    "omf_topk_k": (_c_i64, [_c_i64, _c_f64]),
    "omf_plan_set_topk": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i64, _c_f32, _c_f32]),
    "omf_topk_stats": (ctypes.c_int, [_c_p, ctypes.POINTER(_c_i64), _c_i32]),
    "omf_topk_workspace_bytes": (_c_size, [_c_p, _c_f64]),
    "omf_topk_encode": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i32, _c_f64, _c_f32, _c_p, _c_p, _c_p, _c_size, _c_p]),
    "omf_topk_torch_order": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i32, _c_f64, _c_f32, _c_p, _c_p, _c_p, _c_size,
                                            _c_p, ctypes.POINTER(_c_i64)]),
    "omf_topk_select_host": (ctypes.c_int, [_c_p, _c_i64, _c_i64, _c_p]),
    "omf_topk_decode": (ctypes.c_int, [_c_p, _c_p, _c_i64, _c_p, _c_i64, _c_i32, _c_p]),
    "omf_topk_decode_arena": (ctypes.c_int, [_c_p, _c_f64, _c_p, _c_p, _c_p, _c_i32, _c_p]),
    "omf_topk_decode_workspace_bytes": (_c_size, [_c_p, _c_f64]),
    "omf_topk_decode_arena_ws": (ctypes.c_int, [_c_p, _c_f64, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_size, _c_p]),
    "omf_topk_decode_counts_workspace_bytes": (_c_size, [_c_p, ctypes.POINTER(_c_i64)]),
    "omf_topk_decode_counts": (ctypes.c_int, [_c_p, ctypes.POINTER(_c_i64), _c_p, _c_p, _c_p, _c_i32, _c_p, _c_size,
                                              _c_p]),
    "omf_topk_check_indices": (ctypes.c_int, [_c_p, ctypes.POINTER(_c_i64), _c_p, _c_p, _c_p]),
    "omf_topk_check_duplicates": (ctypes.c_int, [_c_p, ctypes.POINTER(_c_i64), _c_p, _c_p, _c_p]),
}

_lock = threading.Lock()
_lib = None


class CodecError(RuntimeError):
    pass


ABI_VERSION = 112  # include/omf_codec.h OMF_ABI_VERSION; a library of another version is refused


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP codec library; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = os.environ.get("OMF_CODEC_LIB_EXPERIMENT") or LIB_PATH  # variant builds (scripts/exp)
            if not os.path.exists(path):
                raise CodecError(
                    f"HIP codec library not built: {LIB_PATH} is missing "
                    "(run `python -m omnifed_amd.build`); there is no CPU fallback")
            L = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if L.omf_abi_version() != ABI_VERSION:
                raise CodecError(f"{path} has ABI {L.omf_abi_version()}, this package needs {ABI_VERSION} "
                                 "(rebuild: `python -m omnifed_amd.build`)")
            _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc == OMF_OK:
        return
    msg = lib().omf_last_error().decode(errors="replace")
    if rc == OMF_EINVAL:
        raise ValueError(f"{what}: {msg}")
    raise CodecError(f"{what} failed ({rc}): {msg}")
