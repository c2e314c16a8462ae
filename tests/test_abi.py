"""The C ABI library builds for gfx950, loads, and exports every symbol include/omf_codec.h declares."""

import ctypes
import os
import re
import subprocess
import threading

import pytest

from omnifed_amd import _lib
from omnifed_amd.build import INCLUDE, LIB, build

HEADER = os.path.join(INCLUDE, "omf_codec.h")
EXPERIMENTAL = os.path.join(INCLUDE, "omf_codec_experimental.h")


def _declared(path=None):
    paths = [path] if path else [HEADER, EXPERIMENTAL]
    names = set()
    for p in paths:
        src = re.sub(r"/\*.*?\*/", "", open(p).read(), flags=re.S)
        names |= set(re.findall(r"\b(omf_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_drop_in_header_has_no_experiment_hooks():
    """The drop-in boundary (omf_codec.h) declares no tuning / debug hook; those live in
    omf_codec_experimental.h, and neither header declares a symbol twice."""
    main, exp = set(_declared(HEADER)), set(_declared(EXPERIMENTAL))
    assert not main & exp
    assert not any(re.search(r"(debug|ring|set_topk|set_wide|fused_bracket|resident|spec_stats)", n) for n in main), main
    assert {"omf_plan_set_debug", "omf_plan_set_topk", "omf_plan_set_ring"} <= exp


def test_build_and_load():
    path = build()
    assert os.path.exists(path)
    L = _lib.lib()
    assert L.omf_abi_version() == _lib.ABI_VERSION
    # the header's define, the library and the Python binding agree
    assert re.search(r"#define OMF_ABI_VERSION (\d+)", open(HEADER).read()).group(1) == str(_lib.ABI_VERSION)
    seen = []  # a thread that made no call has no error (the string is per thread)
    th = threading.Thread(target=lambda: seen.append(L.omf_last_error()))
    th.start()
    th.join()
    assert seen == [b""]


def test_every_declared_symbol_exported_and_bound():
    build()
    decl = _declared()
    assert len(decl) >= 12
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (omf_[a-z0-9_]+)", out))
    missing = [d for d in decl if d not in exported]
    assert not missing, missing
    assert sorted(_lib.SIGNATURES) == decl  # the ctypes table binds exactly the header


def test_gfx950_code_object():
    build()
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", LIB], capture_output=True,
                         text=True, cwd="/tmp")
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in (out.stdout + out.stderr) or "gfx950" in open(LIB, "rb").read().decode("latin-1")


def test_host_only_entry_points_without_gpu():
    L = _lib.lib()
    assert L.omf_topk_k(32, 0.25) == 8
    assert L.omf_topk_k(100, 0.001) == 1
    assert L.omf_topk_k(11181642, 0.01) == int(11181642 * 0.01)
    # argument validation happens before any device work
    rc = L.omf_plan_create(None, None, 0, 0, 0, ctypes.byref(ctypes.c_void_p()))
    assert rc == _lib.OMF_EINVAL
    assert b"tensor" in L.omf_last_error()
    assert L.omf_qsgd_encode(None, None, 1.0, 4, None, 0, 0, None, None, None, None) == _lib.OMF_EINVAL
    assert L.omf_div_f32(None, -1, 1.0, None) == _lib.OMF_EINVAL
    assert L.omf_topk_decode(None, None, 0, None, 0, 5, None) == _lib.OMF_EINVAL
    with pytest.raises(ValueError):
        _lib.check(_lib.OMF_EINVAL, "probe")


def test_no_oracle_in_product_path():
    """The shipped package never imports the CPU oracle (it is test infrastructure only)."""
    root = os.path.dirname(LIB)
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", txt, flags=re.M), f
