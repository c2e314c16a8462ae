"""Build recipe of the in-tree HIP library ``omnifed_amd/libomf_codec.so`` (gfx950 only).

``python -m omnifed_amd.build`` (or ``__graft_entry__.build()``) compiles every
source under ``omnifed_amd/csrc`` with ``hipcc --offload-arch=gfx950`` into one
shared library that travels with the repo snapshot to the GPU box (it is
git-ignored, not gpurun-ignored).  Rebuilds only when a source is newer.
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "libomf_codec.so")

SOURCES = ["omf_runtime.cpp", "omf_qsgd.hip", "omf_qsgd_ring.hip", "omf_qsgd_pack.hip", "omf_topk.hip",
           "omf_topk_host.cpp"]

# Exact IEEE fp32 (no contraction, denormals kept, correctly rounded / and sqrt): the
# payload must match the reference bit for bit.
FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++20",
    "-fPIC",
    "-ffp-contract=off",
    "-fno-gpu-flush-denormals-to-zero",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall",
    "-Wno-unused-function",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build omnifed_amd)")


def _sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def source_digest() -> str:
    """SHA-256 over the library's sources and headers (stamps measurements taken with a build)."""
    import hashlib

    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h", ".cpp")))
    for f in files:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    for f in sorted(os.listdir(INCLUDE)):
        with open(os.path.join(INCLUDE, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = _sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE)]
    return any(os.path.getmtime(d) > t for d in deps)


def _toolchain_stamp() -> str:
    """The compiler and flags the objects in _obj were built with."""
    return "\n".join([os.path.realpath(hipcc()), *FLAGS]) + "\n"


def build(force: bool = False, verbose: bool = False) -> str:
    objdir = os.path.join(HERE, "_obj")
    # beside the library (it travels with it to the GPU box; _obj does not)
    stamp_path = LIB + ".stamp"
    stamp = _toolchain_stamp()
    try:
        with open(stamp_path) as fh:
            stale = fh.read() != stamp
    except OSError:
        stale = True
    if stale:
        force = True  # another compiler or flag set (or no record of one): nothing is reused
    if not force and not needs_build():
        return LIB
    os.makedirs(objdir, exist_ok=True)
    objs = []
    procs = []
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE)]
    for src in _sources():
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in [src, *headers]):
            continue  # object newer than its source and every header
        cmd = [hipcc(), *FLAGS, "-I", INCLUDE, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), src))
    for p, src in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{out.decode(errors='replace')}")
    tmp = LIB + ".tmp"
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout.decode(errors="replace"))
    os.replace(tmp, LIB)
    with open(stamp_path, "w") as fh:
        fh.write(stamp)
    # the offload linker leaves per-target unbundling temporaries beside the output
    for f in os.listdir(HERE):
        if f.startswith("libomf_codec.so.") and ("-amdhsa-" in f or "-linux-gnu" in f):
            os.remove(os.path.join(HERE, f))
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
