"""Build the MI355X engine in-tree: hipcc --offload-arch=gfx950 -> libtiledb_amd.so.

No torch/JIT involved: the shared library exports the C-ABI declared in
include/tiledb_amd.h and travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libtiledb_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TDBG_ARCH", "gfx950")

SOURCES = ["tdbg_kernels.hip", "tdbg_fast.hip", "tdbg_host.cpp"]
HEADERS = ["tdbg_desc.h", "tdbg_device.h", "tdbg_general.h"]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "tiledb_amd.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    common = ["-O3", "-std=c++17", "-fPIC", "-Wall", f"--offload-arch={ARCH}",
              "-I", os.path.join(ROOT, "include")]
    for src in SOURCES:
        obj = os.path.join(objdir, src + ".o")
        cmd = [HIPCC] + common + ["-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd = [HIPCC, "-x", "hip"] + common + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        objs.append(obj)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
