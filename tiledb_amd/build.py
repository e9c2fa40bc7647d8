"""Build the MI355X engine in-tree: hipcc --offload-arch=gfx950 -> libtiledb_amd.so.

No torch/JIT involved: the shared library exports the C-ABI declared in
include/tiledb_amd.h and travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libtiledb_amd.so")
# The experiments build (timing ablations, A/B switches, fault injection and
# phase clocks read from TDBG_* environment variables, tdbg_hooks.h): the
# units that read hooks are compiled again with -DTDBG_EXPERIMENTS, every
# other object is shared with the product library.  Only tests that inject
# faults (in a subprocess, through TDBG_LIB) and the tools/ studies load it.
EXP_LIB = os.path.join(HERE, "libtiledb_amd_exp.so")
# Build provenance: the digest of every source, header and flag the library
# was built from, written next to it (travels with it to the GPU box, stays
# out of git like the library).  build() rebuilds whenever the tree's digest
# differs from the recorded one, not only on a newer mtime.
MANIFEST = os.path.join(HERE, "libtiledb_amd.build.json")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TDBG_ARCH", "gfx950")

NPART = 6  # fused-kernel spec table split (TDBG_NPART; tdbg_host.cpp TDBG_NPART_HOST)
# (source, object name, extra flags)
UNITS = ([("tdbg_kernels.hip", "tdbg_kernels", []), ("tdbg_chunkdir.hip", "tdbg_chunkdir", []), ("tdbg_host.cpp", "tdbg_host", []),
          ("tdbg_forward.hip", "tdbg_forward", []),
          ("tdbg_c5tile.hip", "tdbg_c5tile", []),
          # the C5 tile kernel's multi-chunk variant (TDBG_MULTI_CHUNK launches)
          ("tdbg_c5tile.hip", "tdbg_c5tile_mc", ["-DTDBG_C5T_MC_UNIT", "-mllvm", "-disable-machine-licm"]),
          ("tdbg_c2tile.hip", "tdbg_c2tile", []),
          ("tdbg_stream_small.hip", "tdbg_stream_small", []),
          ("tdbg_stream_small.hip", "tdbg_stream_small_512", ["-DTDBG_SMALL_NT=512"]),
          ("tdbg_stream_small.hip", "tdbg_stream_small_256np", ["-DTDBG_SMALL_NP=1"]),
          ("tdbg_forward_stream.hip", "tdbg_forward_stream", []),
          ("tdbg_forward_small.hip", "tdbg_forward_small", []),
          ("tdbg_forward_shuffle.hip", "tdbg_forward_shuffle", []),
          ("tdbg_stream_shuffle.hip", "tdbg_stream_shuffle", []),
          ("tdbg_dense.hip", "tdbg_dense", []),
          ("tdbg_io.cpp", "tdbg_io", []),
          # CPU entry: host-only C++, product and sum rounded separately
          # (FLOAT_SCALE parity with the reference's x86-64 build)
          ("tdbg_cpu.cpp", "tdbg_cpu", ["-ffp-contract=off"])] +
         [("tdbg_fast.hip", f"tdbg_fast_p{k}", [f"-DTDBG_PART={k}", f"-DTDBG_NPART={NPART}"])
          for k in range(NPART)])
# Retired C5 kernels (round 4's persistent coded-DD and raw-DD streaming
# kernels, replaced by tdbg_c5tile.hip): only in the experiments library, for
# same-box A/Bs through TDBG_C5_OLD_RAW; the product library does not contain
# them.
EXP_ONLY_UNITS = [("tdbg_stream.hip", "tdbg_stream", []), ("tdbg_stream_raw.hip", "tdbg_stream_raw", [])]
HOST_ONLY = {"tdbg_cpu.cpp"}
NO_SCRATCH = {"tdbg_stream.hip", "tdbg_stream_raw.hip", "tdbg_stream_small.hip", "tdbg_c5tile.hip",
              "tdbg_c2tile.hip"}  # checked with -Rpass-analysis
HEADERS = ["tdbg_desc.h", "tdbg_device.h", "tdbg_general.h", "tdbg_rules.h", "tdbg_stream_common.h", "tdbg_launch.h",
           "tdbg_hooks.h"]
HOOK_UNITS = {"tdbg_host.cpp", "tdbg_io.cpp", "tdbg_c5tile.hip", "tdbg_c2tile.hip", "tdbg_stream.hip", "tdbg_stream_raw.hip",
              "tdbg_stream_small.hip"}


def _deps(src: str):
    d = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in HEADERS]
    d.append(os.path.join(ROOT, "include", "tiledb_amd.h"))
    return d


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def source_digest() -> str:
    """sha256 over the library's sources, headers, the C-ABI header and the
    build flags (arch, fused-spec split, per-unit extra flags)."""
    h = hashlib.sha256()
    files = sorted({d for src, _, _ in UNITS for d in _deps(src)})
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(json.dumps([ARCH, NPART, [(s, n, e) for s, n, e in UNITS]]).encode())
    return h.hexdigest()


def manifest() -> dict:
    """The recorded provenance of the built library ({} if none)."""
    try:
        with open(MANIFEST) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def _stale() -> bool:
    if _newer(LIB, [d for src, _, _ in UNITS for d in _deps(src)]):
        return True
    return manifest().get("sources_sha256") != source_digest()


def build(force: bool = False, verbose: bool = False, experiments: bool = False) -> str:
    lib = _build(force, verbose)
    if experiments:
        _build_exp(force, verbose)
    return lib


def _build(force: bool, verbose: bool) -> str:
    if not force and not _stale():
        return LIB
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC", "-Wall", f"--offload-arch={ARCH}",
              "-I", os.path.join(ROOT, "include")]
    jobs, objs = [], []
    for src, name, extra in UNITS:
        obj = os.path.join(objdir, name + ".o")
        objs.append(obj)
        if not force and not _newer(obj, _deps(src)):
            continue
        if src in HOST_ONLY:
            flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-I", os.path.join(ROOT, "include")]
        else:
            flags = (["-x", "hip"] if src.endswith(".cpp") else []) + common
        cmd = [HIPCC] + flags + extra + ["-c", os.path.join(CSRC, src), "-o", obj]
        jobs.append(cmd)

    _compile(jobs, verbose)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    hipcc = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.strip().splitlines()
    with open(MANIFEST + ".tmp", "w") as fh:
        json.dump({"library": os.path.basename(LIB), "sources_sha256": source_digest(), "arch": ARCH,
                   "units": len(UNITS), "recompiled_units": len(jobs), "forced": bool(force),
                   "hipcc": hipcc[0] if hipcc else "", "lib_sha256": _file_sha(LIB)}, fh, indent=1)
    os.replace(MANIFEST + ".tmp", MANIFEST)
    return LIB


def _compile(jobs, verbose: bool) -> None:
    from concurrent.futures import ThreadPoolExecutor

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        src = cmd[cmd.index("-c") + 1]
        if os.path.basename(src) in NO_SCRATCH:
            r = subprocess.run(cmd + ["-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
            if r.returncode:
                sys.stderr.write(r.stderr)
                raise subprocess.CalledProcessError(r.returncode, cmd)
            bad = [ln for ln in r.stderr.splitlines() if "ScratchSize" in ln and not ln.rstrip().endswith(": 0")
                   and "[bytes/lane]: 0 " not in ln]
            if bad:
                raise RuntimeError(f"{src}: kernels use scratch (counted vmcnt waits would break):\n" + "\n".join(bad))
        else:
            subprocess.check_call(cmd)

    nproc = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(nproc) as ex:
        list(ex.map(run, jobs))


def _build_exp(force: bool, verbose: bool) -> str:
    """libtiledb_amd_exp.so: the product objects, with the hook units
    recompiled under -DTDBG_EXPERIMENTS (the product library is built first)."""
    objdir = os.path.join(HERE, "build")
    common = ["-O3", "-std=c++17", "-fPIC", "-Wall", f"--offload-arch={ARCH}",
              "-I", os.path.join(ROOT, "include"), "-DTDBG_EXPERIMENTS"]
    jobs, objs = [], []
    for src, name, extra in UNITS + EXP_ONLY_UNITS:
        if src not in HOOK_UNITS:
            objs.append(os.path.join(objdir, name + ".o"))
            continue
        obj = os.path.join(objdir, name + "_exp.o")
        objs.append(obj)
        if not force and not _newer(obj, _deps(src)):
            continue
        flags = (["-x", "hip"] if src.endswith(".cpp") else []) + common
        jobs.append([HIPCC] + flags + extra + ["-c", os.path.join(CSRC, src), "-o", obj])
    if not jobs and not _newer(EXP_LIB, objs):
        return EXP_LIB
    _compile(jobs, verbose)
    tmp = EXP_LIB + ".tmp"
    subprocess.check_call([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lpthread"])
    os.replace(tmp, EXP_LIB)
    return EXP_LIB


def _file_sha(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def provenance() -> dict:
    """Whether the library on disk is the one built from this tree: the
    manifest's source digest against the tree's, and its library hash
    against the file."""
    m = manifest()
    ok_src = m.get("sources_sha256") == source_digest()
    ok_lib = os.path.exists(LIB) and m.get("lib_sha256") == _file_sha(LIB)
    return {"sources_match": ok_src, "library_match": ok_lib, "sources_sha256": m.get("sources_sha256", ""),
            "recompiled_units": m.get("recompiled_units"), "hipcc": m.get("hipcc", "")}


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, experiments="--experiments" in sys.argv))
