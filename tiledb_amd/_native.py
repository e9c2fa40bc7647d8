"""ctypes binding of libtiledb_amd.so (the C-ABI in include/tiledb_amd.h).

The library is built in-tree by tiledb_amd/build.py (hipcc, gfx950).  There is
no CPU fallback: if the library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
import re
import sys

try:  # torch ships its own libamdhip64; load it first so one HIP runtime is used
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for pure C-ABI use
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtiledb_amd.so")
# experiments and fault-injection tests only: TDBG_LIB names another in-tree
# build of the same C-ABI in this package directory (the experiments library
# libtiledb_amd_exp.so, or an earlier commit's build for same-box A/B timing)
if os.environ.get("TDBG_LIB"):
    _name = os.environ["TDBG_LIB"]
    if os.path.basename(_name) != _name or not re.fullmatch(r"libtiledb_amd[A-Za-z0-9_]*\.so", _name):
        raise ImportError(f"TDBG_LIB={_name!r}: not a libtiledb_amd*.so in {_HERE}")
    LIB_PATH = os.path.join(_HERE, _name)
    sys.stderr.write(f"tiledb_amd: TDBG_LIB set, loading {LIB_PATH} instead of the product library\n")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build the HIP engine with `python tiledb_amd/build.py` "
        "(or __graft_entry__.build()); there is no CPU fallback")

lib = ctypes.CDLL(LIB_PATH)

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/tiledb_amd.h exactly
SIGNATURES = {
    "tdbg_last_error": (ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t]),
    "tdbg_status_str": (ctypes.c_char_p, [ctypes.c_int]),
    "tdbg_pipeline_create": (ctypes.c_int, [c_u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint8,
                                            ctypes.c_uint64, ctypes.POINTER(c_vp)]),
    "tdbg_pipeline_destroy": (None, [c_vp]),
    "tdbg_pipeline_supported": (ctypes.c_int, [c_vp]),
    "tdbg_pipeline_num_filters": (ctypes.c_uint32, [c_vp]),
    "tdbg_pipeline_filter": (ctypes.c_int, [c_vp, ctypes.c_uint32, c_u8p, c_u8p]),
    "tdbg_context_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_vp)]),
    "tdbg_context_destroy": (None, [c_vp]),
    "tdbg_unfilter_tiles_async": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp,
                                                 ctypes.c_uint32, c_vp, c_vp]),
    "tdbg_unfilter_tiles_sync": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp,
                                                ctypes.c_uint32, c_i32p, c_vp]),
    "tdbg_unfilter_tiles_host": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp,
                                                ctypes.c_uint32, c_i32p, ctypes.c_uint64]),
    "tdbg_unfilter_offsets_host": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                  ctypes.c_uint32, c_i32p, ctypes.c_uint64]),
    "tdbg_add_extra_offsets_async": (ctypes.c_int, [c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "tdbg_unfilter_tiles_multi_gpu": (ctypes.c_int, [c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp,
                                                     ctypes.c_uint32, c_i32p,
                                                     ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                                     ctypes.c_uint64]),
    "tdbg_release_cached_contexts": (ctypes.c_int, []),
    "tdbg_cached_context_count": (ctypes.c_int, []),
    "tdbg_unfilter_tiles_cpu": (ctypes.c_int, [c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp,
                                               ctypes.c_uint32, c_i32p, ctypes.c_uint32]),
    "tdbg_filtered_bound": (ctypes.c_uint64, [c_vp, ctypes.c_uint64, ctypes.c_uint32]),
    "tdbg_filter_tiles_async": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                               ctypes.c_uint32, c_vp, c_vp]),
    "tdbg_filter_tiles_sync": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                              ctypes.c_uint32, c_i32p, c_vp]),
    "tdbg_context_stats": (ctypes.c_int, [c_vp, c_u64p, c_u64p]),
    "tdbg_context_path_stats": (ctypes.c_int, [c_vp, c_u64p, c_u64p, c_u64p]),
    "tdbg_context_stream_stats": (ctypes.c_int, [c_vp, c_u64p]),
    "tdbg_context_stream_raw_stats": (ctypes.c_int, [c_vp, c_u64p]),
    "tdbg_context_forward_stream_stats": (ctypes.c_int, [c_vp, c_u64p]),
    "tdbg_context_last_kernel_ms": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_float)]),
    "tdbg_context_time_launches": (ctypes.c_int, [c_vp, ctypes.c_uint32]),
    "tdbg_context_launch_times": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]),
    "tdbg_debug_phase_clocks": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]),
    "tdbg_shard_tiles": (ctypes.c_int, [ctypes.c_uint64, c_vp, c_vp, ctypes.c_uint32, c_vp]),
    "tdbg_device_alloc": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(c_vp)]),
    "tdbg_device_free": (ctypes.c_int, [c_vp]),
    "tdbg_memcpy_h2d": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64]),
    "tdbg_memcpy_d2h": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64]),
    "tdbg_device_count": (ctypes.c_int, [c_i32p]),
    "tdbg_context_device": (ctypes.c_int, [c_vp]),
    "tdbg_host_alloc_local": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(c_vp)]),
    "tdbg_host_free": (ctypes.c_int, [c_vp]),
    "tdbg_filtered_data_blocks": (ctypes.c_int, [ctypes.c_uint64, c_vp, c_vp, c_vp, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_uint64, c_vp, c_u64p]),
    "tdbg_read_unfilter_tiles": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, ctypes.c_uint32, c_vp, c_vp,
                                                c_vp, c_vp, c_vp, ctypes.c_uint32, c_vp, c_i32p]),
    "tdbg_dense_result_bytes": (ctypes.c_uint64, [c_vp]),
    "tdbg_dense_copy_async": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "tdbg_dense_read_host": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            ctypes.c_uint64, ctypes.c_uint32, c_i32p, ctypes.c_uint64]),
    "tdbg_context_stream_chunk_stats": (ctypes.c_int, [c_vp, c_u64p]),
    "tdbg_context_tile_chunk_stats": (ctypes.c_int, [c_vp, c_u64p]),
    "tdbg_dense_copy_fragments_async": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                       c_vp, c_vp, c_vp]),
    "tdbg_dense_var_offsets_async": (ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                    c_vp, c_vp, c_vp, c_vp]),
    "tdbg_dense_var_copy_async": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "tdbg_dense_var_status": (ctypes.c_int, [c_vp, c_vp, c_i32p]),
    "tdbg_dense_read_var_host": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, c_u64p, c_i32p]),
}

DENSE_MAX_DIMS = 4  # TDBG_DENSE_MAX_DIMS


class ReadConfig(ctypes.Structure):
    """tdbg_read_config (FilteredData block rule + IO threads)."""
    _fields_ = [("min_batch_size", ctypes.c_uint64), ("max_batch_size", ctypes.c_uint64),
                ("min_batch_gap", ctypes.c_uint64), ("io_threads", ctypes.c_uint32),
                ("slots", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class DenseCopyConfig(ctypes.Structure):
    """tdbg_dense_copy_config (DenseReader::copy_fixed_tiles for one fragment)."""
    _fields_ = [("dim_num", ctypes.c_uint32), ("cell_size", ctypes.c_uint32),
                ("cell_order", ctypes.c_uint32), ("layout", ctypes.c_uint32),
                ("tile_extent", ctypes.c_int64 * DENSE_MAX_DIMS),
                ("sub_lo", ctypes.c_int64 * DENSE_MAX_DIMS),
                ("sub_hi", ctypes.c_int64 * DENSE_MAX_DIMS)]


class DenseFragConfig(ctypes.Structure):
    """tdbg_dense_frag_config (several fragments, fill values, var cells)."""
    _fields_ = [("base", DenseCopyConfig), ("nfrag", ctypes.c_uint32), ("nullable", ctypes.c_uint32),
                ("fill_size", ctypes.c_uint32), ("fill_validity", ctypes.c_uint32),
                ("elements_mode", ctypes.c_uint32), ("data_type_size", ctypes.c_uint32)]

# symbols an older experimental build (TDBG_LIB) lacks; the product library
# must export every one
MISSING: set = set()
for _name, (_res, _args) in SIGNATURES.items():
    try:
        _f = getattr(lib, _name)
    except AttributeError:
        if not os.environ.get("TDBG_LIB"):
            raise
        MISSING.add(_name)
        continue
    _f.restype = _res
    _f.argtypes = _args


def last_error() -> str:
    buf = ctypes.create_string_buffer(1024)
    lib.tdbg_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def status_str(code: int) -> str:
    return lib.tdbg_status_str(code).decode()
