"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU oracle (liboracle.so).

The oracle is a plain-C restatement of TileDB's filter pipeline
(tiledb/sm/filter/*.cc, tiledb/sm/compressors/{dd,rle}_compressor.cc); see
tdb_oracle.h for the pinning story.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.  It is the checker, never
the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u64p = ctypes.POINTER(ctypes.c_uint64)
i32p = ctypes.POINTER(ctypes.c_int32)


class OraclePipelineStruct(ctypes.Structure):
    _fields_ = [
        ("max_chunk_size", ctypes.c_uint32),
        ("nfilters", ctypes.c_uint32),
        ("version", ctypes.c_uint32),
        ("on_disk_type", ctypes.c_uint8),
        ("cell_size", ctypes.c_uint64),
        ("f", (ctypes.c_uint64 * 8) * 32),  # opaque, >= sizeof(oracle_filter)[32]
    ]


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "tdb_oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_pipeline_parse.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint8,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_pipeline_serialize.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t,
                                                ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_filter_tile.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64, u64p, ctypes.c_uint64,
                                         ctypes.c_uint64, u8p, ctypes.c_uint64, u64p]
        L.oracle_filtered_bound.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_filtered_bound.restype = ctypes.c_uint64
        L.oracle_unfilter_tile.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64,
                                           ctypes.c_int]
        L.oracle_unfilter_tiles_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u8p, u64p, u64p, u8p,
                                               u64p, u64p, ctypes.c_int, i32p]
        L.oracle_rle_compress.argtypes = [ctypes.c_uint64, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, u64p]
        L.oracle_rle_decompress.argtypes = [ctypes.c_uint64, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64]
        L.oracle_dd_compress.argtypes = [ctypes.c_uint8, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, u64p]
        L.oracle_dd_decompress.argtypes = [ctypes.c_uint8, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64]
        L.oracle_bitshuffle_block.argtypes = [ctypes.c_int, ctypes.c_uint32, u8p, ctypes.c_uint64, u8p]
        L.oracle_byteshuffle.argtypes = [ctypes.c_int, ctypes.c_uint32, u8p, ctypes.c_uint64, u8p]
        L.oracle_compute_chunk_size.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_compute_chunk_size.restype = ctypes.c_uint32
        L.oracle_datatype_size.argtypes = [ctypes.c_uint8]
        L.oracle_datatype_size.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), dtype=np.uint8)
    return np.ascontiguousarray(a).view(np.uint8).reshape(-1)


def _p(a: np.ndarray):
    return a.ctypes.data_as(u8p)


class OracleError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: oracle status {code}")
        self.code = code


class OraclePipeline:
    """A parsed pipeline descriptor (FilterPipeline::deserialize semantics)."""

    def __init__(self, serialized: bytes, version: int, datatype: int, cell_size: int):
        self._s = OraclePipelineStruct()
        buf = _u8(serialized)
        consumed = ctypes.c_size_t(0)
        rc = lib().oracle_pipeline_parse(_p(buf), len(buf), version, datatype, cell_size,
                                         ctypes.byref(self._s), ctypes.byref(consumed))
        if rc:
            raise OracleError(rc, "oracle_pipeline_parse")
        self.consumed = consumed.value
        self.version = version
        self.datatype = datatype
        self.cell_size = cell_size

    @property
    def ptr(self):
        return ctypes.byref(self._s)

    def serialize(self) -> bytes:
        out = np.zeros(4096, dtype=np.uint8)
        n = ctypes.c_size_t(0)
        rc = lib().oracle_pipeline_serialize(self.ptr, _p(out), out.size, ctypes.byref(n))
        if rc:
            raise OracleError(rc, "oracle_pipeline_serialize")
        return out[: n.value].tobytes()

    def filter_tile(self, data, offsets=None, max_chunk: int = 0) -> bytes:
        d = _u8(data)
        bound = lib().oracle_filtered_bound(self.ptr, d.size, max_chunk)
        out = np.zeros(bound, dtype=np.uint8)
        n = ctypes.c_uint64(0)
        if offsets is not None:
            offs = np.ascontiguousarray(offsets, dtype=np.uint64)
            op, no = offs.ctypes.data_as(u64p), offs.size
        else:
            op, no = None, 0
        rc = lib().oracle_filter_tile(self.ptr, _p(d), d.size, op, no, max_chunk, _p(out), out.size,
                                      ctypes.byref(n))
        if rc:
            raise OracleError(rc, "oracle_filter_tile")
        return out[: n.value].tobytes()

    def unfilter_tile(self, filtered, out_size: int, is_offsets: bool = False, fill: int = 0):
        """Returns (status, output bytes as np.uint8).  Output starts as `fill`."""
        f = _u8(filtered)
        out = np.full(out_size, fill, dtype=np.uint8)
        rc = lib().oracle_unfilter_tile(self.ptr, _p(f), f.size, _p(out), out_size, int(is_offsets))
        return rc, out

    def unfilter_tiles_mt(self, in_base: np.ndarray, in_off, in_size, out_base: np.ndarray, out_off,
                          out_size, nthreads: int):
        in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
        in_size = np.ascontiguousarray(in_size, dtype=np.uint64)
        out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
        out_size = np.ascontiguousarray(out_size, dtype=np.uint64)
        st = np.zeros(in_off.size, dtype=np.int32)
        rc = lib().oracle_unfilter_tiles_mt(
            self.ptr, in_off.size, _p(in_base), in_off.ctypes.data_as(u64p), in_size.ctypes.data_as(u64p),
            _p(out_base), out_off.ctypes.data_as(u64p), out_size.ctypes.data_as(u64p), nthreads,
            st.ctypes.data_as(i32p))
        return rc, st


def rle_compress(value_size: int, data) -> bytes:
    d = _u8(data)
    out = np.zeros(d.size * 3 + 64, dtype=np.uint8)
    n = ctypes.c_uint64(0)
    rc = lib().oracle_rle_compress(value_size, _p(d), d.size, _p(out), out.size, ctypes.byref(n))
    if rc:
        raise OracleError(rc, "rle_compress")
    return out[: n.value].tobytes()


def rle_decompress(value_size: int, data, out_size: int):
    d = _u8(data)
    out = np.zeros(out_size, dtype=np.uint8)
    rc = lib().oracle_rle_decompress(value_size, _p(d), d.size, _p(out), out_size)
    return rc, out


def dd_compress(dtype: int, data) -> bytes:
    d = _u8(data)
    out = np.zeros(d.size + 64, dtype=np.uint8)
    n = ctypes.c_uint64(0)
    rc = lib().oracle_dd_compress(dtype, _p(d), d.size, _p(out), out.size, ctypes.byref(n))
    if rc:
        raise OracleError(rc, "dd_compress")
    return out[: n.value].tobytes()


def dd_decompress(dtype: int, data, out_size: int):
    d = _u8(data)
    out = np.zeros(out_size, dtype=np.uint8)
    rc = lib().oracle_dd_decompress(dtype, _p(d), d.size, _p(out), out_size)
    return rc, out


def bitshuffle_block(data, ts: int, inverse: bool = False) -> bytes:
    d = _u8(data)
    out = np.zeros(d.size, dtype=np.uint8)
    lib().oracle_bitshuffle_block(int(inverse), ts, _p(d), d.size, _p(out))
    return out.tobytes()


def byteshuffle(data, ts: int, inverse: bool = False) -> bytes:
    d = _u8(data)
    out = np.zeros(d.size, dtype=np.uint8)
    lib().oracle_byteshuffle(int(inverse), ts, _p(d), d.size, _p(out))
    return out.tobytes()


def compute_chunk_size(tile_size: int, cell_size: int, max_chunk: int = 0) -> int:
    return lib().oracle_compute_chunk_size(tile_size, cell_size, max_chunk)


# ---------------------------------------------------------------------------
# the steps either side of the path, restated in numpy
# ---------------------------------------------------------------------------
def filtered_data_blocks(file_idx, file_offset, size, min_batch_size: int = 20971520,
                         max_batch_size: int = 104857600, min_batch_gap: int = 512000):
    """FilteredData::make_new_block_if_required (filtered_data.h:531-575),
    one TileType: tiles in result-tile order; a tile extends the current block
    iff same fragment, new_size <= max_batch_size and (new_size <=
    min_batch_size or gap <= min_batch_gap), with the reference's unsigned
    64-bit arithmetic for new_size and gap.  Returns the first tile of every
    block followed by ntiles."""
    M = (1 << 64) - 1
    first = []
    cur = None
    boff = bsize = 0
    for i, (f, off, sz) in enumerate(zip(file_idx, file_offset, size)):
        off, sz = int(off), int(sz)
        if cur is None:
            first.append(i)
            boff, bsize, cur = off, sz, int(f)
            continue
        new_size = ((off + sz) - boff) & M
        gap = (off - (boff + bsize)) & M
        if cur == int(f) and new_size <= max_batch_size and (new_size <= min_batch_size or gap <= min_batch_gap):
            bsize = new_size
        else:
            first.append(i)
            boff, bsize, cur = off, sz, int(f)
    return first + [len(size)]


def dense_subarray_cells(tiles, tile_start, tile_extent, cell_size: int, sub_lo, sub_hi,
                         cell_order: int = 0, layout: int = 0) -> np.ndarray:
    """DenseReader::copy_fixed_tiles (dense_reader.cc:1555-1750) for one
    fragment covering the subarray: the subarray's cells, from the tiles
    (tile t holds the cells [tile_start[t], + tile_extent) in cell order
    cell_order: 0 row-major, 1 col-major), in result layout `layout`.  Cells
    are cell_size-byte records."""
    nd = len(tile_extent)
    ext = [int(e) for e in tile_extent]
    lo = [int(x) for x in sub_lo]
    hi = [int(x) for x in sub_hi]
    shape = tuple(h - l + 1 for l, h in zip(lo, hi))
    out = np.zeros(shape + (cell_size,), dtype=np.uint8)
    for t, raw in enumerate(tiles):
        s = [int(x) for x in tile_start[t]]
        a = [max(s[d], lo[d]) for d in range(nd)]
        b = [min(s[d] + ext[d] - 1, hi[d]) for d in range(nd)]
        if any(b[d] < a[d] for d in range(nd)):
            continue
        cells = np.frombuffer(bytes(raw), dtype=np.uint8).reshape(-1, cell_size)
        blk = cells.reshape(tuple(ext) + (cell_size,) if cell_order == 0 else tuple(reversed(ext)) + (cell_size,))
        if cell_order == 1:  # col-major: the first dimension fastest
            blk = np.transpose(blk, tuple(reversed(range(nd))) + (nd,))
        src = tuple(slice(a[d] - s[d], b[d] - s[d] + 1) for d in range(nd))
        dst = tuple(slice(a[d] - lo[d], b[d] - lo[d] + 1) for d in range(nd))
        out[dst] = blk[src]
    if layout == 1:
        out = np.transpose(out, tuple(reversed(range(nd))) + (nd,))
    return np.ascontiguousarray(out).reshape(-1)
