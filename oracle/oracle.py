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


def _tile_cells(raw, ext, cell_size: int, cell_order: int):
    """A tile's cells as an array indexed by (coords..., byte): cell order 0
    row-major (last dimension fastest), 1 col-major."""
    nd = len(ext)
    cells = np.frombuffer(bytes(raw), dtype=np.uint8)[: int(np.prod(ext)) * cell_size].reshape(-1, cell_size)
    blk = cells.reshape((tuple(ext) if cell_order == 0 else tuple(reversed(ext))) + (cell_size,))
    if cell_order == 1:
        blk = np.transpose(blk, tuple(reversed(range(nd))) + (nd,))
    return blk


def _frag_masks(t_start, ext, lo, hi, frag_dom, present):
    """Per space tile: the region (tile box intersected with the subarray, as
    slices on both sides) and, for every fragment domain fd, the cells of the
    region it covers (cell_slab_overlaps_range, dense_reader.cc:1521-1552: a
    cell of a slab overlaps a fragment domain iff every coordinate lies in it)
    -- False where the fragment has no tile here (tile_tuples[fd] == nullptr)."""
    nd = len(ext)
    a = [max(t_start[d], lo[d]) for d in range(nd)]
    b = [min(t_start[d] + ext[d] - 1, hi[d]) for d in range(nd)]
    if any(b[d] < a[d] for d in range(nd)):
        return None
    src = tuple(slice(a[d] - t_start[d], b[d] - t_start[d] + 1) for d in range(nd))
    dst = tuple(slice(a[d] - lo[d], b[d] - lo[d] + 1) for d in range(nd))
    grids = np.meshgrid(*[np.arange(a[d], b[d] + 1) for d in range(nd)], indexing="ij")
    masks = []
    for fd, dom in enumerate(frag_dom):
        m = np.ones(grids[0].shape, dtype=bool) if present[fd] else np.zeros(grids[0].shape, dtype=bool)
        for d in range(nd):
            m &= (grids[d] >= dom[d][0]) & (grids[d] <= dom[d][1])
        masks.append(m)
    return src, dst, masks


def dense_copy_fragments(tiles, tile_start, tile_extent, cell_size: int, sub_lo, sub_hi, frag_dom, fill_value,
                         cell_order: int = 0, layout: int = 0, validity=None, fill_validity: int = 0):
    """DenseReader::copy_fixed_tiles (dense_reader.cc:1555-1750) with several
    fragments: tiles[t][fd] is fragment fd's unfiltered tile of space tile t
    (None: no tile), frag_dom[fd] its domain ((lo, hi) per dimension).  The
    reference walks the fragment domains from the last to the first, each
    copying the cells it overlaps over what the later ones wrote
    (:1600-1660), and fills the cells the last domain does not write with the
    fill value (:1676-1702), or the whole slab when there is no fragment
    (:1708-1719).  Returns the result bytes (and validity bytes when
    `validity` holds per-(t, fd) validity tiles)."""
    nd = len(tile_extent)
    ext = [int(e) for e in tile_extent]
    lo = [int(x) for x in sub_lo]
    hi = [int(x) for x in sub_hi]
    shape = tuple(h - l + 1 for l, h in zip(lo, hi))
    fill = np.frombuffer(bytes(fill_value), dtype=np.uint8)
    assert fill.size == cell_size
    out = np.zeros(shape + (cell_size,), dtype=np.uint8)
    outv = np.zeros(shape, dtype=np.uint8)
    F = len(frag_dom)
    for t in range(len(tiles)):
        s = [int(x) for x in tile_start[t]]
        present = [tiles[t][fd] is not None for fd in range(F)]
        r = _frag_masks(s, ext, lo, hi, frag_dom, present)
        if r is None:
            continue
        src, dst, masks = r
        reg = out[dst]
        regv = outv[dst]
        if F == 0:
            reg[...] = fill
            regv[...] = fill_validity
        for fd in range(F - 1, -1, -1):
            m = masks[fd]
            if present[fd]:
                reg[m] = _tile_cells(tiles[t][fd], ext, cell_size, cell_order)[src][m]
                if validity is not None:
                    regv[m] = _tile_cells(validity[t][fd], ext, 1, cell_order)[src][..., 0][m]
            if fd == F - 1:
                reg[~m] = fill
                regv[~m] = fill_validity
        out[dst] = reg
        outv[dst] = regv
    if layout == 1:
        out = np.transpose(out, tuple(reversed(range(nd))) + (nd,))
        outv = np.transpose(outv, tuple(reversed(range(nd))))
    res = np.ascontiguousarray(out).reshape(-1)
    return (res, np.ascontiguousarray(outv).reshape(-1)) if validity is not None else res


def dense_var_read(off_tiles, var_tiles, tile_start, tile_extent, sub_lo, sub_hi, frag_dom, fill_value,
                   cell_order: int = 0, layout: int = 0, elements_mode: bool = False, type_size: int = 1):
    """The dense read of a var-sized attribute with several fragments:
    DenseReader::copy_offset_tiles (dense_reader.cc:1753-1926) writes each
    result cell's size (offsets tile entries i + 1 - i, of the unfiltered
    offsets tile with its extra offset, tile.h:144-146; divided by the type
    size in elements mode) and the address of its bytes in the var tile, or
    the max sentinel for cells no fragment writes; fix_offsets_buffer
    (:1199-1236) turns the sizes into offsets (a sentinel becomes the fill
    value's size and the fill value's bytes); copy_var_tiles (:1929-2000)
    copies each cell's bytes to its offset (times the type size in elements
    mode).  off_tiles[t][fd] / var_tiles[t][fd]: fragment fd's unfiltered
    offsets tile (uint64, cells + 1 entries) and var tile of space tile t.
    Returns (offsets as uint64 in result order, var bytes)."""
    nd = len(tile_extent)
    ext = [int(e) for e in tile_extent]
    lo = [int(x) for x in sub_lo]
    hi = [int(x) for x in sub_hi]
    shape = tuple(h - l + 1 for l, h in zip(lo, hi))
    F = len(frag_dom)
    SENT = (1 << 64) - 1
    size = np.full(shape, SENT, dtype=np.uint64)
    ref_t = np.full(shape, -1, dtype=np.int64)   # (t, fd, var byte offset) of each cell's bytes
    ref_f = np.full(shape, -1, dtype=np.int64)
    ref_o = np.zeros(shape, dtype=np.uint64)
    div = type_size if elements_mode else 1
    for t in range(len(off_tiles)):
        s = [int(x) for x in tile_start[t]]
        present = [off_tiles[t][fd] is not None for fd in range(F)]
        r = _frag_masks(s, ext, lo, hi, frag_dom, present)
        if r is None:
            continue
        src, dst, masks = r
        for fd in range(F - 1, -1, -1):
            m = masks[fd]
            if present[fd]:
                offs = np.frombuffer(bytes(off_tiles[t][fd]), dtype=np.uint64)
                ncell = int(np.prod(ext))
                pos = np.arange(ncell, dtype=np.int64).reshape(tuple(ext) if cell_order == 0 else tuple(reversed(ext)))
                if cell_order == 1:
                    pos = np.transpose(pos)
                p = pos[src]
                sz = (offs[p + 1] - offs[p]) // np.uint64(div)
                size[dst][m] = sz[m]
                ref_t[dst][m] = t
                ref_f[dst][m] = fd
                ref_o[dst][m] = offs[p][m]
            if fd == F - 1:
                size[dst][~m] = SENT
                ref_t[dst][~m] = -1
        if F == 0:
            size[dst] = SENT
            ref_t[dst] = -1
    if layout == 1:
        size, ref_t, ref_f, ref_o = (np.transpose(x) for x in (size, ref_t, ref_f, ref_o))
    size, ref_t, ref_f, ref_o = (np.ascontiguousarray(x).reshape(-1) for x in (size, ref_t, ref_f, ref_o))
    fill = bytes(fill_value)
    fill_sz = len(fill) // type_size if elements_mode else len(fill)
    offsets = np.zeros(size.size, dtype=np.uint64)
    total = 0
    for i in range(size.size):  # fix_offsets_buffer
        v = int(size[i])
        if v == SENT:
            v = fill_sz
            ref_t[i] = -1
        offsets[i] = total
        total += v
    mult = type_size if elements_mode else 1
    data = bytearray(total * mult)
    for i in range(size.size):  # copy_var_tiles
        o = int(offsets[i]) * mult
        n = (int(offsets[i + 1]) if i + 1 < size.size else total) * mult - o
        if ref_t[i] < 0:
            data[o:o + n] = fill[:n]
        else:
            vt = bytes(var_tiles[int(ref_t[i])][int(ref_f[i])])
            b = int(ref_o[i])
            data[o:o + n] = vt[b:b + n]
    return offsets, bytes(data)
