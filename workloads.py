"""Synthetic BASELINE workloads for bench.py (numpy, independent of oracle/).

Writes on-disk filtered tiles for every BASELINE config: C1
[BYTESHUFFLE], C2/C2i [BITSHUFFLE, BWR], C3a [DD], C3b [RLE], C4 [PD, BWR] and
the headline C5 [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION(256)] on
INT32, restating the forward direction of
  ByteshuffleFilter::run_forward      byteshuffle_filter.cc:60-89
  CompressionFilter::run_forward      compression_filter.cc:240-301
  DoubleDelta::compress<int>          dd_compressor.cc:211-312
  BitWidthReductionFilter::run_forward<int> bit_width_reduction_filter.cc:167-280
  FilterPipeline::filter_chunks_forward     filter_pipeline.cc:208-369
as vectorized numpy.  tests/test_oracle.py checks it byte-for-byte against
the oracle's forward pass, which makes it a second, independent restatement.
"""
from __future__ import annotations

import struct
from typing import List, Tuple

import numpy as np

TILE_VALUES = 16384          # 64 KiB of int32 per tile (one 64 KiB chunk)
TILE_BYTES = TILE_VALUES * 4
C5S_VALUES = 10000           # bench.py --config c5s: 40,000-B tiles


def _dd_int32(v: np.ndarray) -> bytes:
    """DoubleDelta::compress<int> of one part (values as int32)."""
    n = v.size
    x = v.astype(np.int64)
    if n <= 2:
        b = 0
    else:
        d = np.diff(x)
        dd = np.diff(d)
        m = max(int(np.abs(d[0])), int(np.abs(dd).max()) if dd.size else 0)
        b = max(1, int(m).bit_length())
    hdr = struct.pack("<BQ", b, n)
    if b >= 31:
        return hdr + v.astype("<i4").tobytes()
    out = hdr + v[:2].astype("<i4").tobytes()[: 4 * min(n, 2)]
    if n <= 2:
        return out
    d = np.diff(x)
    dd = np.diff(d)
    sign = (dd < 0).astype(np.uint8)
    mag = np.abs(dd).astype(np.uint64)
    shifts = np.arange(b - 1, -1, -1, dtype=np.uint64)
    bits = ((mag[:, None] >> shifts[None, :]) & np.uint64(1)).astype(np.uint8)
    codes = np.concatenate([sign[:, None], bits], axis=1).reshape(-1)
    pad = (-codes.size) % 64
    codes = np.concatenate([codes, np.zeros(pad, dtype=np.uint8)])
    be = np.packbits(codes.reshape(-1, 64), axis=1, bitorder="big")  # MSB-first per word
    words = be.view(">u8").reshape(-1).astype("<u8")
    return out + words.tobytes()


def _bwr_int32(data: bytes, window: int = 256) -> Tuple[bytes, bytes]:
    """BitWidthReductionFilter::run_forward<int> of one part -> (md, data)."""
    L = len(data)
    ws = min(L, window) // 4 * 4
    nwin = L // ws + (1 if L % ws else 0)
    md = [struct.pack("<II", L, nwin)]
    out = []
    buf = np.frombuffer(data, dtype=np.uint8)
    for k in range(nwin):
        nb = min(ws, L - k * ws)
        ne = nb // 4
        seg = buf[k * ws: k * ws + nb]
        bits, minv = 32, 0
        if ne:
            vals = seg[: ne * 4].view("<i4").astype(np.int64)
            mn, mx = int(vals.min()), int(vals.max())
            rng = mx - mn
            if not (rng > 2**31 - 1 or rng + 1 > 2**31 - 1):
                ro = rng + 1
                bits = 8 if ro <= 127 else 16 if ro <= 32767 else 32 if ro <= 2**31 - 1 else 64
                minv = mn
        md.append(struct.pack("<iBI", minv, bits, nb))
        if bits >= 32 or nb % 4:
            out.append(seg.tobytes())
        else:
            rel = vals - minv
            out.append(rel.astype("<i1" if bits == 8 else "<i2").tobytes())
    return b"".join(md), b"".join(out)


def c5_filter_tile(values: np.ndarray) -> bytes:
    """One C5 tile (int32 values, <= 64 KiB -> one chunk) in the on-disk layout."""
    raw = np.ascontiguousarray(values, dtype="<i4")
    nbytes = raw.nbytes
    # byteshuffle: md [u32 nparts][u32 size]
    shuf = raw.view(np.uint8).reshape(-1, 4).T.reshape(-1).tobytes()
    bs_md = struct.pack("<II", 1, nbytes)
    # DD over md part (as int32) and data part
    c0 = _dd_int32(np.frombuffer(bs_md, dtype="<i4"))
    c1 = _dd_int32(np.frombuffer(shuf, dtype="<i4"))
    dd_md = struct.pack("<IIIIII", 1, 1, len(bs_md), len(c0), nbytes, len(c1))
    bwr_md, bwr_data = _bwr_int32(c0 + c1, 256)
    md = bwr_md + dd_md
    return struct.pack("<QIII", 1, nbytes, len(bwr_data), len(md)) + md + bwr_data


# ---------------------------------------------------------------------------
# generic forward restatements (numpy) for the other BASELINE configs
# ---------------------------------------------------------------------------
_UT = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}
_ST = {1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}


def tile_image(orig: int, md: bytes, data: bytes) -> bytes:
    """One-chunk tile: [u64 1][u32 orig][u32 filtered][u32 md_len][md][data]
    (filter_pipeline.cc:332-363, format_spec/tile.md)."""
    return struct.pack("<QIII", 1, orig, len(data), len(md)) + md + data


def byteshuffle_fwd(data: bytes, ts: int) -> bytes:
    """blosc2 generic shuffle (byteshuffle_filter.cc:97): byte planes, tail kept."""
    b = np.frombuffer(data, dtype=np.uint8)
    n = b.size // ts
    body = b[: n * ts].reshape(n, ts).T.reshape(-1)
    return body.tobytes() + b[n * ts:].tobytes()


def bitshuffle_fwd(data: bytes, ts: int) -> Tuple[bytes, bytes]:
    """BitshuffleFilter::run_forward (bitshuffle_filter.cc:60-126) -> (md, data):
    parts [size - size%8][size%8]; a part is transformed in 8192-B blocks when
    size % 8 == 0 and size % ts == 0 (bit planes of the first n - n%8 elements)."""
    b = np.frombuffer(data, dtype=np.uint8)
    parts = [b[: b.size - b.size % 8]] + ([b[b.size - b.size % 8:]] if b.size % 8 else [])
    out = []
    for part in parts:
        if part.size % 8 or part.size % ts:
            out.append(part.tobytes())
            continue
        for o in range(0, part.size, 8192):
            blk = part[o:o + 8192]
            ne = blk.size // ts
            n8 = ne - ne % 8
            x = blk[: n8 * ts].reshape(n8, ts)
            bits = np.unpackbits(x, axis=1, bitorder="little")          # (n8, 8ts): col 8b+k
            planes = np.packbits(bits.T, axis=1, bitorder="little")      # (8ts, n8/8)
            out.append(planes.tobytes() + blk[n8 * ts:].tobytes())
    md = struct.pack("<I", len(parts)) + b"".join(struct.pack("<I", p.size) for p in parts)
    return md, b"".join(out)


def bwr_fwd(data: bytes, window: int, w: int, signed: bool) -> Tuple[bytes, bytes]:
    """BitWidthReductionFilter::run_forward<T> (bit_width_reduction_filter.cc:167-280,
    406-447); the offset of an overflowing window is written as 0 (the reference
    leaves it uninitialized)."""
    L = len(data)
    ws = min(L, window) // w * w
    nwin = L // ws + (1 if L % ws else 0)
    md = [struct.pack("<II", L, nwin)]
    out = []
    buf = np.frombuffer(data, dtype=np.uint8)
    lim = (1 << (8 * w - 1)) - 1 if signed else (1 << (8 * w)) - 1
    for k in range(nwin):
        nb = min(ws, L - k * ws)
        ne = nb // w
        seg = buf[k * ws: k * ws + nb]
        bits, minv = 8 * w, 0
        if ne:
            vals = seg[: ne * w].view(("<i" if signed else "<u") + str(w))
            mn, mx = int(vals.min()), int(vals.max())
            rng = mx - mn
            if rng <= lim and rng + 1 <= lim:
                ro = rng + 1
                if signed:
                    bits = 8 if ro <= 127 else 16 if ro <= 32767 else 32 if ro <= 2**31 - 1 else 64
                else:
                    nbits = ro.bit_length()
                    bits = 8 if nbits <= 8 else 16 if nbits <= 16 else 32 if nbits <= 32 else 64
                minv = mn
        fmt = "<" + ({1: "b", 2: "h", 4: "i", 8: "q"} if signed else {1: "B", 2: "H", 4: "I", 8: "Q"})[w]
        md.append(struct.pack(fmt, minv) + struct.pack("<BI", bits, nb))
        if bits >= 8 * w or nb % w:
            out.append(seg.tobytes())
        else:
            rel = (vals.astype(np.int64 if signed else np.uint64) -
                   np.array(minv, dtype=np.int64 if signed else np.uint64))
            out.append(rel.astype(_UT[bits // 8]).tobytes())
    return b"".join(md), b"".join(out)


def dd_fwd(v: np.ndarray, w: int) -> bytes:
    """DoubleDelta::compress<T> (dd_compressor.cc:211-312); v holds the T values."""
    n = v.size
    x = v.astype(np.int64)
    if n <= 2:
        b = 0
    else:
        d = np.diff(x)
        dd = np.diff(d)
        m = max(int(np.abs(d[0])), int(np.abs(dd).max()) if dd.size else 0)
        b = max(1, int(m).bit_length())
    hdr = struct.pack("<BQ", b, n)
    raw = v.astype(("<u" if v.dtype.kind == "u" else "<i") + str(w)).tobytes()
    if b >= 8 * w - 1:
        return hdr + raw
    out = hdr + raw[: w * min(n, 2)]
    if n <= 2:
        return out
    d = np.diff(x)
    dd = np.diff(d)
    sign = (dd < 0).astype(np.uint8)
    mag = np.abs(dd).astype(np.uint64)
    shifts = np.arange(b - 1, -1, -1, dtype=np.uint64)
    bits = ((mag[:, None] >> shifts[None, :]) & np.uint64(1)).astype(np.uint8)
    codes = np.concatenate([sign[:, None], bits], axis=1).reshape(-1)
    pad = (-codes.size) % 64
    codes = np.concatenate([codes, np.zeros(pad, dtype=np.uint8)])
    be = np.packbits(codes.reshape(-1, 64), axis=1, bitorder="big")  # MSB-first per word
    return out + be.view(">u8").reshape(-1).astype("<u8").tobytes()


def rle_fwd(data: bytes, cs: int) -> bytes:
    """RLE::compress (rle_compressor.cc:51-101): [value][len_hi][len_lo], runs <= 65535."""
    v = np.frombuffer(data, dtype=np.uint8).reshape(-1, cs)
    keys = v.view(np.dtype((np.void, cs))).reshape(-1)
    starts = np.concatenate([[0], np.nonzero(keys[1:] != keys[:-1])[0] + 1, [keys.size]])
    out = []
    for a, e in zip(starts[:-1], starts[1:]):
        n = int(e - a)
        while n > 0:
            k = min(n, 65535)
            out.append(v[a].tobytes() + bytes([k >> 8, k & 255]))
            n -= k
    return b"".join(out)


def pd_fwd(data: bytes, window: int, w: int) -> Tuple[bytes, bytes]:
    """PositiveDeltaFilter::run_forward<T> (positive_delta_filter.cc:140-245);
    the input is nondecreasing (offsets), so no window errors."""
    L = len(data)
    ws = min(L, window) // w * w
    nwin = L // ws + (1 if L % ws else 0)
    buf = np.frombuffer(data, dtype=np.uint8)
    md, out = [struct.pack("<I", nwin)], []
    for k in range(nwin):
        nb = min(ws, L - k * ws)
        seg = buf[k * ws: k * ws + nb]
        first = seg[:w].tobytes() if seg.size >= w else seg.tobytes().ljust(w, b"\0")
        md.append(first + struct.pack("<I", nb))
        if nb % w:
            out.append(seg.tobytes())
        else:
            vals = seg.view("<u" + str(w)).astype(np.uint64)
            d = np.diff(vals, prepend=vals[:1])
            out.append(d.astype(_UT[w]).tobytes())
    return b"".join(md), b"".join(out)


def comp_frame(md_parts, data_parts) -> bytes:
    """CompressionFilter metadata (compression_filter.cc:269-300)."""
    h = struct.pack("<II", len(md_parts), len(data_parts))
    return h + b"".join(struct.pack("<II", u, c) for u, c in list(md_parts) + list(data_parts))


# ---------------------------------------------------------------------------
# BASELINE configs C1-C4; values per config, tiles on disk
# ---------------------------------------------------------------------------
def c1_values(variant: str, k: int, rng: np.random.Generator) -> np.ndarray:
    """2D int32 2048x2048, 128x128 tiles: a[r][c] = r*2048 + c + 1 (ramp)."""
    if variant == "rand":
        return rng.integers(-2**31, 2**31, 16384, dtype=np.int64).astype(np.int32)
    tr, tc = divmod(k % 256, 16)
    r = np.arange(128)[:, None] + 128 * tr
    c = np.arange(128)[None, :] + 128 * tc
    return (r * 2048 + c + 1).astype(np.int32).reshape(-1)


def c1_tile(v: np.ndarray) -> bytes:
    raw = v.astype("<i4").tobytes()
    return tile_image(len(raw), struct.pack("<II", 1, len(raw)), byteshuffle_fwd(raw, 4))


def c2_values(k: int, rng: np.random.Generator) -> np.ndarray:
    g = np.arange(16384, dtype=np.float64) + 16384 * k
    return (1000.0 * np.sin(1e-3 * g) + rng.normal(0, 0.01, 16384)).astype(np.float32)


def c2_tile(v: np.ndarray, int_typed: bool) -> bytes:
    raw = v.tobytes()
    bmd, bdata = bitshuffle_fwd(raw, 4)
    if not int_typed:  # BWR on FLOAT32 is a pass-through (bwr.cc:166-176)
        return tile_image(len(raw), bmd, bdata)
    wmd, wdata = bwr_fwd(bdata, 256, 4, True)
    return tile_image(len(raw), wmd + bmd, wdata)


def c3_values(k: int, rng: np.random.Generator) -> np.ndarray:
    """Sorted uint64 coords: runs of 64 equal values, gaps U{1..16}."""
    steps = np.zeros(8192, dtype=np.uint64)
    steps[64::64] = rng.integers(1, 17, 8192 // 64 - 1).astype(np.uint64)
    return np.uint64(1000 * k) + np.cumsum(steps, dtype=np.uint64)


def c3a_tile(v: np.ndarray) -> bytes:
    c = dd_fwd(v, 8)
    return tile_image(v.nbytes, comp_frame([], [(v.nbytes, len(c))]), c)


def c3b_tile(v: np.ndarray) -> bytes:
    c = rle_fwd(v.astype("<u8").tobytes(), 8)
    return tile_image(v.nbytes, comp_frame([], [(v.nbytes, len(c))]), c)


def c4_values(k: int, rng: np.random.Generator) -> np.ndarray:
    lens = rng.integers(0, 33, 8192).astype(np.uint64)
    offs = np.zeros(8192, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return offs


def c4_tile(v: np.ndarray) -> bytes:
    raw = v.astype("<u8").tobytes()
    pmd, pdata = pd_fwd(raw, 1024, 8)
    wmd, wdata = bwr_fwd(pdata, 256, 8, False)
    return tile_image(len(raw), wmd + pmd, wdata)


def config(name: str):
    """(serialized pipeline, on-disk datatype, cell size, values(variant, k, rng), tile(values))."""
    from tiledb_amd.filter_pipeline import (BitshuffleFilter, BitWidthReductionFilter,
                                            ByteshuffleFilter, CompressionFilter, Compressor,
                                            Datatype, FilterPipeline, FloatScalingFilter,
                                            PositiveDeltaFilter, XORFilter)
    dd = CompressionFilter(Compressor.DOUBLE_DELTA, -1)
    rle = CompressionFilter(Compressor.RLE, -1)
    P = lambda *f: FilterPipeline(65536, list(f)).serialize()  # noqa: E731
    table = {
        "c1": (P(ByteshuffleFilter()), Datatype.INT32, 4, c1_values, c1_tile),
        "c2": (P(BitshuffleFilter(), BitWidthReductionFilter(256)), Datatype.FLOAT32, 4,
               lambda var, k, rng: c2_values(k, rng), lambda v: c2_tile(v, False)),
        "c2i": (P(BitshuffleFilter(), BitWidthReductionFilter(256)), Datatype.INT32, 4,
                lambda var, k, rng: c2_values(k, rng), lambda v: c2_tile(v, True)),
        "c3a": (P(dd), Datatype.UINT64, 8, lambda var, k, rng: c3_values(k, rng), c3a_tile),
        "c3b": (P(rle), Datatype.UINT64, 8, lambda var, k, rng: c3_values(k, rng), c3b_tile),
        "c4": (P(PositiveDeltaFilter(1024), BitWidthReductionFilter(256)), Datatype.UINT64, 8,
               lambda var, k, rng: c4_values(k, rng), c4_tile),
        "c5": (c5_pipeline_bytes(), Datatype.INT32, 4, c5_values, c5_filter_tile),
        # C5's pipeline over 40,000-B tiles (10,000 values: one chunk that is
        # not 64 KiB, planes not 16-B aligned in the BWR output)
        "c5s": (c5_pipeline_bytes(), Datatype.INT32, 4,
                lambda var, k, rng: c5_values(var, k, rng, C5S_VALUES), c5_filter_tile),
        # C5's pipeline over 4 MiB tiles (64 chunks of 64 KiB): the chunk-
        # parallel launch (device chunk directory) against tile-serial chunks
        "c5big": (c5_pipeline_bytes(), Datatype.INT32, 4,
                  lambda var, k, rng: np.concatenate([c5_values(var, 64 * k + i, rng) for i in range(64)]),
                  c5_multi_tile),
        # XOR / DELTA / FLOAT_SCALE pipelines: tiles are
        # encoded by the device forward path (tile = None; bench.py)
        "xor": (P(XORFilter(), BitWidthReductionFilter(256)), Datatype.FLOAT32, 4,
                lambda var, k, rng: c2_values(k, rng), None),
        "delta": (P(ByteshuffleFilter(), CompressionFilter(Compressor.DELTA, -1), BitWidthReductionFilter(256)),
                  Datatype.INT32, 4, c5_values, None),
        "fscale": (P(FloatScalingFilter(1e-3, 0.0, 4), BitWidthReductionFilter(256)), Datatype.FLOAT64, 8,
                   lambda var, k, rng: np.sin(1e-2 * np.arange(8192) + k) + rng.normal(0, 1e-4, 8192), None),
    }
    return table[name]


def expected(name: str, v: np.ndarray) -> np.ndarray:
    """The values an unfilter of the config's tiles returns: the input, except
    FLOAT_SCALE's lossy quantization (float_scaling_filter.cc:60-99, 164-197:
    q = round((x - offset) / scale) to the stored width, then
    scale * double(q) + offset, each operation rounded once)."""
    if name != "fscale":
        return v
    q = (v - 0.0) / 1e-3
    q = (np.sign(q) * np.floor(np.abs(q) + 0.5)).astype(np.int64).astype(np.int32)  # std::round
    return 1e-3 * q.astype(np.float64) + 0.0


def pool(name: str, variant: str, nunique: int, seed: int, encode=None):
    """nunique distinct on-disk tiles of a config + their unfiltered values.
    Configs without a numpy encoder take `encode(values list) -> tiles`."""
    ser, dt, cs, values, tile = config(name)
    rng = np.random.default_rng(seed)
    vals = [values(variant, k, rng) for k in range(nunique)]
    if tile is None:
        if encode is None:
            raise ValueError(f"{name}: tiles are encoded by the device forward path")
        return encode(vals), vals
    return [tile(v) for v in vals], vals


def c5_values(variant: str, tile_index: int, rng: np.random.Generator, n: int = TILE_VALUES) -> np.ndarray:
    """C5 tile values (n of them: 16,384 for a 64 KiB tile).
    rand:   uniform int32; every byte moves, DD falls back to raw and every BWR
            window is raw (two stages are views).
    ramp:   a = tile*16384 + i; DD raw (bitsize 33 >= 31), half the BWR windows
            8-bit.
    active: a low-cardinality step column (runs of U{256..2047} equal values,
            values U{0..15}): all three stages do work -- DoubleDelta bitsize 28
            (< 31: the bit-packed path), ~92 % of the BWR windows over DD's
            output 8-bit, byteshuffle over the whole tile (~20 KB filtered).
    walk:   dense codes -- the byteshuffled stream is a random walk (steps
            U{-500..500}), so DoubleDelta codes are nonzero almost everywhere
            (the bit-packed path with no all-zero wave) and the BWR windows over
            DD's output are mostly raw.  Not a BASELINE variant: the bench's
            c5_dense_codes leg, the coded path's rate when no wave can skip its
            codes."""
    if variant == "walk":
        steps = rng.integers(-500, 501, n).astype(np.int64)
        s = (np.cumsum(steps) + int(rng.integers(-2**20, 2**20))).astype(np.int32)
        # the values whose 4-byte byteshuffle is s
        return s.astype("<i4").view(np.uint8).reshape(4, n).T.reshape(-1).view("<i4").copy()
    if variant == "ramp":
        return (np.arange(n, dtype=np.int64) + tile_index * n).astype(np.int32)
    if variant == "rand":
        return rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    if variant == "active":
        out = np.empty(n, dtype=np.int32)
        i = 0
        while i < n:
            run = int(rng.integers(256, 2048))
            out[i:i + run] = rng.integers(0, 16)
            i += run
        return out
    raise ValueError(variant)


def c5_multi_tile(values: np.ndarray) -> bytes:
    """A C5 tile of several 64 KiB chunks: WriterTile's chunking
    (tile.cc:87-100) cuts the tile at 16,384 int32 values, and each chunk
    record is the one a single-chunk tile of those values holds."""
    recs = [c5_filter_tile(values[i:i + TILE_VALUES])[8:] for i in range(0, values.size, TILE_VALUES)]
    return struct.pack("<Q", len(recs)) + b"".join(recs)


def c5_dd_bitsize(values: np.ndarray) -> int:
    """DoubleDelta bitsize of a C5 tile's data part (after the byteshuffle)."""
    raw = np.ascontiguousarray(values, dtype="<i4")
    shuf = raw.view(np.uint8).reshape(-1, 4).T.reshape(-1)
    return _dd_int32(shuf.view("<i4"))[0]


def c5_pool(variant: str, nunique: int, seed: int = 5) -> Tuple[List[bytes], List[np.ndarray]]:
    rng = np.random.default_rng(seed)
    vals = [c5_values(variant, k, rng) for k in range(nunique)]
    return [c5_filter_tile(v) for v in vals], vals


def c5_pipeline_bytes() -> bytes:
    """Serialized [BYTESHUFFLE, DOUBLE_DELTA(ANY), BIT_WIDTH_REDUCTION(256)]."""
    from tiledb_amd.filter_pipeline import (BitWidthReductionFilter, ByteshuffleFilter,
                                            CompressionFilter, Compressor, FilterPipeline)
    return FilterPipeline(65536, [ByteshuffleFilter(), CompressionFilter(Compressor.DOUBLE_DELTA, -1),
                                  BitWidthReductionFilter(256)]).serialize()
