"""Synthetic BASELINE workloads for bench.py (numpy, independent of oracle/).

Writes on-disk filtered tiles for the C5 pipeline
[BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION(256)] on INT32,
restating the forward direction of
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


def c5_values(variant: str, tile_index: int, rng: np.random.Generator) -> np.ndarray:
    if variant == "ramp":
        return (np.arange(TILE_VALUES, dtype=np.int64) + tile_index * TILE_VALUES).astype(np.int32)
    if variant == "rand":
        return rng.integers(-2**31, 2**31, TILE_VALUES, dtype=np.int64).astype(np.int32)
    raise ValueError(variant)


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
