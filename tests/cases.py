"""Parity cases: BASELINE.json configs C1-C5 at test sizes,
the edge-case list of SURVEY.md A.5, and random pipelines in the style of
tiledb/sm/filter/test/unit_run_filter_pipeline.cc:800-912.

A case is an unfiltered tile set + a pipeline; the oracle's forward pass
(FilterPipeline::run_forward restated) produces the on-disk tiles, which the
oracle and the GPU then unfilter.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from tiledb_amd.filter_pipeline import (FORMAT_VERSION, BitshuffleFilter, BitWidthReductionFilter,
                                        ByteshuffleFilter, CompressionFilter, Compressor, Datatype,
                                        FilterPipeline, NoopFilter, PositiveDeltaFilter,
                                        FloatScalingFilter, XORFilter, datatype_size)


@dataclass
class Case:
    name: str
    pipeline: FilterPipeline
    dtype: int
    cell_size: int
    tiles: List[np.ndarray]
    version: int = FORMAT_VERSION
    max_chunk: int = 0           # WriterTile::max_tile_chunk_size_ override (0 = 64 KiB)
    offsets: Optional[List[np.ndarray]] = None  # var-size chunking offsets per tile
    offsets_tile: bool = False   # tile is an offsets tile (expected size - 8)
    extra: dict = field(default_factory=dict)

    @property
    def serialized(self) -> bytes:
        return self.pipeline.serialize()


def P(*filters, max_chunk_size: int = 65536) -> FilterPipeline:
    return FilterPipeline(max_chunk_size, filters)


def DD(reinterpret=Datatype.ANY):
    return CompressionFilter(Compressor.DOUBLE_DELTA, -1, reinterpret_datatype=reinterpret)


def RLE():
    return CompressionFilter(Compressor.RLE, -1)


def DELTA(reinterpret=Datatype.ANY):
    return CompressionFilter(Compressor.DELTA, -1, reinterpret_datatype=reinterpret)


def as_u8(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a).view(np.uint8).reshape(-1)


# ---------------------------------------------------------------------------
# BASELINE configs (data per SURVEY.md 8(d))
# ---------------------------------------------------------------------------
def c1_tiles(ntiles: int, variant: str = "ramp", seed: int = 1) -> List[np.ndarray]:
    """2D int32 dense 2048x2048, 128x128 tiles; a[r][c] = r*2048 + c + 1."""
    out = []
    rng = np.random.default_rng(seed)
    per_row = 2048 // 128
    for t in range(ntiles):
        tr, tc = divmod(t % (per_row * per_row), per_row)
        if variant == "ramp":
            r = np.arange(128, dtype=np.int64)[:, None] + tr * 128
            c = np.arange(128, dtype=np.int64)[None, :] + tc * 128
            a = (r * 2048 + c + 1).astype(np.int32)
        else:
            a = rng.integers(-2**31, 2**31, size=(128, 128), dtype=np.int64).astype(np.int32)
        out.append(as_u8(a))
    return out


def c2_tiles(ntiles: int, n: int = 16384, seed: int = 2) -> List[np.ndarray]:
    rng = np.random.default_rng(seed)
    out = []
    for t in range(ntiles):
        g = np.arange(n, dtype=np.float64) + t * n
        v = (1000.0 * np.sin(1e-3 * g) + rng.normal(0, 0.01, n)).astype(np.float32)
        out.append(as_u8(v))
    return out


def c3_tiles(ntiles: int, n: int = 8192, seed: int = 3) -> List[np.ndarray]:
    """Sorted uint64 coords, runs of 64, gaps U{1..16}."""
    rng = np.random.default_rng(seed)
    out = []
    for t in range(ntiles):
        gaps = np.where(np.arange(n) % 64 == 0, rng.integers(1, 17, n), 0).astype(np.uint64)
        gaps[0] = 0
        x = np.uint64(1000 * t) + np.cumsum(gaps, dtype=np.uint64)
        out.append(as_u8(x))
    return out


def c4_tiles(ntiles: int, n: int = 8192, seed: int = 4) -> List[np.ndarray]:
    """Var-length attribute offsets: start 0, lengths U{0..32}."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(ntiles):
        lens = rng.integers(0, 33, n).astype(np.uint64)
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        out.append(as_u8(offs))
    return out


def c5_tiles(ntiles: int, variant: str = "ramp", n: int = 16384, seed: int = 5) -> List[np.ndarray]:
    rng = np.random.default_rng(seed)
    out = []
    for t in range(ntiles):
        if variant == "ramp":
            a = (np.arange(n, dtype=np.int64) + t * n).astype(np.int32)
        else:
            a = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
        out.append(as_u8(a))
    return out


def config_cases(ntiles: int = 4) -> List[Case]:
    I32, U64, F32 = Datatype.INT32, Datatype.UINT64, Datatype.FLOAT32
    return [
        Case("C1_ramp", P(ByteshuffleFilter()), I32, 4, c1_tiles(ntiles, "ramp")),
        Case("C1_rand", P(ByteshuffleFilter()), I32, 4, c1_tiles(ntiles, "rand")),
        Case("C2_float", P(BitshuffleFilter(), BitWidthReductionFilter(256)), F32, 4,
             c2_tiles(ntiles)),
        Case("C2i_int32", P(BitshuffleFilter(), BitWidthReductionFilter(256)), I32, 4,
             c2_tiles(ntiles)),
        Case("C3a_dd", P(DD()), U64, 8, c3_tiles(ntiles)),
        Case("C3b_rle", P(RLE()), U64, 8, c3_tiles(ntiles)),
        Case("C4_pd_bwr", P(PositiveDeltaFilter(1024), BitWidthReductionFilter(256)), U64, 8,
             c4_tiles(ntiles)),
        Case("C5_ramp", P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256)), I32, 4,
             c5_tiles(ntiles, "ramp")),
        Case("C5_rand", P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256)), I32, 4,
             c5_tiles(ntiles, "rand")),
    ]


# ---------------------------------------------------------------------------
# Edge cases
# ---------------------------------------------------------------------------
def edge_cases() -> List[Case]:
    rng = np.random.default_rng(11)
    I32, U64, I64 = Datatype.INT32, Datatype.UINT64, Datatype.INT64
    cases: List[Case] = []
    ramp64 = as_u8(np.arange(1000, dtype=np.uint64))
    cases.append(Case("empty_pipeline", P(), U64, 8, [ramp64]))
    # DD n <= 2 (dd_compressor.cc:240-247)
    for n in (1, 2, 3, 4):
        cases.append(Case(f"dd_n{n}", P(DD()), I64, 8,
                          [as_u8(np.array([5, -7, 9, 100][:n], dtype=np.int64))]))
    # tails not divisible by 8 / by ts (unit_bitshuffle_pipeline.cc: 1001 uint32)
    t1001 = as_u8(rng.integers(0, 2**32, 1001, dtype=np.uint64).astype(np.uint32))
    cases.append(Case("bitshuffle_1001_u32", P(BitshuffleFilter()), Datatype.UINT32, 4, [t1001]))
    cases.append(Case("byteshuffle_1001_u32", P(ByteshuffleFilter()), Datatype.UINT32, 4, [t1001]))
    for ts_dt, n in ((Datatype.INT16, 777), (Datatype.INT64, 333), (Datatype.UINT8, 999)):
        sz = datatype_size(ts_dt)
        data = rng.integers(0, 256, n * sz, dtype=np.uint8)
        cases.append(Case(f"bitshuffle_{ts_dt.name}_{n}", P(BitshuffleFilter()), ts_dt, sz, [data]))
        cases.append(Case(f"byteshuffle_{ts_dt.name}_{n}", P(ByteshuffleFilter()), ts_dt, sz, [data]))
    # bitshuffle multi-block (8192-B blocks) with a partial last block
    big = rng.integers(0, 256, 8192 * 3 + 424, dtype=np.uint8)
    cases.append(Case("bitshuffle_blocks_u64", P(BitshuffleFilter()), U64, 8, [big]))
    # BWR windows (unit_bit_width_reduction_pipeline.cc:106-108)
    inc = as_u8(np.arange(1000, dtype=np.uint64))
    for w in (32, 64, 128, 256, 437, 512, 1024, 2000):
        cases.append(Case(f"bwr_window_{w}", P(BitWidthReductionFilter(w)), U64, 8, [inc]))
    sv = as_u8(rng.integers(-200, 200, 1000).astype(np.int32))
    cases.append(Case("bwr_signed_i32", P(BitWidthReductionFilter(128)), I32, 4, [sv]))
    s16 = as_u8(rng.integers(-30000, 30000, 999).astype(np.int16))
    cases.append(Case("bwr_signed_i16", P(BitWidthReductionFilter(64)), Datatype.INT16, 2, [s16]))
    u16 = as_u8(rng.integers(0, 65536, 1001).astype(np.uint16))
    cases.append(Case("bwr_u16_tail", P(BitWidthReductionFilter(100)), Datatype.UINT16, 2, [u16]))
    # full-range windows (overflow path, bwr.cc:421-430)
    fr = np.array([-2**31, 2**31 - 1] * 64, dtype=np.int32)
    cases.append(Case("bwr_full_range_i32", P(BitWidthReductionFilter(256)), I32, 4, [as_u8(fr)]))
    fu = np.array([0, 2**64 - 1, 5, 7] * 32, dtype=np.uint64)
    cases.append(Case("bwr_full_range_u64", P(BitWidthReductionFilter(256)), U64, 8, [as_u8(fu)]))
    # mixed-width windows: 8/16/32-bit ranges
    mix = np.concatenate([np.arange(64) * 1, np.arange(64) * 1000, np.arange(64) * 10**7,
                          np.arange(64) * 10**12]).astype(np.int64)
    cases.append(Case("bwr_mixed_widths_i64", P(BitWidthReductionFilter(512)), I64, 8,
                      [as_u8(mix)]))
    # DD raw fallback (random u64) and negative dd
    cases.append(Case("dd_raw_random_u64", P(DD()), U64, 8,
                      [as_u8(rng.integers(0, 2**62, 4096, dtype=np.int64).astype(np.uint64))]))
    zig = (np.cumsum(rng.integers(-50, 50, 5000)) * 3).astype(np.int64)
    cases.append(Case("dd_negative_i64", P(DD()), I64, 8, [as_u8(zig)]))
    for dt in (Datatype.INT8, Datatype.UINT8, Datatype.INT16, Datatype.UINT16, Datatype.INT32,
               Datatype.UINT32):
        sz = datatype_size(dt)
        n = 3001
        base = np.cumsum(rng.integers(-3, 4, n)).astype(np.int64)
        raw = (base.astype(np.int64) & ((1 << (8 * sz)) - 1)).astype(np.uint64)
        data = as_u8(raw.astype({1: np.uint8, 2: np.uint16, 4: np.uint32}[sz]))
        cases.append(Case(f"dd_{dt.name}", P(DD()), dt, sz, [data]))
    # DD with reinterpret datatype (v >= 20)
    cases.append(Case("dd_reinterpret_u8_as_u32", P(DD(Datatype.UINT32)), Datatype.UINT8, 1,
                      [as_u8(np.arange(4000, dtype=np.uint32))]))
    cases.append(Case("dd_datetime_ns", P(DD()), Datatype.DATETIME_NS, 8,
                      [as_u8(np.arange(2000, dtype=np.int64) * 1_000_000_007)]))
    # RLE run exactly 65535 and 65536 (rle_compressor.cc:56-100)
    for n in (65535, 65536, 70030):
        d = np.full(n, 7, dtype=np.int32)
        d[:3] = [1, 2, 3]
        if n == 70030:
            d[:10] = np.arange(10)
            d[70010:] = np.arange(70010, 70030)
        cases.append(Case(f"rle_run_{n}", P(RLE()), I32, 4, [as_u8(d)], max_chunk=1 << 20))
    cases.append(Case("rle_cell1_bytes", P(RLE()), Datatype.UINT8, 1,
                      [np.repeat(rng.integers(0, 4, 500).astype(np.uint8), rng.integers(1, 9, 500))]))
    cases.append(Case("rle_cell12", P(RLE()), Datatype.UINT32, 12,
                      [as_u8(np.repeat(rng.integers(0, 3, (300, 3)).astype(np.uint32), 5, axis=0))]))
    # PD with equal values / windows
    eq = np.repeat(np.arange(100, dtype=np.uint32), 10)
    cases.append(Case("pd_equal_u32", P(PositiveDeltaFilter(64)), Datatype.UINT32, 4, [as_u8(eq)]))
    cases.append(Case("pd_i8", P(PositiveDeltaFilter(33)), Datatype.INT8, 1,
                      [as_u8(np.sort(rng.integers(-128, 128, 777)).astype(np.int8))]))
    cases.append(Case("pd_tail_u64", P(PositiveDeltaFilter(1000)), U64, 8,
                      [as_u8(np.arange(1001, dtype=np.uint64) * 3)]))
    # multi-chunk tiles with a short last chunk
    mc = as_u8(np.arange(20000, dtype=np.uint64) * 7)
    cases.append(Case("multichunk_bwr", P(BitWidthReductionFilter(256)), U64, 8, [mc]))
    cases.append(Case("multichunk_80B", P(ByteshuffleFilter(), BitWidthReductionFilter(32)), U64, 8,
                      [as_u8(np.arange(1003, dtype=np.uint64))], max_chunk=80))
    cases.append(Case("multichunk_c5_small_chunks",
                      P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256)), I32, 4,
                      [as_u8(np.arange(50000, dtype=np.int32))], max_chunk=4096))
    # datetime at format versions 19 and 20 (bwr.cc:322-332)
    dt_data = as_u8(np.arange(3000, dtype=np.int64) * 86400)
    for v in (19, 20):
        cases.append(Case(f"datetime_bwr_pd_v{v}",
                          P(PositiveDeltaFilter(512), BitWidthReductionFilter(256)),
                          Datatype.DATETIME_DAY, 8, [dt_data], version=v))
    # offsets tile: unfiltered size = tile size - 8 (tile.cc:241-248)
    offs = c4_tiles(1, 777)[0]
    cases.append(Case("offsets_tile", P(PositiveDeltaFilter(1024), BitWidthReductionFilter(256)),
                      U64, 8, [offs], offsets_tile=True))
    # metadata stacks through compression filters
    cases.append(Case("bwr_then_dd", P(BitWidthReductionFilter(128), DD()), I32, 4,
                      [as_u8(np.cumsum(rng.integers(0, 100, 5000)).astype(np.int32))]))
    cases.append(Case("byte_bit_dd_two_md_parts",
                      P(ByteshuffleFilter(), BitshuffleFilter(), DD()), I32, 4,
                      [as_u8(np.arange(4001, dtype=np.int32) // 3)]))
    cases.append(Case("rle_then_bwr", P(RLE(), BitWidthReductionFilter(64)), Datatype.UINT64, 8,
                      [as_u8(np.repeat(np.arange(300, dtype=np.uint64), 9))]))
    cases.append(Case("dd_then_rle_cell1", P(DD(), RLE()), Datatype.UINT8, 1,
                      [as_u8(np.arange(5000, dtype=np.uint64).astype(np.uint8))]))
    cases.append(Case("noop_and_none", P(NoopFilter(), CompressionFilter(Compressor.NO_COMPRESSION),
                                         ByteshuffleFilter()), I32, 4,
                      [as_u8(np.arange(999, dtype=np.int32))]))
    cases.append(Case("pd_float_passthrough", P(PositiveDeltaFilter(64), BitshuffleFilter()),
                      Datatype.FLOAT64, 8, [as_u8(rng.normal(size=500))]))
    # var-size chunking (filter_pipeline.cc:151-206)
    lens = rng.integers(1, 3000, 200)
    offs_v = np.zeros(200, dtype=np.uint64)
    offs_v[1:] = np.cumsum(lens[:-1])
    vdata = rng.integers(0, 3, int(lens.sum())).astype(np.uint8)
    cases.append(Case("var_chunks_bytes", P(RLE(), BitshuffleFilter()), Datatype.UINT8, 1, [vdata],
                      offsets=[offs_v], max_chunk=8192))
    # tile sizes 1 and 0
    cases.append(Case("one_byte_tile", P(ByteshuffleFilter()), Datatype.UINT8, 1,
                      [np.array([42], dtype=np.uint8)]))
    # incompressible C1/C5 shapes (every stage before the byteshuffle takes
    # its raw path) at every element width, ragged sizes (16-B unit tails,
    # plane tails), unaligned outputs (ragged tiles packed back to back),
    # raw and compressed tiles mixed in one batch, offsets tiles
    c5p = P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256))
    for dt, n in ((Datatype.INT16, 32768), (Datatype.INT32, 16383), (Datatype.INT64, 8191),
                  (Datatype.INT32, 1000), (Datatype.UINT16, 32767)):
        sz = datatype_size(dt)
        tiles = [rng.integers(0, 256, n * sz, dtype=np.uint8) for _ in range(3)]
        cases.append(Case(f"incomp_c5_rand_{dt.name}_{n}", c5p, dt, sz, tiles))
        cases.append(Case(f"incomp_c1_rand_{dt.name}_{n}", P(ByteshuffleFilter()), dt, sz, tiles))
    mixed = [rng.integers(0, 256, 65536, dtype=np.uint8), as_u8(np.arange(16384, dtype=np.int32)),
             rng.integers(0, 256, 65532, dtype=np.uint8), as_u8(np.arange(16383, dtype=np.int32) * 7)]
    cases.append(Case("incomp_c5_mixed_raw_and_packed", c5p, I32, 4, mixed))
    cases.append(Case("incomp_c5_offsets_u64", c5p, U64, 8,
                      [rng.integers(0, 256, 8 * 8191, dtype=np.uint8)], offsets_tile=True))
    # XOR (xor_filter.cc): every width, float inputs whose
    # XOR output type (INT32/INT64) makes a following BWR / DD active,
    # multi-chunk tiles, XOR after a shuffle (md stack)
    for dt in (Datatype.INT8, Datatype.UINT16, Datatype.INT32, Datatype.UINT64):
        sz = datatype_size(dt)
        v = np.cumsum(rng.integers(0, 50, 4000)).astype(np.int64).astype(
            {1: np.uint8, 2: np.uint16, 4: np.int32, 8: np.uint64}[sz])
        cases.append(Case(f"xor_{dt.name}", P(XORFilter()), dt, sz, [as_u8(v)]))
    f32 = (1000 * np.sin(np.arange(16384) * 1e-3)).astype(np.float32)
    cases.append(Case("xor_f32_then_bwr", P(XORFilter(), BitWidthReductionFilter(256)),
                      Datatype.FLOAT32, 4, [as_u8(f32)]))
    f64 = 1.0 + np.cumsum(rng.integers(0, 9, 8192)) * 2.0 ** -30  # one exponent: small XORs
    cases.append(Case("xor_f64_then_dd", P(XORFilter(), DD()), Datatype.FLOAT64, 8, [as_u8(f64)]))
    cases.append(Case("xor_multichunk_i32", P(XORFilter(), BitshuffleFilter()), I32, 4,
                      [as_u8(np.arange(30000, dtype=np.int32) * 3)], max_chunk=4096))
    cases.append(Case("byteshuffle_then_xor_i64", P(ByteshuffleFilter(), XORFilter()), I64, 8,
                      [as_u8(np.arange(7000, dtype=np.int64) ** 2)]))
    # DELTA compressor (delta_compressor.cc): widths, wrapping
    # differences, reinterpret, md parts (shuffle md through the frame), multi-chunk
    cases.append(Case("delta_i32", P(DELTA()), I32, 4,
                      [as_u8(np.cumsum(rng.integers(-1000, 1000, 16384)).astype(np.int32))]))
    cases.append(Case("delta_u8_wrap", P(DELTA()), Datatype.UINT8, 1,
                      [rng.integers(0, 256, 5000, dtype=np.uint8)]))
    cases.append(Case("delta_u64_extremes", P(DELTA()), U64, 8,
                      [as_u8(np.array([0, 2**64 - 1, 1, 2**63, 5] * 300, dtype=np.uint64))]))
    cases.append(Case("delta_i16_one_value", P(DELTA()), Datatype.INT16, 2,
                      [as_u8(np.array([-7], dtype=np.int16))]))
    cases.append(Case("delta_reinterpret_u8_as_i32", P(DELTA(Datatype.INT32)), Datatype.UINT8, 1,
                      [as_u8(np.arange(4000, dtype=np.int32) * 3)]))
    cases.append(Case("byteshuffle_delta_bwr", P(ByteshuffleFilter(), DELTA(), BitWidthReductionFilter(256)),
                      I32, 4, [as_u8(np.arange(16384, dtype=np.int32) * 5)]))
    cases.append(Case("delta_multichunk_i64", P(DELTA()), I64, 8,
                      [as_u8(np.cumsum(rng.integers(0, 9, 30000)).astype(np.int64))], max_chunk=8192))
    # FLOAT_SCALE (float_scaling_filter.cc).  Exact cases:
    # values on the scale grid (binary scale/offset) round-trip bit-exactly;
    # lossy cases (decimal scale) are still GPU-vs-oracle bit-exact
    k = rng.integers(-30000, 30000, 16384)
    for bw in (2, 4, 8):
        cases.append(Case(f"fscale_f32_exact_bw{bw}", P(FloatScalingFilter(0.125, -3.0, bw)),
                          Datatype.FLOAT32, 4, [as_u8((-3.0 + 0.125 * k).astype(np.float32))]))
    cases.append(Case("fscale_f64_exact_bw8", P(FloatScalingFilter(2.0 ** -20, 1.5, 8)),
                      Datatype.FLOAT64, 8, [as_u8(1.5 + k.astype(np.float64) * 2.0 ** -20)]))
    cases.append(Case("fscale_f32_lossy_bw1", P(FloatScalingFilter(0.01, 0.5, 1)), Datatype.FLOAT32, 4,
                      [as_u8(rng.uniform(-0.7, 1.7, 5000).astype(np.float32))],
                      extra={"lossy": (np.float32, 0.01)}))
    cases.append(Case("fscale_f64_lossy_then_bwr",
                      P(FloatScalingFilter(1e-3, 0.0, 4), BitWidthReductionFilter(256)),
                      Datatype.FLOAT64, 8, [as_u8(np.sin(np.arange(8192) * 1e-2))],
                      extra={"lossy": (np.float64, 1e-3)}))
    cases.append(Case("fscale_f32_then_delta_bitshuffle",
                      P(FloatScalingFilter(0.5, 0.0, 4), DELTA(), BitshuffleFilter()),
                      Datatype.FLOAT32, 4, [as_u8((0.5 * np.arange(20000)).astype(np.float32))],
                      max_chunk=16384))
    return cases


# ---------------------------------------------------------------------------
# random pipelines (unit_run_filter_pipeline.cc:800-912 style)
# ---------------------------------------------------------------------------
_INT_TYPES = [Datatype.INT8, Datatype.UINT8, Datatype.INT16, Datatype.UINT16, Datatype.INT32,
              Datatype.UINT32, Datatype.INT64, Datatype.UINT64]


def random_cases(n: int, seed: int = 1234, max_elems: int = 3000) -> List[Case]:
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        dt = _INT_TYPES[rng.integers(len(_INT_TYPES))]
        sz = datatype_size(dt)
        nflt = int(rng.integers(1, 5))
        filters = []
        for i in range(nflt):
            choice = int(rng.integers(0, 6 if i else 7))
            if choice == 0:
                filters.append(BitWidthReductionFilter(int(rng.choice([32, 64, 256, 437]))))
            elif choice == 1:
                filters.append(BitshuffleFilter())
            elif choice == 2:
                filters.append(ByteshuffleFilter())
            elif choice == 3:
                filters.append(DD())
            elif choice == 4:
                filters.append(RLE())
            elif choice == 5:
                filters.append(NoopFilter())
            else:
                filters.insert(0, PositiveDeltaFilter(int(rng.choice([64, 1024]))))
        ne = int(rng.integers(1, max_elems))
        kind = rng.integers(3)
        if kind == 0:
            vals = np.sort(rng.integers(0, 1 << min(8 * sz - 1, 40), ne))
        elif kind == 1:
            vals = np.repeat(rng.integers(0, 50, ne // 4 + 1), 4)[:ne]
        else:
            vals = rng.integers(0, 1 << min(8 * sz, 62), ne)
        if filters and isinstance(filters[0], PositiveDeltaFilter):
            vals = np.sort(vals)
        np_t = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[sz]
        cell = sz if rng.integers(4) else sz * 2
        data = as_u8(vals.astype(np.uint64).astype(np_t))
        data = data[: data.size // cell * cell] if data.size >= cell else data
        mc = int(rng.choice([0, 0, 1024, 4096]))
        out.append(Case(f"random_{k}", P(*filters), dt, cell, [data], max_chunk=mc))
    return out


# ---------------------------------------------------------------------------
# one case per fused-kernel spec (tdbg_fast.hip SPECS): tiles the fused LDS
# kernel must take without declining (single 64 KiB chunks, encoder-uniform
# windows), so tests can assert the fallback counter stays 0
# ---------------------------------------------------------------------------
def fused_spec_cases(ntiles: int = 3) -> List[Case]:
    rng = np.random.default_rng(21)
    I16, I32, U32, I64, U64 = (Datatype.INT16, Datatype.INT32, Datatype.UINT32, Datatype.INT64,
                               Datatype.UINT64)
    F32, F64 = Datatype.FLOAT32, Datatype.FLOAT64
    B, T, W = ByteshuffleFilter, BitshuffleFilter, BitWidthReductionFilter

    def smooth(dt, n, k):
        """slowly varying values (BWR windows narrow, DD compresses)."""
        base = np.cumsum(rng.integers(0, 40, n)).astype(np.int64) + 1000 * k
        np_t = {I16: np.int16, I32: np.int32, U32: np.uint32, I64: np.int64, U64: np.uint64}[dt]
        return as_u8(base.astype(np_t))

    def tiles(dt, nbytes=65536):
        sz = datatype_size(dt)
        return [smooth(dt, nbytes // sz, k) for k in range(ntiles)]

    def rand(nbytes=65536):
        return [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(ntiles)]

    def small64(k):
        """64-bit values whose every byte is < 0x40: the byteshuffled planes read
        as 64-bit words stay below 2^62, so DoubleDelta's checked deltas cannot
        overflow (dd_compressor.cc:281-294) and the C5 shape encodes."""
        a = rng.integers(0, 0x40, (8192, 8), dtype=np.uint8)
        a[:, 2:] = 0
        a[:, 0] = (np.arange(8192) // 7 + k) % 0x40
        return a.reshape(-1)

    f64 = [as_u8(np.sin(np.arange(8192) * 1e-3 + k)) for k in range(ntiles)]
    out = [
        Case("spec01_byte_i32", P(B()), I32, 4, tiles(I32) + rand()),
        Case("spec02_byte_i64", P(B()), I64, 8, tiles(I64) + rand()),
        Case("spec03_byte_i16", P(B()), I16, 2, tiles(I16) + rand()),
        Case("spec04_bit_pass_f32", P(T(), W(256)), F32, 4, c2_tiles(ntiles)),
        Case("spec05_bit_pass_f64", P(T(), W(256)), F64, 8, f64),
        Case("spec06_bit_i32", P(T()), I32, 4, tiles(I32)),
        Case("spec07_bit_u64", P(T()), U64, 8, tiles(U64)),
        Case("spec08_bit_bwr_i32", P(T(), W(256)), I32, 4, tiles(I32) + rand()),
        Case("spec09_bit_bwr_u32", P(T(), W(256)), U32, 4, tiles(U32)),
        Case("spec10_bit_bwr_i64", P(T(), W(256)), I64, 8, tiles(I64)),
        Case("spec11_bit_bwr_u64", P(T(), W(256)), U64, 8, tiles(U64) + rand()),
        Case("spec12_dd_u64", P(DD()), U64, 8, c3_tiles(ntiles)),
        Case("spec13_dd_i32", P(DD()), I32, 4, tiles(I32)),
        Case("spec14_rle_u64", P(RLE()), U64, 8, c3_tiles(ntiles)),
        Case("spec15_pd_bwr_u64", P(PositiveDeltaFilter(1024), W(256)), U64, 8, c4_tiles(ntiles)),
        Case("spec16_pd_bwr_i64", P(PositiveDeltaFilter(1024), W(256)), I64, 8, tiles(I64)),
        Case("spec17_pd_bwr_u32", P(PositiveDeltaFilter(512), W(256)), U32, 4, tiles(U32)),
        Case("spec18_pd_bwr_i32", P(PositiveDeltaFilter(1024), W(256)), I32, 4, tiles(I32)),
        Case("spec19_c5_i32", P(B(), DD(), W(256)), I32, 4, c5_tiles(ntiles, "ramp") + c5_tiles(ntiles, "rand")
             + tiles(I32)),
        Case("spec20_c5_u32", P(B(), DD(), W(256)), U32, 4, tiles(U32)),
        Case("spec21_c5_i64", P(B(), DD(), W(256)), I64, 8, [small64(k) for k in range(ntiles)]),
        Case("spec22_c5_u64", P(B(), DD(), W(256)), U64, 8, [small64(k) for k in range(ntiles)]),
        Case("spec23_dd_bwr_i64", P(DD(), W(256)), I64, 8, tiles(I64)),
        Case("spec24_dd_bwr_u64", P(DD(), W(256)), U64, 8, tiles(U64)),
        Case("spec25_bwr_i32", P(W(256)), I32, 4, tiles(I32) + rand()),
        Case("spec26_bwr_u64", P(W(256)), U64, 8, tiles(U64)),
        Case("spec27_bwr_i64", P(W(256)), I64, 8, tiles(I64) + rand()),
        # XOR / DELTA / FLOAT_SCALE pipelines
        Case("spec28_xor_bwr_f32", P(XORFilter(), W(256)), F32, 4, c2_tiles(ntiles)),
        Case("spec29_xor_bwr_f64", P(XORFilter(), W(256)), F64, 8, f64),
        Case("spec30_xor_i32", P(XORFilter()), I32, 4, tiles(I32) + rand()),
        Case("spec31_xor_u64", P(XORFilter()), U64, 8, tiles(U64)),
        Case("spec32_byte_delta_bwr_i32", P(B(), DELTA(), W(256)), I32, 4, tiles(I32) + rand()),
        Case("spec33_delta_i32", P(DELTA()), I32, 4, tiles(I32) + rand()),
        Case("spec34_delta_i64", P(DELTA()), I64, 8, tiles(I64)),
        Case("spec35_fscale_f64_bw4_bwr", P(FloatScalingFilter(1e-3, 0.0, 4), W(256)), F64, 8, f64),
        Case("spec36_fscale_f32_bw4", P(FloatScalingFilter(0.125, -3.0, 4)), F32, 4, c2_tiles(ntiles)),
        Case("spec37_fscale_f64_bw8_bwr", P(FloatScalingFilter(2.0 ** -20, 1.5, 8), W(256)), F64, 8, f64),
    ]
    return out
