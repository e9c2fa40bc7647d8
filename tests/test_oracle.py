"""CPU tests: pin the oracle (tdb_oracle.c) before trusting it as the checker.

Pins, in order of strength:
  * golden bytes / known answers the reference's own tests hold
    - pipeline descriptor bytes   tiledb/sm/filter/test/unit_filter_pipeline.cc:59-126
    - RLE compressed sizes        test/src/unit-compression-rle.cc:75-289
    - BWR header fields           tiledb/sm/filter/test/unit_bit_width_reduction_pipeline.cc:61-90
    - DD overflow expectations    tiledb/sm/filter/test/unit_double_delta_pipeline.cc:88-135
  * an independent implementation of the third-party arithmetic: kiyo-masui
    bitshuffle (imagecodecs 2021.8.26) fixtures, tests/golden/bitshuffle_kiyo.npz
  * the normative layouts of format_spec/filters/double_delta.md and tile.md,
    hand-assembled byte by byte
  * a second, independent restatement (workloads.py, numpy) producing
    identical bytes for the C5 pipeline
  * round trips over every config, edge case and random pipeline, which is
    how the reference's filter tests check themselves.
"""
from __future__ import annotations

import os
import struct

import numpy as np
import pytest

from tests.cases import DD, P, RLE, as_u8, config_cases, edge_cases, random_cases
from tiledb_amd.filter_pipeline import (BitWidthReductionFilter, Compressor, CompressionFilter,
                                        Datatype, FilterPipeline, FilterType)

HERE = os.path.dirname(os.path.abspath(__file__))


# ---------------------------------------------------------------------------
# descriptor golden bytes (unit_filter_pipeline.cc:59-126)
# ---------------------------------------------------------------------------
def _golden_descriptor() -> bytes:
    b = bytearray(38)
    struct.pack_into("<II", b, 0, 4096, 3)
    struct.pack_into("<BIBi", b, 8, FilterType.FILTER_ZSTD, 5, Compressor.ZSTD, 1)
    struct.pack_into("<BIB", b, 18, FilterType.FILTER_RLE, 5, Compressor.RLE)  # level left 0
    struct.pack_into("<BIBi", b, 28, FilterType.FILTER_GZIP, 5, Compressor.GZIP, 1)
    return bytes(b)


def test_descriptor_golden_python_and_oracle(oracle_mod):
    g = _golden_descriptor()
    p = FilterPipeline.deserialize(g, 23, Datatype.INT32)
    assert p.max_chunk_size == 4096 and p.size() == 3
    assert [f.type for f in p.filters] == [FilterType.FILTER_ZSTD, FilterType.FILTER_RLE,
                                          FilterType.FILTER_GZIP]
    assert p.filters[0].level == 1 and p.filters[2].level == 1
    assert p.serialize() == g
    op = oracle_mod.OraclePipeline(g, 23, int(Datatype.INT32), 4)
    assert op.consumed == 38
    assert op.serialize() == g


def test_descriptor_roundtrip_all_cases(oracle_mod):
    for c in config_cases(1) + edge_cases() + random_cases(50):
        ser = c.serialized
        op = oracle_mod.OraclePipeline(ser, c.version, int(c.dtype), c.cell_size)
        assert op.serialize() == ser, c.name
        back = FilterPipeline.deserialize(ser, c.version, c.dtype)
        assert back.serialize() == ser, c.name


def test_descriptor_truncated_is_error(oracle_mod):
    g = _golden_descriptor()
    for n in (0, 4, 7, 9, 20, 37):
        with pytest.raises(oracle_mod.OracleError):
            oracle_mod.OraclePipeline(g[:n], 23, 0, 4)


# ---------------------------------------------------------------------------
# RLE known sizes (unit-compression-rle.cc)
# ---------------------------------------------------------------------------
def test_rle_known_sizes(oracle_mod):
    O = oracle_mod
    same = np.full(100, 111, dtype=np.int32)
    assert len(O.rle_compress(4, same)) == 6
    mixed = np.array(list(range(10)) + [110] * 90 + list(range(100, 110)), dtype=np.int32)
    assert len(O.rle_compress(4, mixed)) == 21 * 6
    big = np.array(list(range(10)) + [20] * 70000 + list(range(70010, 70030)), dtype=np.int32)
    c = O.rle_compress(4, big)
    assert len(c) == 32 * 6
    rc, out = O.rle_decompress(4, c, big.nbytes)
    assert rc == 0 and np.array_equal(out.view(np.int32), big)
    # double:2 (value size 16): 21 runs x 18 B
    data = np.zeros(220)
    j, k = 0.1, 0.2
    for i in range(10):
        j += 10000.12
        k += 1000.12
        data[2 * i], data[2 * i + 1] = j, k
    j += 10000.12
    k += 1000.12
    for i in range(10, 100):
        data[2 * i] = data[2 * i + 1] = j
    for i in range(100, 110):
        j += 10000.12
        k += 1000.12
        data[2 * i], data[2 * i + 1] = j, k
    assert len(O.rle_compress(16, data)) == 21 * 18
    uniq = np.arange(100, dtype=np.int32)
    rc, out = O.rle_decompress(4, O.rle_compress(4, uniq), uniq.nbytes)
    assert rc == 0 and np.array_equal(out.view(np.int32), uniq)


def test_rle_invalid_format(oracle_mod):
    O = oracle_mod
    with pytest.raises(O.OracleError):  # 5 bytes with value size 4 (rle.cc:68-71)
        O.rle_compress(4, np.array([0, 0, 0, 0, 97], dtype=np.uint8))
    rc, _ = O.rle_decompress(4, np.zeros(7, dtype=np.uint8), 100)  # 7 % 6 != 0
    assert rc == 7  # TDBG_E_RLE_FORMAT


def test_rle_run_split_at_65535(oracle_mod):
    c = oracle_mod.rle_compress(4, np.full(65536, 9, dtype=np.int32))
    assert len(c) == 12
    assert c[4:6] == b"\xff\xff" and c[10:12] == b"\x00\x01"  # big-endian u16 lengths


# ---------------------------------------------------------------------------
# BWR header fields (unit_bit_width_reduction_pipeline.cc:61-90)
# ---------------------------------------------------------------------------
def test_bwr_header_fields(oracle_mod):
    p = P(BitWidthReductionFilter())  # default window 256
    op = oracle_mod.OraclePipeline(p.serialize(), 23, int(Datatype.UINT64), 8)
    nelts = 1000
    f = op.filter_tile(np.arange(nelts, dtype=np.uint64))
    off = 8 + 4 + 4 + 4
    assert struct.unpack_from("<I", f, off)[0] == nelts * 8           # original length
    assert struct.unpack_from("<I", f, off + 4)[0] == (8000 // 256 + 1)  # window count
    assert len(f) < nelts * 8
    for w in (32, 64, 128, 256, 437, 512, 1024, 2000):
        op = oracle_mod.OraclePipeline(P(BitWidthReductionFilter(w)).serialize(), 23,
                                       int(Datatype.UINT64), 8)
        rc, out = op.unfilter_tile(op.filter_tile(np.arange(nelts, dtype=np.uint64)), 8000)
        assert rc == 0 and np.array_equal(out.view(np.uint64), np.arange(nelts, dtype=np.uint64))


# ---------------------------------------------------------------------------
# DD overflow expectations (unit_double_delta_pipeline.cc:88-135)
# ---------------------------------------------------------------------------
def _expect_overflow(vals: np.ndarray, signed: bool) -> bool:
    v = [int(x) for x in vals]
    if len(v) <= 2:
        return False
    d = []
    for i in range(1, len(v)):
        x = v[i] - v[i - 1]
        if not (-2**63 <= x <= 2**63 - 1):
            return True
        d.append(x)
    for i in range(1, len(d)):
        if not (-2**63 <= d[i] - d[i - 1] <= 2**63 - 1):
            return True
    return False


@pytest.mark.parametrize("signed", [True, False])
def test_dd_overflow_expectation(oracle_mod, signed):
    rng = np.random.default_rng(5 + signed)
    dt = Datatype.INT64 if signed else Datatype.UINT64
    for trial in range(300):
        n = int(rng.integers(1, 12))
        if signed:
            vals = rng.integers(-2**63, 2**63, n, dtype=np.int64)
        else:
            vals = rng.integers(0, 2**64, n, dtype=np.uint64)
        if trial % 3 == 0:
            vals = np.sort(vals)
        exp = _expect_overflow(vals, signed)
        try:
            c = oracle_mod.dd_compress(int(dt), vals)
            got_overflow = False
        except oracle_mod.OracleError as e:
            assert e.code == 13
            got_overflow = True
        assert got_overflow == exp, (vals, exp)
        if not got_overflow:
            rc, out = oracle_mod.dd_decompress(int(dt), c, vals.nbytes)
            assert rc == 0 and np.array_equal(out.view(vals.dtype), vals)


# ---------------------------------------------------------------------------
# format_spec/filters/double_delta.md, hand-assembled
# ---------------------------------------------------------------------------
def test_dd_format_spec_known_answer(oracle_mod):
    vals = np.array([1, 3, 6, 10, 13, 13], dtype=np.int64)
    # deltas 2,3,4,3,0 ; dd = 1,1,-1,-3 ; bitsize over |d1|=2 and |dd| -> 2
    exp = struct.pack("<BQqq", 2, 6, 1, 3)
    bits = ""
    for dd in (1, 1, -1, -3):
        bits += ("1" if dd < 0 else "0") + format(abs(dd), "02b")
    bits = bits.ljust(64, "0")
    exp += struct.pack("<Q", int(bits, 2))
    got = oracle_mod.dd_compress(int(Datatype.INT64), vals)
    assert got == exp
    rc, out = oracle_mod.dd_decompress(int(Datatype.INT64), exp, vals.nbytes)
    assert rc == 0 and np.array_equal(out.view(np.int64), vals)


def test_dd_raw_fallback_layout(oracle_mod):
    # bitsize >= 8*sizeof(T)-1: header then the raw input (dd_compressor.cc:233-236)
    vals = np.array([0, 2**30, -2**30, 2**30, -2**30], dtype=np.int32)
    got = oracle_mod.dd_compress(int(Datatype.INT32), vals)
    assert got[0] >= 31 and struct.unpack_from("<Q", got, 1)[0] == 5
    assert got[9:] == vals.tobytes()


# ---------------------------------------------------------------------------
# shuffles: blosc2 semantics
# ---------------------------------------------------------------------------
def test_bitshuffle_vs_kiyo_masui_fixtures(oracle_mod):
    z = np.load(os.path.join(HERE, "golden", "bitshuffle_kiyo.npz"))
    n = 0
    for k in z.files:
        if not k.startswith("in_"):
            continue
        ts = int(k.split("_")[1][2:])
        data, exp = z[k], z["out" + k[2:]]
        enc = b"".join(oracle_mod.bitshuffle_block(data[i:i + 8192], ts)
                       for i in range(0, data.size, 8192))
        assert enc == exp.tobytes(), k
        dec = b"".join(oracle_mod.bitshuffle_block(exp[i:i + 8192], ts, inverse=True)
                       for i in range(0, exp.size, 8192))
        assert dec == data.tobytes(), k
        n += 1
    assert n == 24


@pytest.mark.parametrize("ts", [1, 2, 3, 4, 8, 16])
def test_byteshuffle_vs_numpy_transpose(oracle_mod, ts):
    rng = np.random.default_rng(ts)
    for n in (0, 1, ts, 7 * ts + 3, 1000, 4099):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        N = n // ts
        exp = np.concatenate([d[: N * ts].reshape(N, ts).T.reshape(-1), d[N * ts:]])
        assert oracle_mod.byteshuffle(d, ts) == exp.tobytes()
        assert oracle_mod.byteshuffle(exp, ts, inverse=True) == d.tobytes()


# ---------------------------------------------------------------------------
# second restatement: workloads.py (numpy) == oracle forward, byte for byte
# ---------------------------------------------------------------------------
def test_c5_active_variant_exercises_every_stage():
    """The 'active' C5 variant: DoubleDelta takes its bit-packed path
    (bitsize < 8*sizeof(int32) - 1, dd_compressor.cc:233-236) and most BWR
    windows over DD's output narrow to 8 bits."""
    import struct
    import workloads as W
    rng = np.random.default_rng(3)
    for t in range(8):
        v = W.c5_values("active", t, rng)
        assert W.c5_dd_bitsize(v) < 31
        f = W.c5_filter_tile(v)
        ml = struct.unpack_from("<I", f, 16)[0]
        nw = struct.unpack_from("<I", f, 24)[0]
        bits = [f[20 + 8 + k * 9 + 4] for k in range(nw)]
        assert sum(b == 8 for b in bits) > 0.8 * nw
        assert len(f) < 0.4 * v.nbytes and ml > 0


@pytest.mark.parametrize("variant", ["ramp", "rand", "active"])
def test_numpy_c5_encoder_matches_oracle(oracle_mod, variant):
    import workloads as W
    op = oracle_mod.OraclePipeline(W.c5_pipeline_bytes(), 23, int(Datatype.INT32), 4)
    rng = np.random.default_rng(1)
    for t in range(4):
        v = W.c5_values(variant, t, rng)
        f = W.c5_filter_tile(v)
        assert f == op.filter_tile(v)
        rc, out = op.unfilter_tile(f, v.nbytes)
        assert rc == 0 and np.array_equal(out, v.view(np.uint8))


# ---------------------------------------------------------------------------
# round trips (how the reference's filter tests check themselves)
# ---------------------------------------------------------------------------
def _roundtrip(O, case):
    op = O.OraclePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    n = 0
    for i, t in enumerate(case.tiles):
        try:
            f = op.filter_tile(t, case.offsets[i] if case.offsets else None, case.max_chunk)
        except O.OracleError:
            continue
        osz = t.size + (8 if case.offsets_tile else 0)
        rc, out = op.unfilter_tile(f, osz, case.offsets_tile)
        assert rc == 0, (case.name, rc)
        if "lossy" in case.extra:  # FLOAT_SCALE quantization: |x' - x| <= scale / 2
            ft, scale = case.extra["lossy"]
            err = np.abs(out[: t.size].view(ft).astype(np.float64) - t.view(ft).astype(np.float64))
            assert err.max() <= scale / 2 * (1 + 1e-6) + 1e-6, case.name
        else:
            assert np.array_equal(out[: t.size], t), case.name
        n += 1
    return n


@pytest.mark.parametrize("case", config_cases(2), ids=lambda c: c.name)
def test_oracle_roundtrip_configs(oracle_mod, case):
    assert _roundtrip(oracle_mod, case) == len(case.tiles)


@pytest.mark.parametrize("case", edge_cases(), ids=lambda c: c.name)
def test_oracle_roundtrip_edges(oracle_mod, case):
    _roundtrip(oracle_mod, case)


def test_config_c3_literal_dd_then_rle_is_rejected(oracle_mod):
    """BASELINE config 3 as written ([DOUBLE_DELTA, RLE] on 8-byte cells)
    throws in the reference: DD output is 9 + 8k bytes, not a multiple of the
    RLE cell size (rle_compressor.cc:68-71)."""
    from tests.cases import c3_tiles
    op = oracle_mod.OraclePipeline(P(DD(), RLE()).serialize(), 23, int(Datatype.UINT64), 8)
    with pytest.raises(oracle_mod.OracleError) as e:
        op.filter_tile(c3_tiles(1)[0])
    assert e.value.code == 7


def test_pd_rejects_decreasing(oracle_mod):
    from tiledb_amd.filter_pipeline import PositiveDeltaFilter
    op = oracle_mod.OraclePipeline(P(PositiveDeltaFilter()).serialize(), 23,
                                   int(Datatype.UINT64), 8)
    with pytest.raises(oracle_mod.OracleError) as e:
        op.filter_tile(np.array([5, 4, 3], dtype=np.uint64))
    assert e.value.code == 12


def test_offsets_tile_expected_size(oracle_mod):
    from tiledb_amd.filter_pipeline import PositiveDeltaFilter
    op = oracle_mod.OraclePipeline(P(PositiveDeltaFilter()).serialize(), 23,
                                   int(Datatype.UINT64), 8)
    t = np.arange(100, dtype=np.uint64)
    f = op.filter_tile(t)
    rc, _ = op.unfilter_tile(f, t.nbytes + 8, is_offsets=True)
    assert rc == 0
    rc, _ = op.unfilter_tile(f, t.nbytes, is_offsets=True)
    assert rc == 3  # TDBG_E_TILE_SIZE (tile.cc:308-309)


def test_mt_batch_equals_single(oracle_mod):
    import workloads as W
    op = oracle_mod.OraclePipeline(W.c5_pipeline_bytes(), 23, 0, 4)
    tiles, vals = W.c5_pool("ramp", 6)
    sizes = np.array([len(t) for t in tiles], dtype=np.uint64)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    packed = np.frombuffer(b"".join(tiles), dtype=np.uint8).copy()
    out = np.zeros(6 * 65536, dtype=np.uint8)
    rc, st = op.unfilter_tiles_mt(packed, offs, sizes, out, np.arange(6, dtype=np.uint64) * 65536,
                                  np.full(6, 65536, dtype=np.uint64), 3)
    assert rc == 0 and not st.any()
    for i, v in enumerate(vals):
        assert np.array_equal(out[i * 65536:(i + 1) * 65536], v.view(np.uint8))


@pytest.mark.parametrize("name", ["c1", "c2", "c2i", "c3a", "c3b", "c4", "c5"])
def test_numpy_config_encoders_match_oracle(oracle_mod, name):
    """workloads.py's forward restatements (the bench's inputs) equal the
    oracle's forward pass byte for byte, and unfilter back to the values."""
    import workloads as W
    ser, dt, cs, values, tile = W.config(name)
    op = oracle_mod.OraclePipeline(ser, 23, int(dt), cs)
    rng = np.random.default_rng(7)
    for variant in ("ramp", "rand"):
        for k in range(3):
            v = values(variant, k, rng)
            f = tile(v)
            assert f == op.filter_tile(v), f"{name} {variant} tile {k}"
            rc, out = op.unfilter_tile(f, v.nbytes)
            assert rc == 0 and np.array_equal(out, v.view(np.uint8))


def test_xor_known_answer_and_type_chain(oracle_mod):
    """XOR forward = x[j] ^ x[j-1] with x[0] kept (xor_filter.cc:149-177), its
    reverse the prefix XOR (:260-286); the output type is the signed integer of
    the input width (:63-78), so BWR after XOR on FLOAT32 is active."""
    from tiledb_amd.filter_pipeline import XORFilter, BitWidthReductionFilter
    x = np.array([5, 3, 3, 8, -1, 0x7FFFFFFF], dtype=np.int32)
    op = oracle_mod.OraclePipeline(P(XORFilter()).serialize(), 23, int(Datatype.INT32), 4)
    f = np.frombuffer(op.filter_tile(as_u8(x)), dtype=np.uint8)
    # tile header 8 + chunk header 12 + md [u32 nparts=1][u32 24] + data
    assert int(f[16:20].view(np.uint32)[0]) == 8
    assert f[20:28].view(np.uint32).tolist() == [1, 24]
    want = x.copy()
    want[1:] = x[1:] ^ x[:-1]
    assert np.array_equal(f[28:].view(np.int32), want)
    rc, back = op.unfilter_tile(f, x.nbytes)
    assert rc == 0 and np.array_equal(back.view(np.int32), x)
    # FLOAT32 -> XOR -> INT32: the BWR md then holds window entries
    v = (np.arange(1024) * 0.5).astype(np.float32)
    ser = P(XORFilter(), BitWidthReductionFilter(256)).serialize()
    fp = FilterPipeline.deserialize(ser, 23, Datatype.FLOAT32)
    assert fp.filters[1].filter_data_type == Datatype.INT32
    op2 = oracle_mod.OraclePipeline(ser, 23, int(Datatype.FLOAT32), 4)
    f2 = np.frombuffer(op2.filter_tile(as_u8(v)), dtype=np.uint8)
    md_len = int(f2[16:20].view(np.uint32)[0])
    assert md_len == 8 + 16 * 9 + 8  # BWR: orig, nwin, 16 x (i32, u8, u32); XOR: nparts, size
    rc, back = op2.unfilter_tile(f2, v.nbytes)
    assert rc == 0 and np.array_equal(back.view(np.float32), v)


def test_delta_known_answer(oracle_mod):
    """DELTA part = [u64 num][T x0][T x[i]-x[i-1]...] (delta_compressor.cc:224-249) in the
    compression frame [u32 n_md][u32 n_data][u32 orig][u32 comp] (compression_filter.cc:240-301)."""
    from tests.cases import DELTA
    x = np.array([10, 7, 7, 20], dtype=np.int32)
    op = oracle_mod.OraclePipeline(P(DELTA()).serialize(), 23, int(Datatype.INT32), 4)
    f = np.frombuffer(op.filter_tile(as_u8(x)), dtype=np.uint8)
    assert int(f[16:20].view(np.uint32)[0]) == 16
    assert f[20:36].view(np.uint32).tolist() == [0, 1, 16, 24]
    assert int(f[36:44].view(np.uint64)[0]) == 4
    assert f[44:60].view(np.int32).tolist() == [10, -3, 0, 13]
    rc, back = op.unfilter_tile(f, x.nbytes)
    assert rc == 0 and np.array_equal(back.view(np.int32), x)
    # num claims more values than the part holds: the read fails first
    g = f.copy()
    g[36] = 5
    rc, _ = op.unfilter_tile(g, x.nbytes)
    assert rc == 5  # TDBG_E_DATA_READ


def test_float_scale_known_answer(oracle_mod):
    """FLOAT_SCALE: stored W = round((x - offset) / scale) in T (float_scaling_filter.cc:60-99),
    read back as T(scale * T(W) + offset) (:164-197); descriptor = FilterConfig (24 B)."""
    from tiledb_amd.filter_pipeline import FloatScalingFilter
    x = np.array([1.0, 1.26, -2.5, 100.0], dtype=np.float32)
    fp = P(FloatScalingFilter(0.5, 1.0, 2))
    ser = fp.serialize()
    assert ser[8:13] == bytes([15, 24, 0, 0, 0])
    assert FilterPipeline.deserialize(ser, 23, Datatype.FLOAT32).serialize() == ser
    op = oracle_mod.OraclePipeline(ser, 23, int(Datatype.FLOAT32), 4)
    assert op.serialize() == ser
    f = np.frombuffer(op.filter_tile(as_u8(x)), dtype=np.uint8)
    assert f[20:28].view(np.uint32).tolist() == [1, 8]
    assert f[28:36].view(np.int16).tolist() == [0, 1, -7, 198]   # round(0.52) = 1
    rc, back = op.unfilter_tile(f, x.nbytes)
    assert rc == 0
    assert back.view(np.float32).tolist() == [1.0, 1.5, -2.5, 100.0]
