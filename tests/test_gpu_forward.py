"""GPU parity of the forward (filter) direction: tdbg_filter_tiles_* against
the oracle's FilterPipeline::run_forward restatement (oracle_filter_tile) --
bit-exact filtered tiles, identical statuses on inputs the reference rejects,
and the round trip through the device unfilter.  The BWR offset of a window
whose range overflows T (uninitialized in the reference,
bit_width_reduction_filter.cc:421-430) is written as 0 by both sides, so
those bytes compare exactly here but are parity-unpinned against the
reference itself.
"""
from __future__ import annotations

import numpy as np
import pytest

from tests.cases import config_cases, edge_cases, fused_spec_cases, random_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from tiledb_amd import engine
    return engine


@pytest.fixture(scope="module")
def ctx(eng):
    return eng.Context(0)


def forward_parity(eng, ctx, O, case, roundtrip=True):
    if case.offsets:
        pytest.skip("var-size chunking (offsets) is not on the forward device path")
    op = O.OraclePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    st, got = ctx.filter(dp, case.tiles, max_chunk=case.max_chunk)
    for i, t in enumerate(case.tiles):
        try:
            ref = np.frombuffer(op.filter_tile(t, None, case.max_chunk), dtype=np.uint8)
            rc = 0
        except O.OracleError as e:
            ref, rc = None, e.code
        assert int(st[i]) == rc, f"{case.name} tile {i}: gpu status {st[i]} oracle {rc}"
        if rc:
            continue
        if not np.array_equal(got[i], ref):
            n = min(got[i].size, ref.size)
            bad = np.nonzero(got[i][:n] != ref[:n])[0]
            raise AssertionError(f"{case.name} tile {i}: sizes {got[i].size}/{ref.size}, "
                                 f"{bad.size} bytes differ, first at {bad[:1]}")
    if roundtrip:
        ok = [i for i in range(len(case.tiles)) if st[i] == 0]
        if ok:
            osz = [case.tiles[i].size + (8 if case.offsets_tile else 0) for i in ok]
            batch = eng.TileBatch.from_host([got[i] for i in ok], osz)
            rst = ctx.unfilter(dp, batch, offsets_tiles=case.offsets_tile)
            assert not rst.any()
            for k, i in enumerate(ok):
                # lossy stages (float scale) do not restore the input: the
                # round trip is checked against the oracle's unfilter instead
                urc, want = op.unfilter_tile(got[i], osz[k], case.offsets_tile)
                assert urc == 0
                assert np.array_equal(batch.output(k)[: case.tiles[i].size], want[: case.tiles[i].size])
    return st


_CONFIG = config_cases(3)
_EDGE = edge_cases()
_SPECS = fused_spec_cases(2)


@pytest.mark.parametrize("case", _CONFIG + _SPECS, ids=[c.name for c in _CONFIG + _SPECS])
def test_forward_config_parity(eng, ctx, oracle_mod, case):
    forward_parity(eng, ctx, oracle_mod, case)


@pytest.mark.parametrize("case", _EDGE, ids=[c.name for c in _EDGE])
def test_forward_edge_parity(eng, ctx, oracle_mod, case):
    forward_parity(eng, ctx, oracle_mod, case)


def test_forward_random_pipelines(eng, ctx, oracle_mod):
    n = 0
    for case in random_cases(120):
        if case.offsets:
            continue
        forward_parity(eng, ctx, oracle_mod, case)
        n += 1
    assert n > 100


def test_forward_rejections(eng, ctx, oracle_mod):
    """Inputs the reference rejects on write: decreasing positive-delta data,
    DoubleDelta int64 overflow, DoubleDelta on floats (statuses equal the oracle's)."""
    from tests.cases import Case, P, DD, RLE, as_u8
    from tiledb_amd.filter_pipeline import Datatype, PositiveDeltaFilter
    cases = [
        Case("pd_decreasing", P(PositiveDeltaFilter(64)), Datatype.UINT32, 4,
             [as_u8(np.array([5, 4, 3] * 50, dtype=np.uint32))]),
        Case("dd_overflow_i64", P(DD()), Datatype.INT64, 8,
             [as_u8(np.array([-2**63, 2**63 - 1, 0, 5], dtype=np.int64))]),
        Case("dd_float", P(DD()), Datatype.FLOAT32, 4, [as_u8(np.arange(100, dtype=np.float32))]),
    ]
    for c in cases:
        st = forward_parity(eng, ctx, oracle_mod, c, roundtrip=False)
        assert st[0] != 0, c.name
    # a tile that is not a multiple of the cell is chunked at cell multiples
    # (the 2-byte tail chunk holds no whole cell): accepted by both sides
    c = Case("rle_ragged", P(RLE()), Datatype.UINT8, 4, [np.arange(10, dtype=np.uint8)])
    assert forward_parity(eng, ctx, oracle_mod, c, roundtrip=False)[0] == 0


def test_forward_sync_statuses_after_status_buffer_growth(eng, oracle_mod):
    """tdbg_filter_tiles_sync on a fresh context, first with one tile, then
    with more tiles than its status buffer holds: the buffer grows before
    the kernel is handed its address, so the statuses read back are the ones
    the kernel wrote (a rejected tile among them keeps its error; before the
    fix the kernel wrote into the freed buffer and the copy read the new,
    unwritten one)."""
    from tests.cases import Case, P, as_u8
    from tiledb_amd.filter_pipeline import Datatype, PositiveDeltaFilter
    ctx = eng.Context(0)
    good = as_u8(np.arange(1000, dtype=np.uint32))
    bad = as_u8(np.array([5, 4, 3] * 50, dtype=np.uint32))
    forward_parity(eng, ctx, oracle_mod, Case("pd_one", P(PositiveDeltaFilter(64)), Datatype.UINT32, 4, [good]),
                   roundtrip=False)
    for n in (40, 3000):
        tiles = [good] * n
        tiles[n // 2] = bad
        st = forward_parity(eng, ctx, oracle_mod,
                            Case(f"pd_{n}", P(PositiveDeltaFilter(64)), Datatype.UINT32, 4, tiles), roundtrip=False)
        assert st[n // 2] != 0 and not np.delete(st, n // 2).any()


@pytest.mark.parametrize("kind", ["c3a_u64", "c3a_i64", "c3b_u64", "c4_u64"])
def test_forward_small_kernel(eng, ctx, oracle_mod, kind):
    """The LDS-resident forward kernel of the scan configs
    (tdbg_forward_small.hip): C3a [DOUBLE_DELTA] on uint64 / int64 and C3b
    [RLE] with 8-byte cells and C4 [POSITIVE_DELTA(1024), BWR(256)] on uint64,
    320 tiles bit-exact with the oracle (statuses too).  The
    kernel takes the SURVEY coordinate tiles, constant tiles and DD bit sizes
    up to 30; it leaves to the general kernel (same bytes and statuses) the
    tiles it does not build -- values at or beyond 2^61, DD bit sizes above
    30, more than 2,048 RLE runs, decreasing or wide C4 deltas -- and the
    stats count exactly the ones it took."""
    import workloads as W
    from tests.cases import Case, P, DD, RLE, as_u8
    from tiledb_amd.filter_pipeline import Datatype
    rng = np.random.default_rng(71)
    signed = kind == "c3a_i64"
    dt = np.int64 if signed else np.uint64
    uniq, took = [], []
    for k in range(8):  # SURVEY C3 coordinates (runs of 64, small gaps)
        uniq.append(W.c3_values(k, rng).astype(dt))
        took.append(True)
    uniq.append(np.full(8192, 7, dtype=dt))  # one run, bit size 1
    took.append(True)
    if kind == "c4_u64":
        uniq, took = [], []
        for k in range(8):  # SURVEY C4 offsets (lengths U{0..32})
            uniq.append(W.c4_values(k, rng))
            took.append(True)
        uniq.append(np.full(8192, 5, dtype=np.uint64))
        took.append(True)
        v = W.c4_values(9, rng)
        v[5000] = v[4999] - np.uint64(1)  # decreasing inside a window: the reference's error
        uniq.append(v)
        took.append(False)
        v = W.c4_values(10, rng)
        v[4096:] += np.uint64(1 << 40)  # a jump at a window start: no error, one raw-free window
        uniq.append(v)
        took.append(True)
        uniq.append(np.cumsum(rng.integers(0, 1 << 12, 8192)).astype(np.uint64))  # 16-bit windows: 20 KB of data
        took.append(True)
        uniq.append(np.cumsum(rng.integers(0, 1 << 20, 8192)).astype(np.uint64))  # 32-bit windows: too big here
        took.append(False)
    elif kind == "c3b_u64":
        uniq.append(np.arange(8192, dtype=dt))  # 8192 runs: general kernel
        took.append(False)
        uniq.append(np.repeat(np.arange(2048, dtype=dt), 4))  # exactly 2,048 runs
        took.append(True)
        uniq.append(np.repeat(np.arange(4096, dtype=dt), 2))  # 4,096 runs
        took.append(False)
    else:
        def walk(b):  # double deltas in [-2^b, 2^b), values shifted to >= 0 (< 2^(b + 26))
            v = np.cumsum(np.cumsum(rng.integers(-(1 << b), 1 << b, 8192)))
            return (v - v.min()).astype(dt)
        for b in (5, 14, 28):  # bit sizes up to 30: this kernel
            uniq.append(walk(b))
            took.append(True)
        uniq.append(walk(33))  # bit size > 30: the general kernel
        took.append(False)
        big = np.arange(8192, dtype=np.uint64) + np.uint64(1 << 61)  # beyond 2^61
        uniq.append(big.astype(dt) if not signed else (-big.astype(np.int64)).astype(dt))
        took.append(False)
        if signed:
            uniq.append((np.arange(8192, dtype=np.int64) - (1 << 61)).astype(dt))  # -2^61 is inside
            took.append(True)
    idx = [i % len(uniq) for i in range(320)]
    tiles = [as_u8(uniq[i]) for i in idx]
    from tiledb_amd.filter_pipeline import BitWidthReductionFilter, PositiveDeltaFilter
    pipe = (P(RLE()) if kind == "c3b_u64" else
            P(PositiveDeltaFilter(1024), BitWidthReductionFilter(256)) if kind == "c4_u64" else P(DD()))
    case = Case(kind, pipe, Datatype.INT64 if signed else Datatype.UINT64, 8, tiles)
    s0 = ctx.forward_stream_tiles()
    st = forward_parity(eng, ctx, oracle_mod, case)  # (statuses equal the oracle's)
    assert (st != 0).sum() == (sum(1 for i in idx if i == 9) if kind == "c4_u64" else 0)
    assert ctx.forward_stream_tiles() - s0 == sum(took[i] for i in idx)


@pytest.mark.parametrize("kind", ["c1_i32", "c2_f32", "c2_bitshuffle_only", "c2i_i32", "c2i_u32"])
def test_forward_shuffle_kernel(eng, ctx, oracle_mod, kind):
    """The shuffle forward kernel (tdbg_forward_shuffle.hip): C1 [BYTESHUFFLE],
    C2 [BITSHUFFLE, BWR] on FLOAT32 (BWR a pass-through) and [BITSHUFFLE]
    alone, C2i [BITSHUFFLE, BWR(256)] on INT32 / UINT32 -- 320 tiles
    bit-exact with the oracle, 8/16/32-bit and raw BWR windows, and the
    stats count exactly the 64 KiB tiles it took (a shorter tile goes to the
    general kernel)."""
    import workloads as W
    from tests.cases import Case, P, as_u8
    from tiledb_amd.filter_pipeline import BitshuffleFilter, BitWidthReductionFilter, ByteshuffleFilter, Datatype
    rng = np.random.default_rng(83)
    uniq = []
    for k in range(6):
        if kind == "c1_i32":
            uniq.append(W.c1_values("rand" if k % 2 else "ramp", k, rng).astype(np.int32))
        else:
            uniq.append(W.c2_values(k, rng))
    if kind != "c1_i32":
        # windows of every width after the bitshuffle: small ints (sparse
        # bit rows, 8-bit), noisy ramps, full-range random (raw)
        uniq.append(np.arange(16384, dtype=np.int32).view(np.float32))
        uniq.append(rng.integers(-2**31, 2**31, 16384, dtype=np.int64).astype(np.int32).view(np.float32))
        uniq.append((rng.integers(0, 7, 16384) * 1000).astype(np.int32).view(np.float32))
    dt = {"c1_i32": Datatype.INT32, "c2_f32": Datatype.FLOAT32, "c2_bitshuffle_only": Datatype.FLOAT32,
          "c2i_i32": Datatype.INT32, "c2i_u32": Datatype.UINT32}[kind]
    pipe = {"c1_i32": P(ByteshuffleFilter()), "c2_bitshuffle_only": P(BitshuffleFilter())}.get(
        kind, P(BitshuffleFilter(), BitWidthReductionFilter(256)))
    tiles = [as_u8(uniq[i % len(uniq)]) for i in range(320)]
    tiles[-1] = tiles[-1][:-8]  # not 64 KiB: the general kernel (last: the packed inputs stay 16-B aligned)
    case = Case(kind, pipe, dt, 4, tiles)
    s0 = ctx.forward_stream_tiles()
    st = forward_parity(eng, ctx, oracle_mod, case)
    assert not st.any()
    assert ctx.forward_stream_tiles() - s0 == 319


def test_forward_full_size_c5(eng, ctx, oracle_mod):
    """A BASELINE C5 shard's worth of tiles (2,000 x 64 KiB, active + ramp +
    rand): forward on the device, every tile equal to the oracle's bytes and
    the device round trip restores the values."""
    import workloads as W
    from tests.cases import c5_tiles, P, DD, Case
    from tiledb_amd.filter_pipeline import ByteshuffleFilter, BitWidthReductionFilter, Datatype
    rng = np.random.default_rng(4)
    uniq = (c5_tiles(8, "ramp") + c5_tiles(8, "rand") +
            [W.c5_values("active", k, rng).view(np.uint8) for k in range(16)])
    tiles = [uniq[i % len(uniq)] for i in range(2000)]
    case = Case("c5_full", P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256)), Datatype.INT32, 4,
                tiles)
    forward_parity(eng, ctx, oracle_mod, case)


def test_forward_stream_c5_kernel(eng, ctx, oracle_mod):
    """The LDS-resident C5 forward kernel (tdbg_forward_stream.hip): every DD
    bit size (raw and coded, 1..32), active / ramp / rand tiles, INT32 and
    UINT32, bit-exact with the oracle, and proven to have filtered them
    (tdbg_context_forward_stream_stats)."""
    import workloads as W
    from tests.cases import c5_tiles, P, DD, Case
    from tests.test_gpu_c5tile import step_values
    from tiledb_amd.filter_pipeline import ByteshuffleFilter, BitWidthReductionFilter, Datatype
    rng = np.random.default_rng(61)
    vals = [step_values(b, rng) for b in range(1, 33)]
    vals += [W.c5_values(v, k, rng) for v in ("active", "ramp", "rand") for k in range(3)]
    vals.append(np.zeros(16384, dtype=np.int32))
    vals.append(np.full(16384, -7, dtype=np.int32))
    pipe = P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256))
    for dt, cast in ((Datatype.INT32, np.int32), (Datatype.UINT32, np.uint32)):
        tiles = [np.ascontiguousarray(v).view(cast).view(np.uint8) for v in vals]
        f0 = ctx.forward_stream_tiles()
        forward_parity(eng, ctx, oracle_mod, Case(f"c5fs_{int(dt)}", pipe, dt, 4, tiles))
        assert ctx.forward_stream_tiles() - f0 == len(tiles)


def test_forward_stream_c5_declines(eng, ctx, oracle_mod):
    """Tiles the C5 forward kernel does not take (not 64 KiB, not 16-B
    aligned in the packed input, another BWR window, a different max chunk)
    run on the general forward kernel with the oracle's bytes; a 64 KiB tile
    at an aligned start next to them is still taken."""
    import workloads as W
    from tests.cases import P, DD, Case
    from tiledb_amd.filter_pipeline import ByteshuffleFilter, BitWidthReductionFilter, Datatype
    rng = np.random.default_rng(62)
    full = W.c5_values("active", 1, rng).view(np.uint8)
    odd = [full[:4000].copy(), full[:65532].copy(), np.concatenate([full, full[:400]])]
    pipe = P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256))
    f0 = ctx.forward_stream_tiles()
    # (ctx.filter packs the inputs back to back: the last full tile starts
    # 135,468 bytes in, not 16-B aligned)
    forward_parity(eng, ctx, oracle_mod, Case("c5fs_odd", pipe, Datatype.INT32, 4, [full] + odd + [full]))
    assert ctx.forward_stream_tiles() - f0 == 1
    f0 = ctx.forward_stream_tiles()
    forward_parity(eng, ctx, oracle_mod, Case("c5fs_w512", P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(512)),
                                              Datatype.INT32, 4, [full, full]))
    case = Case("c5fs_chunk", pipe, Datatype.INT32, 4, [full, full], max_chunk=16384)
    forward_parity(eng, ctx, oracle_mod, case)
    assert ctx.forward_stream_tiles() == f0
