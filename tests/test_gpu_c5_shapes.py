"""GPU parity of the C5 tile kernel (tdbg_c5tile.hip) on chunk shapes other
than 64 KiB: TileDB cuts a tile into chunks of max(cell, floor(min(64 KiB,
tile) / cell) * cell) bytes (tile.cc:87-100; filter_pipeline.cc:151-206 and
:439-517 for the reverse walk), so tiles under 64 KiB, cell sizes that do not
divide 64 KiB (12-B cells: 65,532-B chunks) and short last chunks are
TileDB's everyday unit of work, not edge cases.

[BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION(256)] on INT32 / UINT32,
bit-exact against the oracle (statuses and bytes), with the kernel's
counters proving which tiles / chunks it took: every chunk of 4 n bytes
(16 <= n <= 16,384 values) whose BWR windows are a power of two >= 256 B,
whatever n mod 4 (the byte planes then start at every byte alignment of the
BWR output) and whatever the output's 4-B alignment.
"""
from __future__ import annotations

import numpy as np
import pytest

import workloads as W
from tests.cases import Case, DD, P, as_u8
from tiledb_amd.filter_pipeline import BitWidthReductionFilter, ByteshuffleFilter, Datatype

pytestmark = pytest.mark.gpu

MIN_TILES = 320  # a tile-mode launch (at least one tile per CU)


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from tiledb_amd import engine
    return engine


@pytest.fixture(scope="module")
def ctx(eng):
    return eng.Context(0)


def _pipe():
    return P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256))


def values(variant: str, n: int, rng, k: int = 0) -> np.ndarray:
    """n int32 values: SURVEY's C5 variants, or 'step<b>' (DD bitsize ~b:
    every code width of the coded-DD path)."""
    if variant.startswith("step"):
        bits = int(variant[4:])
        out = np.zeros(n, dtype=np.int64)
        i, j = 0, 0
        while i < n:
            run = int(rng.integers(64, 512))
            out[i:i + run] = 0 if j == 0 else (1 << bits) - 1 if j == 1 else rng.integers(0, 1 << bits)
            i += run
            j += 1
        # (values whose byteshuffle is the step stream)
        s = out.astype(np.int32)
        return s.astype("<i4").view(np.uint8).reshape(4, n).T.reshape(-1).view("<i4").copy()
    return W.c5_values(variant, k, rng, n)


def chunk_taken(f: np.ndarray, off: int = 8) -> bool:
    """The C5 tile kernel decodes this chunk (header at `off`): BWR window 0
    a power of two in [256, 4096] B (the encoder's window is min(256, L))
    and a DoubleDelta part that is raw or bit-packed with bitsize >= 1."""
    orig, fl, ml = (int(x) for x in np.frombuffer(f[off:off + 12].tobytes(), dtype="<u4"))
    m = off + 12
    nwin = int(np.frombuffer(f[m + 4:m + 8].tobytes(), dtype="<u4")[0])
    ws = int(np.frombuffer(f[m + 13:m + 17].tobytes(), dtype="<u4")[0])
    return orig >= 64 and orig % 4 == 0 and ws >= 256 and ws & (ws - 1) == 0 and nwin <= 320


def _tile_mode(eng, ctx, O, case, align=1):
    """Tile-mode launch of >= MIN_TILES tiles cycling over the case's tiles:
    bit-exact vs the oracle; returns (tiles, fused, fallback, streamed)."""
    from tests.test_gpu_parity import check_parity_replicated, encode
    _, enc = encode(O, case)
    assert len(enc) == len(case.tiles)
    n = max(MIN_TILES, len(enc))
    f0, b0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    check_parity_replicated(eng, ctx, O, case, enc, n, align=align)
    f1, b1, _ = ctx.path_stats()
    idx = np.arange(n) % len(enc)
    want = sum(chunk_taken(enc[i][0]) for i in idx)
    return enc, n, f1 - f0, b1 - b0, ctx.stream_tiles() - s0, want


@pytest.mark.parametrize("align", [1, 16])
@pytest.mark.parametrize("variant", ["rand", "ramp", "active"])
def test_c5_40000B_tiles(eng, ctx, oracle_mod, variant, align):
    """40,000-B tiles (10,000 values, one chunk), the bench's c5s leg: every
    tile taken by the C5 tile kernel, raw-DD (rand, ramp) and coded (active)."""
    rng = np.random.default_rng(101 + len(variant))
    vals = [values(variant, 10000, rng, k) for k in range(12)]
    case = Case(f"c5_40000_{variant}", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case, align)
    assert want == n
    assert fb == 0 and fused == n
    assert st == n, f"C5 tile kernel took {st} of {n}"


# n mod 4 = 0, 1, 2, 3 (orig mod 16 = 0, 4, 8, 12) at small, middle and
# near-64 KiB sizes, plus tiles too small for 256-B windows (declined)
_SIZES = [64, 76, 260, 1000, 1004, 4100, 4104, 4108, 40000, 40004, 40008, 40012, 65520, 65524, 65528, 65532]


@pytest.mark.parametrize("variant", ["rand", "ramp", "active", "step3", "step17", "step30"])
def test_c5_every_size_class(eng, ctx, oracle_mod, variant):
    """One launch of tiles of every size class (mixed sizes back to back, so
    outputs start at every 4-B alignment): bit-exact, and the kernel takes
    exactly the tiles whose windows it decodes."""
    rng = np.random.default_rng(202 + sum(map(ord, variant)))
    vals = [values(variant, nb // 4, rng, k) for k, nb in enumerate(_SIZES)]
    case = Case(f"c5_sizes_{variant}", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case)
    assert want >= n // 2, want
    assert fb == 0
    assert st == want, f"C5 tile kernel took {st}, expected {want}"


def test_c5_sizes_uint32(eng, ctx, oracle_mod):
    """UINT32 (BWR zero-extends its windows) at n mod 4 = 1, 2, 3."""
    rng = np.random.default_rng(303)
    vals = [values(v, nb // 4, rng, k).view(np.uint32) for k, (v, nb) in
            enumerate((v, nb) for v in ("ramp", "active", "step9") for nb in (40004, 40008, 65532))]
    case = Case("c5_sizes_u32", _pipe(), Datatype.UINT32, 4, [as_u8(v) for v in vals])
    enc, n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case)
    assert want == n and fb == 0 and st == n


def _chunk_headers(t):
    n = int(np.frombuffer(t[:8].tobytes(), dtype=np.uint64)[0])
    o, hs = 8, []
    for _ in range(n):
        orig, fl, ml = (int(x) for x in np.frombuffer(t[o:o + 12].tobytes(), dtype=np.uint32))
        hs.append(o)
        o += 12 + ml + fl
    return hs


def _chunk_mode(eng, ctx, O, ser, dtype, cell, vals, ntiles, fill=0):
    """Chunk-parallel launch (device chunk directory) of ntiles tiles cycling
    over vals: bit-exact vs the oracle; returns (chunks the kernel should
    take, chunks it took, chunks in all)."""
    op = O.OraclePipeline(ser, 23, int(dtype), cell)
    dp = eng.DevicePipeline(ser, 23, int(dtype), cell)
    enc = [np.frombuffer(op.filter_tile(as_u8(v)), dtype=np.uint8) for v in vals]
    filt = [enc[i % len(enc)] for i in range(ntiles)]
    osz = [vals[i % len(vals)].nbytes for i in range(ntiles)]
    batch = eng.TileBatch.from_host(filt, osz, fill=fill)
    c0 = ctx.stream_chunks()
    st = ctx.unfilter(dp, batch, chunk_parallel=True)
    took = ctx.stream_chunks() - c0
    assert not st.any()
    out = batch.outputs_host()
    for i in range(ntiles):
        o = int(batch.out_off[i])
        assert np.array_equal(out[o:o + osz[i]], as_u8(vals[i % len(vals)])), f"tile {i}"
    want = sum(sum(chunk_taken(f, h) for h in _chunk_headers(f)) for f in filt)
    total = sum(len(_chunk_headers(f)) for f in filt)
    del dp
    return want, took, total


@pytest.mark.parametrize("variant", ["rand", "active"])
def test_c5_12B_cells_65532B_chunks(eng, ctx, oracle_mod, variant):
    """INT32 with 12-B cells (3 values per cell): chunks of 65,532 B
    (16,383 values, planes at byte shifts 2, 1, 0, 3 of the BWR output),
    chunk outputs 4-B aligned.  Chunk mode: every chunk taken."""
    rng = np.random.default_rng(404)
    ser = P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256)).serialize()
    vals = [np.concatenate([values(variant, 16383, rng, 3 * k + c) for c in range(3)]) for k in range(4)]
    vals.append(values(variant, 16383, rng, 99))  # a one-chunk tile
    want, took, total = _chunk_mode(eng, ctx, oracle_mod, ser, Datatype.INT32, 12, vals, 24)
    assert total == 20 * 3 + 4 and want == total
    assert took == want


def test_c5_12B_cells_tile_mode(eng, ctx, oracle_mod):
    """12-B cells, one 65,532-B chunk per tile, tile mode: every tile taken."""
    rng = np.random.default_rng(405)
    vals = [values(v, 16383, rng, k) for k, v in enumerate(["rand", "ramp", "active", "step21"] * 2)]
    case = Case("c5_cell12", _pipe(), Datatype.INT32, 12, [as_u8(v) for v in vals])
    enc, n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case)
    assert want == n and fb == 0 and st == n


@pytest.mark.parametrize("variant", ["ramp", "active"])
def test_c5_1MiB_plus_4B_tiles(eng, ctx, oracle_mod, variant):
    """1 MiB + 4 B tiles (262,145 values): 16 chunks of 64 KiB and a last
    chunk of one value (4 B: too small for the tile kernel, decoded by the
    fused kernel).  Chunk mode: the 16 full chunks of every tile taken."""
    rng = np.random.default_rng(505)
    ser = W.c5_pipeline_bytes()
    vals = [np.concatenate([values(variant, 16384, rng, 16 * k + c) for c in range(16)] +
                           [values(variant, 1, rng, 7)]) for k in range(3)]
    want, took, total = _chunk_mode(eng, ctx, oracle_mod, ser, Datatype.INT32, 4, vals, 6, fill=0x33)
    assert total == 6 * 17 and want == 6 * 16
    assert took == want


def test_c5_short_last_chunks(eng, ctx, oracle_mod):
    """Tiles of 16 chunks whose last chunk holds 1..15 values more than a
    multiple of 4 (every n mod 4): chunk mode, every chunk of >= 16 values
    taken, bit-exact."""
    rng = np.random.default_rng(606)
    ser = W.c5_pipeline_bytes()
    vals = []
    for k, last in enumerate((16, 17, 18, 19, 1001, 4098, 16383)):
        v = "rand" if k % 2 else "active"
        vals.append(np.concatenate([values(v, 16384, rng, 16 * k + c) for c in range(15)] +
                                   [values(v, last, rng, 3)]))
    want, took, total = _chunk_mode(eng, ctx, oracle_mod, ser, Datatype.INT32, 4, vals, 14)
    assert want >= 14 * 15 and took == want


# a tile-mode launch of multi-chunk tiles: at least two tiles per CU (fewer
# go through the device chunk directory, tdbg_host.cpp launch())
MC_TILES = 544


def _mc_taken(f: np.ndarray) -> bool:
    """The multi-chunk variant takes the tile: every chunk one the tile
    kernel decodes (the tile is declined whole otherwise)."""
    return all(chunk_taken(f, h) for h in _chunk_headers(f))


def _mc_tile_mode(eng, ctx, O, case, n=MC_TILES, align=1):
    """TDBG_MULTI_CHUNK tile-mode launch (the engine's default for tiles over
    64 KiB) of n tiles cycling over the case's: bit-exact vs the oracle and
    identical statuses; returns (expected chunks, chunks taken, tiles the
    kernel should take, tiles the tile kernels took, fallback)."""
    from tests.test_gpu_parity import check_parity_replicated, encode
    import torch
    assert n >= 2 * torch.cuda.get_device_properties(0).multi_processor_count
    _, enc = encode(O, case)
    f0, b0, _ = ctx.path_stats()
    s0, k0, c0 = ctx.stream_tiles(), ctx.tile_chunks(), ctx.stream_chunks()
    check_parity_replicated(eng, ctx, O, case, enc, n, align=align, chunk_parallel=None)
    f1, b1, _ = ctx.path_stats()
    idx = np.arange(n) % len(enc)
    want_tiles = sum(_mc_taken(enc[i][0]) for i in idx)
    want_chunks = sum(len(_chunk_headers(enc[i][0])) for i in idx if _mc_taken(enc[i][0]))
    assert ctx.stream_chunks() == c0, "tile mode expected, not the chunk directory"
    return want_chunks, ctx.tile_chunks() - k0, want_tiles, ctx.stream_tiles() - s0, b1 - b0


@pytest.mark.parametrize("align", [1, 16])
def test_c5_multichunk_tile_mode(eng, ctx, oracle_mod, align):
    """multi-chunk tiles in tile mode on the C5 tile kernel
    (FilterPipeline::run_reverse's loop over chunks, filter_pipeline.cc:
    439-517): 2, 3 and 4-chunk tiles, raw (rand, ramp) and coded (active,
    step) chunks mixed inside a tile, short last chunks of every n mod 4.
    Every tile whose chunks the kernel decodes is taken whole, chunk by
    chunk (counter TDBG_STAT_TILE_CHUNKS); a tile with a chunk too small for
    256-B windows goes to the fused kernel whole; bit-exact either way."""
    rng = np.random.default_rng(707)
    vals = []
    for k, (kinds, last) in enumerate([(("rand", "active"), 16384), (("active", "ramp", "rand"), 16384),
                                       (("ramp", "ramp"), 1001), (("step17", "active", "rand"), 4098),
                                       (("rand", "rand", "active", "ramp"), 16383), (("active",), 2),
                                       (("step3", "step30"), 40000 // 4 + 1)]):
        parts = [values(v, 16384, rng, 8 * k + c) for c, v in enumerate(kinds)]
        parts.append(values(kinds[-1], last, rng, 8 * k + 7))
        vals.append(np.concatenate(parts))
    case = Case("c5_mc", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    want_c, took_c, want_t, took_t, fb = _mc_tile_mode(eng, ctx, oracle_mod, case, align=align)
    # (the fused kernel passes the 2-value chunk's tiles on to the general
    # interpreter: only tiles the tile kernel declined may fall back)
    assert fb <= MC_TILES - want_t
    assert want_t < MC_TILES and want_t > MC_TILES // 2  # (the 2-value last chunk's tiles are declined)
    assert took_c == want_c, f"took {took_c} chunks, expected {want_c}"
    assert took_t == want_t


def test_c5_multichunk_tile_mode_corrupt(eng, ctx, oracle_mod):
    """Multi-chunk tiles whose later chunk is malformed (an original size that
    breaks the tile's unfiltered size, tile.cc:305-309; a BWR window size off
    the tile kernel's shapes; a chunk header pointing past the tile): the
    tile kernel declines them whole after writing earlier chunks, and the
    statuses are the oracle's (bytes compared for good tiles only)."""
    from tests.test_gpu_parity import encode
    rng = np.random.default_rng(808)
    vals = [np.concatenate([values(v, 16384, rng, 3 * k + c) for c, v in enumerate(("rand", "active", "ramp"))])
            for k in range(4)]
    case = Case("c5_mc_bad", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    op, enc = encode(oracle_mod, case)
    tiles = [e[0].copy() for e in enc]
    h = _chunk_headers(tiles[1])
    tiles[1][h[2]:h[2] + 4] = np.frombuffer(np.uint32(65532).tobytes(), dtype=np.uint8)  # orig of chunk 2
    h = _chunk_headers(tiles[2])
    tiles[2][h[1] + 4:h[1] + 8] = np.frombuffer(np.uint32(1 << 30).tobytes(), dtype=np.uint8)  # filtered past the tile
    dp = eng.DevicePipeline(case.serialized, 23, int(Datatype.INT32), 4)
    refs = [op.unfilter_tile(t, e[2]) for t, e in zip(tiles, enc)]
    assert refs[0][0] == 0 and refs[3][0] == 0 and refs[1][0] != 0 and refs[2][0] != 0
    idx = np.arange(MC_TILES) % len(tiles)
    batch = eng.TileBatch.from_host([tiles[i] for i in idx], [enc[i][2] for i in idx])
    k0 = ctx.tile_chunks()
    st = ctx.unfilter(dp, batch)
    out = batch.outputs_host()
    for k, i in enumerate(idx):
        assert int(st[k]) == refs[i][0], f"tile {k}: status {st[k]} oracle {refs[i][0]}"
        if refs[i][0] == 0:
            o = int(batch.out_off[k])
            assert np.array_equal(out[o:o + enc[i][2]], refs[i][1]), f"tile {k}"
    assert ctx.tile_chunks() - k0 == 3 * sum(1 for i in idx if refs[i][0] == 0)
