"""GPU parity of the small-image streaming kernels for the scan pipelines on
8-byte values (tiledb_amd/csrc/tdbg_stream_small.hip): BASELINE C3a
[DOUBLE_DELTA], C3b [RLE] and C4 [POSITIVE_DELTA, BIT_WIDTH_REDUCTION],
through the C-ABI.

Bit-exact against the oracle, with the kernel proven to have taken the tiles
it is built for (tdbg_context_stream_stats): every DD code width cb = 2..7,
run tables up to the 8 KB staging (814 runs), BWR windows of 8/16/32 bits and raw,
signed and unsigned, PD windows of 2..64 lanes.  Tiles it declines (wider
codes, more runs, other window sizes, corrupted metadata, wrong output
sizes, offsets tiles) must come out exactly as the oracle says through the
fused kernel and the general interpreter behind it.
"""
from __future__ import annotations

import numpy as np
import pytest

import workloads as W
from tests.cases import DD, RLE, Case, P, as_u8
from tiledb_amd.filter_pipeline import BitWidthReductionFilter, Datatype, PositiveDeltaFilter

pytestmark = pytest.mark.gpu

MIN_TILES = 320  # launches below one tile per CU go chunk-parallel (no streaming kernel)


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from tiledb_amd import engine
    return engine


@pytest.fixture(scope="module")
def ctx(eng):
    return eng.Context(0)


def _run(eng, ctx, O, case, align=1):
    """Encode with the oracle, replicate to >= MIN_TILES tiles, check parity;
    returns (tiles, fused, fallback, streamed) deltas."""
    from tests.test_gpu_parity import check_parity, encode
    _, enc = encode(O, case)
    assert len(enc) == len(case.tiles)
    enc = enc * -(-MIN_TILES // len(enc))
    f0, b0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    check_parity(eng, ctx, O, case, [e[0] for e in enc], [e[2] for e in enc], [e[1] for e in enc], align=align)
    f1, b1, _ = ctx.path_stats()
    return enc, f1 - f0, b1 - b0, ctx.stream_tiles() - s0


def _taken_bounds(enc, cap):
    """(min, max) tiles the kernel can take by image size alone: an image
    of size + 15 <= cap fits at any alignment, one bigger than cap never."""
    return sum(e[0].size + 15 <= cap for e in enc), sum(e[0].size <= cap for e in enc)


def _pd_bwr(pd=1024, bwr=256):
    return P(PositiveDeltaFilter(pd), BitWidthReductionFilter(bwr))


# ---------------------------------------------------------------------------
# BASELINE configs
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("align", [1, 16])
@pytest.mark.parametrize("cfg", ["c3a", "c3b", "c4"])
def test_small_config_tiles(eng, ctx, oracle_mod, cfg, align):
    """SURVEY's C3a / C3b / C4 tiles: every one taken by the streaming kernel."""
    ser, dt, cs, values, tile = W.config(cfg)
    rng = np.random.default_rng(41)
    vals = [values("coords", k, rng) for k in range(16)]
    pipe = {"c3a": P(DD()), "c3b": P(RLE()), "c4": _pd_bwr()}[cfg]
    assert pipe.serialize() == ser
    case = Case(cfg, pipe, dt, cs, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case, align)
    for e in enc[:16]:  # the numpy encoders agree with the oracle's forward pass
        assert e[0].tobytes() == tile(e[1].view(np.uint64)) or cfg == "c4"
    assert fb == 0 and fused == len(enc)
    assert st == len(enc), f"streaming kernel took {st} of {len(enc)} tiles"


# ---------------------------------------------------------------------------
# DoubleDelta
# ---------------------------------------------------------------------------
def dd_values(bits: int, rng, n: int = 8192, signed=False) -> np.ndarray:
    """Values whose DoubleDelta bitsize is exactly `bits`: second differences
    below 2^bits in magnitude, one of them 2^bits - 1."""
    hi = (1 << bits) - 1
    dd = rng.integers(-hi, hi + 1, n - 2, dtype=np.int64) if bits < 62 else None
    dd = np.where(rng.random(n - 2) < 0.7, 0, dd)
    dd[int(rng.integers(0, n - 2))] = -hi if rng.random() < 0.5 else hi
    d = np.concatenate([[int(rng.integers(0, min(hi, 3) + 1))], dd]).cumsum()  # first delta small
    x0 = (1 << 60) + int(rng.integers(0, 1 << 40))  # the walk stays positive (no unsigned wrap)
    x = (np.concatenate([[0], d]).cumsum() + x0).astype(np.uint64)
    return x.view(np.int64) if signed else x


def test_small_dd_every_code_width(eng, ctx, oracle_mod):
    """DD bitsize 1..6 (code widths 2..7, every instantiation: the stream of
    8,192 values fits the kernel's 8 KB staging) taken; bitsize 7..40
    declined to the fused kernel; all bit-exact."""
    rng = np.random.default_rng(42)
    bits = list(range(1, 41))
    vals = [dd_values(b, rng) for b in bits]
    for b, v in zip(bits, vals):
        c = W.dd_fwd(v, 8)
        assert c[0] == b, (b, c[0])
    case = Case("c3a_widths", P(DD()), Datatype.UINT64, 8, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    rep = len(enc) // len(vals)
    assert fb == 0 and fused == len(enc)
    assert st == rep * sum(b <= 6 for b in bits), f"took {st}"


@pytest.mark.parametrize("dt", [Datatype.INT64, Datatype.UINT64, Datatype.DATETIME_NS])
def test_small_dd_types(eng, ctx, oracle_mod, dt):
    """8-byte DD types (values wrap modulo 2^64, negative and huge values)."""
    rng = np.random.default_rng(43 + int(dt))
    vals = [dd_values(int(b), rng, signed=True) for b in (1, 3, 5, 6)]
    vals.append(np.full(8192, -5, dtype=np.int64))          # all dd = 0
    vals.append((np.arange(8192, dtype=np.int64) * -3) - (1 << 62))
    case = Case("c3a_types", P(DD()), dt, 8, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and fused == len(enc) and st == len(enc)


# ---------------------------------------------------------------------------
# RLE
# ---------------------------------------------------------------------------
def rle_values(nruns: int, rng, n: int = 8192) -> np.ndarray:
    """uint64 cells in exactly `nruns` runs of random lengths."""
    cuts = np.sort(rng.choice(np.arange(1, n), nruns - 1, replace=False)) if nruns > 1 else np.array([], int)
    lens = np.diff(np.concatenate([[0], cuts, [n]]))
    vals = rng.integers(0, 1 << 63, nruns, dtype=np.int64).astype(np.uint64)
    for k in range(1, nruns):  # neighbours differ
        if vals[k] == vals[k - 1]:
            vals[k] += np.uint64(1)
    return np.repeat(vals, lens)


@pytest.mark.parametrize("nruns", [1, 2, 17, 130, 512, 800, 814, 820, 1025, 4000])
def test_small_rle_run_counts(eng, ctx, oracle_mod, nruns):
    """Tiles whose image (36 + 10 runs bytes) fits the 8 KB staging at any
    alignment (<= 814 runs) taken
    (one scan, 4 runs per thread); more runs are declined; random run
    boundaries, lane- and wave-crossing."""
    rng = np.random.default_rng(44 + nruns)
    vals = [rle_values(nruns, rng) for _ in range(4)]
    case = Case(f"c3b_runs{nruns}", P(RLE()), Datatype.UINT64, 8, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    if nruns <= 2047:  # (the fused kernel's run table: more go to the general interpreter)
        assert fb == 0 and fused == len(enc)
    assert st == (len(enc) if nruns <= 814 else 0)


def test_small_rle_types_and_cells(eng, ctx, oracle_mod):
    """8-byte cells of other types are taken; 4-byte cells (INT32) are not
    (the fused kernel runs them), bit-exact either way."""
    rng = np.random.default_rng(45)
    v64 = [rle_values(int(k), rng).view(np.int64) for k in (3, 64, 300)]
    case = Case("c3b_i64", P(RLE()), Datatype.INT64, 8, [as_u8(v) for v in v64])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and st == len(enc)
    v32 = [np.repeat(rng.integers(0, 1 << 31, 64), 256).astype(np.int32) for _ in range(3)]
    case = Case("c3b_i32", P(RLE()), Datatype.INT32, 4, [as_u8(v) for v in v32])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and st == 0


def test_small_rle_crafted_runs(eng, ctx, oracle_mod):
    """Hand-made RLE streams the encoder never writes (zero-length runs,
    adjacent equal runs): the kernel's run search must skip empty runs."""
    from tests.test_gpu_parity import check_parity
    import struct
    rng = np.random.default_rng(46)
    tiles = []
    for k in range(6):
        lens = rng.integers(0, 40, 400)
        lens[::7] = 0
        lens[-1] = 8192 - int(lens[:-1].sum()) if lens[:-1].sum() < 8192 else 0
        while lens.sum() > 8192:
            i = int(np.nonzero(lens)[0][-1])
            lens[i] -= min(lens[i], lens.sum() - 8192)
        assert lens.sum() == 8192
        vals = rng.integers(0, 1 << 63, lens.size, dtype=np.int64).astype(np.uint64)
        vals[1::5] = vals[0::5][: vals[1::5].size]  # equal neighbours
        recs = b"".join(struct.pack("<Q", int(v)) + bytes([int(n) >> 8, int(n) & 255]) for v, n in zip(vals, lens))
        tiles.append(np.frombuffer(W.tile_image(65536, W.comp_frame([], [(65536, len(recs))]), recs), dtype=np.uint8))
    tiles = tiles * -(-MIN_TILES // len(tiles))
    case = Case("c3b_crafted", P(RLE()), Datatype.UINT64, 8, [])
    s0 = ctx.stream_tiles()
    check_parity(eng, ctx, oracle_mod, case, tiles, [65536] * len(tiles))
    assert ctx.stream_tiles() - s0 == len(tiles)


# ---------------------------------------------------------------------------
# PD + BWR
# ---------------------------------------------------------------------------
def pd_values(kinds, rng, n: int = 8192, bwr: int = 256, signed=False, small=False) -> np.ndarray:
    """Nondecreasing values whose PD deltas, in BWR windows of `bwr` bytes,
    have the given kinds (cycled): 8, 16, 32 bits or 64 (raw).  small: every
    fourth window only (the rest 8-bit), so the image fits 16 KB."""
    per = bwr // 8
    d = np.empty(n, dtype=np.uint64)
    for wi in range(n // per):
        k = kinds[(wi // 4) % len(kinds)] if small and wi % 4 == 0 else 8 if small else kinds[wi % len(kinds)]
        top = {8: 100, 16: 30000, 32: 1 << 30, 64: 1 << 40}[k]
        d[wi * per:(wi + 1) * per] = rng.integers(0, top, per).astype(np.uint64)
        if k == 64:
            d[wi * per] = np.uint64(1 << 41)
    x = np.cumsum(d, dtype=np.uint64)
    if signed:
        return (x.view(np.int64) - (1 << 50)).astype(np.int64)
    return x


@pytest.mark.parametrize("kinds", [(8,), (16, 8), (8, 16, 32), (32, 64), (64,), (8, 8, 8, 64, 16)],
                         ids=lambda k: "w" + "_".join(map(str, k)))
@pytest.mark.parametrize("dt", [Datatype.UINT64, Datatype.INT64])
def test_small_pdbwr_window_kinds(eng, ctx, oracle_mod, kinds, dt):
    """BWR windows of every compressed width and raw, mixed within a wave
    (the general decoder) or all 8-bit (the fast one); signed and unsigned.
    The images that fit the kernel's 16 KB staging are taken, the others
    (many raw windows) declined."""
    rng = np.random.default_rng(47 + sum(kinds) + int(dt))
    vals = [pd_values(kinds, rng, signed=dt == Datatype.INT64, small=True) for _ in range(4)]
    case = Case("c4_kinds", _pd_bwr(), dt, 8, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    lo, hi = _taken_bounds(enc, 16384)
    assert fb == 0 and fused == len(enc) and lo <= st <= hi
    # 8/16/32-bit and raw windows each appear in some case whose images fit
    if kinds in ((8,), (16, 8), (8, 16, 32), (8, 8, 8, 64, 16)):
        assert lo == len(enc)


@pytest.mark.parametrize("pd,bwr,taken", [(256, 256, True), (512, 256, True), (2048, 512, True),
                                          (4096, 4096, True), (8192, 256, True), (128, 256, False),
                                          (1024, 128, False), (1536, 256, False), (1024, 384, False),
                                          (16384, 256, False)])
def test_small_pdbwr_window_sizes(eng, ctx, oracle_mod, pd, bwr, taken):
    """PD windows of 2..64 lanes and BWR windows >= 256 B (powers of two) are
    taken; smaller, bigger or non-power-of-two windows are declined."""
    rng = np.random.default_rng(pd + bwr)
    vals = [W.c4_values(k, rng) for k in range(4)]
    case = Case(f"c4_w{pd}_{bwr}", _pd_bwr(pd, bwr), Datatype.UINT64, 8, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    if taken:  # (declined ones: parity checked, whichever path ran them)
        assert fb == 0 and fused == len(enc)
    assert st == (len(enc) if taken else 0)


# ---------------------------------------------------------------------------
# declined and corrupted tiles
# ---------------------------------------------------------------------------
def _corrupt(pool, rng, extra_pos):
    tiles = []
    for f in pool:
        f = np.frombuffer(f, dtype=np.uint8)
        tiles.append(f.copy())
        ml = int(f[16:20].view("<u4")[0])
        data0 = 20 + ml
        for pos in [0, 8, 12, 16, 20, 24, 28, 32, data0, data0 + 1, f.size - 3] + extra_pos(f, ml, data0):
            if pos >= f.size:
                continue
            g = f.copy()
            g[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
            tiles.append(g)
        tiles.append(f[: f.size - 1].copy())
        tiles.append(f[: f.size // 2].copy())
    return tiles * -(-MIN_TILES // len(tiles))


@pytest.mark.parametrize("cfg", ["c3a", "c3b", "c4"])
def test_small_corrupted_tiles(eng, ctx, oracle_mod, cfg):
    """Bit flips in headers, metadata, frame and data, and truncations, get
    the oracle's status and bytes; intact tiles beside them stream."""
    from tests.test_gpu_parity import check_parity
    rng = np.random.default_rng(48)
    pool, _ = W.pool(cfg, "coords", 3, seed=49)
    extra = {"c3a": lambda f, ml, d0: [d0 + 5, d0 + 9, d0 + 17, d0 + 25, d0 + 200],
             "c3b": lambda f, ml, d0: [d0 + 8, d0 + 9, d0 + 18, d0 + 19, d0 + 500],
             # BWR md (orig, nwin, window 0, window 255), PD md (nwin, window 0), data
             "c4": lambda f, ml, d0: [36, 37, 40, 44, 28 + 13 * 255 + 9, 28 + 13 * 256, 28 + 13 * 256 + 4,
                                      28 + 13 * 256 + 12, 20 + ml - 4, d0 + 300]}[cfg]
    tiles = _corrupt(pool, rng, extra)
    ser, dt, cs, _, _ = W.config(cfg)
    pipe = {"c3a": P(DD()), "c3b": P(RLE()), "c4": _pd_bwr()}[cfg]
    case = Case(f"{cfg}_corrupt", pipe, dt, cs, [])
    s0 = ctx.stream_tiles()
    check_parity(eng, ctx, oracle_mod, case, tiles, [65536] * len(tiles))
    assert ctx.stream_tiles() > s0


@pytest.mark.parametrize("cfg", ["c3a", "c3b", "c4"])
def test_small_wrong_sizes_and_offsets(eng, ctx, oracle_mod, cfg):
    """Wrong output sizes are declined and get the oracle's status; the same
    tiles as offsets tiles (expected size - 8) too."""
    from tests.test_gpu_parity import check_parity
    pool, _ = W.pool(cfg, "coords", 4, seed=50)
    tiles = [np.frombuffer(f, dtype=np.uint8) for f in pool]
    tiles = tiles * -(-MIN_TILES // len(tiles))
    ser, dt, cs, _, _ = W.config(cfg)
    pipe = {"c3a": P(DD()), "c3b": P(RLE()), "c4": _pd_bwr()}[cfg]
    sizes = [65536 + (8 if i % 3 == 1 else -8 if i % 3 == 2 else 0) for i in range(len(tiles))]
    check_parity(eng, ctx, oracle_mod, Case(f"{cfg}_sizes", pipe, dt, cs, []), tiles, sizes)
    case = Case(f"{cfg}_offs", pipe, dt, cs, [], offsets_tile=True)
    check_parity(eng, ctx, oracle_mod, case, tiles, [65536 + 8] * len(tiles))


# ---------------------------------------------------------------------------
# C1: [BYTESHUFFLE] on 4-byte values (tdbg_stream_shuffle.hip)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("align", [1, 16])
@pytest.mark.parametrize("ntiles", [7, 256, 700])
def test_shuffle4_config_tiles(eng, ctx, oracle_mod, ntiles, align):
    """SURVEY's C1 tiles (ramp and rand), back to back or 16-B aligned: every
    one taken by the unit-parallel kernel; a batch of fewer tiles than CUs runs
    chunk-parallel (the device chunk directory), as any pipeline's does."""
    from tests.test_gpu_parity import check_parity, encode
    from tests.cases import c1_tiles
    from tiledb_amd.filter_pipeline import ByteshuffleFilter
    tiles = c1_tiles(4, "ramp") + c1_tiles(4, "rand")
    case = Case("c1", P(ByteshuffleFilter()), Datatype.INT32, 4, tiles)
    _, enc = encode(oracle_mod, case)
    enc = (enc * -(-ntiles // len(enc)))[:ntiles]
    f0, b0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    check_parity(eng, ctx, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc], [e[1] for e in enc],
                 align=align)
    f1, b1, _ = ctx.path_stats()
    assert b1 - b0 == 0 and f1 - f0 == ntiles
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert ctx.stream_tiles() - s0 == (ntiles if ntiles >= cus else 0)


def test_shuffle4_few_multichunk_tiles_chunk_parallel(eng, ctx, oracle_mod):
    """A few multi-chunk [BYTESHUFFLE] int32 tiles (1 MiB = 16 chunks each,
    fewer tiles than CUs): the launch runs chunk-parallel, not on the
    unit-parallel kernel (which takes only one-chunk tiles), so every chunk is
    its own work item; bit-exact vs the oracle."""
    from tests.test_gpu_parity import check_parity, encode
    from tiledb_amd.filter_pipeline import ByteshuffleFilter
    rng = np.random.default_rng(64)
    tiles = [as_u8(rng.integers(-2**31, 2**31, 262144 - 7 * k, dtype=np.int64).astype(np.int32)) for k in range(4)]
    case = Case("c1_multichunk", P(ByteshuffleFilter()), Datatype.INT32, 4, tiles)
    _, enc = encode(oracle_mod, case)
    assert all(int(np.frombuffer(e[0][:8].tobytes(), dtype=np.uint64)[0]) == 16 for e in enc)
    f0, b0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    check_parity(eng, ctx, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc], [e[1] for e in enc])
    f1, b1, _ = ctx.path_stats()
    assert b1 - b0 == 0 and f1 - f0 == len(tiles)
    assert ctx.stream_tiles() == s0


def test_shuffle4_declined_tiles(eng, ctx, oracle_mod):
    """Other shapes (other sizes, two parts, UINT32 is taken, INT16 is not),
    corrupted headers, wrong output sizes and offsets tiles get the oracle's
    status and bytes."""
    from tests.test_gpu_parity import check_parity, encode
    from tests.cases import c1_tiles
    from tiledb_amd.filter_pipeline import ByteshuffleFilter
    rng = np.random.default_rng(63)
    pipe = P(ByteshuffleFilter())
    base = c1_tiles(3, "rand")
    odd = [base[0][:4000].copy(), base[1][:65532].copy()]
    case = Case("c1_odd", pipe, Datatype.INT32, 4, base + odd)
    _, enc = encode(oracle_mod, case)
    tiles = [e[0] for e in enc]
    sizes = [e[2] for e in enc]
    for f in list(tiles[:3]):
        for pos in (0, 4, 8, 12, 16, 20, 24, 28, f.size - 1):
            g = f.copy()
            g[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
            tiles.append(g)
            sizes.append(65536)
        tiles.append(f[: f.size - 1].copy())
        sizes.append(65536)
        tiles.append(f.copy())
        sizes.append(65536 + 8)
    rep = -(-320 // len(tiles))
    check_parity(eng, ctx, oracle_mod, Case("c1_mix", pipe, Datatype.INT32, 4, []), tiles * rep, sizes * rep)
    off = Case("c1_offs", pipe, Datatype.INT32, 4, [], offsets_tile=True)
    check_parity(eng, ctx, oracle_mod, off, [e[0] for e in enc] * 64, [e[2] + 8 for e in enc] * 64)
    i16 = Case("c1_i16", pipe, Datatype.INT16, 2, [t.copy() for t in base])
    s0 = ctx.stream_tiles()
    _run(eng, ctx, oracle_mod, i16)
    assert ctx.stream_tiles() == s0


@pytest.mark.parametrize("cfg", ["c3a", "c3b", "c4"])
def test_small_every_chunk_size(eng, ctx, oracle_mod, cfg):
    """C3a / C3b / C4 tiles of one chunk under 64 KiB (16 .. 8,190 u64
    values: the last unit of two values half used, BWR / PD last windows
    partial), mixed back to back: bit-exact, no fallback, and the streaming
    kernel takes at least every tile of >= 1 KiB (tiles too small for its
    256-B windows may go to the fused kernel)."""
    rng = np.random.default_rng(71)
    gen = W.c4_values if cfg == "c4" else W.c3_values
    sizes = [128, 1024, 4000, 8192, 16000, 40000, 64000, 65520]
    vals = [gen(k, rng)[: nb // 8] for k, nb in enumerate(sizes)]
    ser, dt, cs, _, _ = W.config(cfg)
    pipe = {"c3a": P(DD()), "c3b": P(RLE()), "c4": _pd_bwr()}[cfg]
    case = Case(f"{cfg}_sizes", pipe, dt, cs, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0
    want_min = sum(e[2] >= 1024 for e in enc)
    assert want_min <= st <= len(enc), (st, want_min, len(enc))


def test_shuffle4_every_tile_size(eng, ctx, oracle_mod):
    """One-chunk [BYTESHUFFLE] int32 / uint32 tiles of every size class up to
    64 KiB (n = 4 .. 16,384 values, n mod 4 = 0..3: planes at every byte
    alignment, a partial last unit), mixed back to back (outputs 4-B
    aligned): every tile taken by the unit-parallel kernel, bit-exact."""
    from tests.test_gpu_parity import check_parity_replicated, encode
    from tiledb_amd.filter_pipeline import ByteshuffleFilter
    rng = np.random.default_rng(65)
    sizes = [16, 20, 24, 28, 1000, 4004, 4008, 4012, 40000, 40004, 65520, 65524, 65528, 65532, 65536]
    for dt, npt in ((Datatype.INT32, np.int32), (Datatype.UINT32, np.uint32)):
        tiles = [as_u8(rng.integers(-2**31, 2**31, nb // 4, dtype=np.int64).astype(npt)) for nb in sizes]
        case = Case("c1_sizes", P(ByteshuffleFilter()), dt, 4, tiles)
        _, enc = encode(oracle_mod, case)
        assert len(enc) == len(sizes)
        f0, b0, _ = ctx.path_stats()
        s0 = ctx.stream_tiles()
        check_parity_replicated(eng, ctx, oracle_mod, case, enc, 330)
        f1, b1, _ = ctx.path_stats()
        assert b1 - b0 == 0 and f1 - f0 == 330
        assert ctx.stream_tiles() - s0 == 330


@pytest.mark.parametrize("cfg", ["c3a", "c3b", "c4"])
def test_small_chunk_stream_multichunk(eng, ctx, oracle_mod, cfg):
    """Multi-chunk C3a / C3b / C4 tiles (16 chunks of 8,192 u64 values, the
    last one short) in a chunk-parallel launch: the small-image streaming
    kernel takes every chunk -- the short last ones included -- of each tile
    whose output starts 16-B aligned from the device chunk directory, the
    fused kernel the other tiles' chunks; bit-exact vs the oracle."""
    from tests.test_gpu_parity import check_parity, encode
    rng = np.random.default_rng(77)
    gen = W.c4_values if cfg == "c4" else W.c3_values
    vals = [np.concatenate([gen(16 * k + c, rng) for c in range(16)])[: 131072 - 5 * k - 1] for k in range(4)]
    ser, dt, cs, _, _ = W.config(cfg)
    pipe = {"c3a": P(DD()), "c3b": P(RLE()), "c4": _pd_bwr()}[cfg]
    case = Case(f"{cfg}_multichunk", pipe, dt, cs, [as_u8(v) for v in vals])
    _, enc = encode(oracle_mod, case)
    assert len(enc) == 4 and all(int(np.frombuffer(e[0][:8].tobytes(), dtype=np.uint64)[0]) == 16 for e in enc)
    n = 24
    f0, b0, _ = ctx.path_stats()
    c0 = ctx.stream_chunks()
    check_parity(eng, ctx, oracle_mod, case, [enc[i % 4][0] for i in range(n)], [enc[i % 4][2] for i in range(n)])
    f1, b1, _ = ctx.path_stats()
    assert b1 - b0 == 0 and f1 - f0 == n
    # every chunk of a tile whose output starts 16-B aligned (outputs packed
    # back to back, TileBatch.from_packed; the small kernel's store rule),
    # the rest by the fused kernel
    osz = np.array([enc[i % 4][2] for i in range(n)], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(osz)[:-1]])
    aligned = int((off % 16 == 0).sum())
    assert 0 < aligned < n
    assert ctx.stream_chunks() - c0 == 16 * aligned
