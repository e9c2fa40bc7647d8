"""GPU parity of the C5 tile kernel (tiledb_amd/csrc/tdbg_c5tile.hip,
unfilter_c5tile_kernel: one workgroup per tile) for the headline pipeline
[BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION(256)] on INT32 / UINT32,
DoubleDelta bit-packed (the coded path) and stored raw (the raw path),
through the C-ABI.  (These tests exercised round 4's streaming kernels,
tdbg_stream.hip / tdbg_stream_raw.hip, before the tile kernel replaced them;
those now live in the experiments library only.)

Bit-exact against the oracle, with the tile kernel proven to have taken the
tiles it is built for (tdbg_context_stream_stats: coded + raw tiles;
tdbg_context_stream_raw_stats: raw tiles), every DD code width cb = 2..31 and
every raw-path window decoder (all-raw, all-8-bit, mixed/16-bit) exercised;
tiles they decline (odd shapes, corrupted) must come out exactly as the
oracle says through the fused kernel and the general interpreter behind it.
"""
from __future__ import annotations

import numpy as np
import pytest

import workloads as W
from tests.cases import Case, DD, P, as_u8
from tiledb_amd.filter_pipeline import BitWidthReductionFilter, ByteshuffleFilter, Datatype

pytestmark = pytest.mark.gpu

CCAP = 22016  # (round 4's coded-kernel image cap: tiles on both sides of it are tested)


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from tiledb_amd import engine
    return engine


@pytest.fixture(scope="module")
def ctx(eng):
    return eng.Context(0)


def unshuffle(s: np.ndarray) -> np.ndarray:
    """int32 values whose 4-byte byteshuffle is the int32 stream s."""
    n = s.size
    return s.astype("<i4").view(np.uint8).reshape(4, n).T.reshape(-1).view("<i4").copy()


def step_values(bits: int, rng, n: int = 16384) -> np.ndarray:
    """Values whose byteshuffled stream is a step function with jumps below
    2^bits: DoubleDelta codes are mostly zero (BWR windows 8-bit) and its
    bitsize is about `bits`."""
    s = np.empty(n, dtype=np.int64)
    i = 0
    hi = 1 << bits
    k = 0
    while i < n:
        run = int(rng.integers(2048, 8192))
        # the first jump is 2^bits - 1: the bitsize is exactly `bits`
        s[i:i + run] = 0 if k == 0 else hi - 1 if k == 1 else rng.integers(0, hi)
        i += run
        k += 1
    return unshuffle(s.astype(np.int32))


def _pipe():
    return P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256))


MIN_TILES = 320  # launches below one tile per CU go chunk-parallel (no streaming kernel)


def _run(eng, ctx, O, case, align=1):
    from tests.test_gpu_parity import check_parity, encode
    _, enc = encode(O, case)
    assert len(enc) == len(case.tiles)
    enc = enc * -(-MIN_TILES // len(enc))
    f0, b0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    check_parity(eng, ctx, O, case, [e[0] for e in enc], [e[2] for e in enc], [e[1] for e in enc],
                 align=align)
    f1, b1, _ = ctx.path_stats()
    s1 = ctx.stream_tiles()
    return enc, f1 - f0, b1 - b0, s1 - s0


def _eligible(f: np.ndarray, vals: np.ndarray) -> bool:
    """Taken by the coded-DD kernel: the image fits its staging, DD bit-packed."""
    return f.size + 15 <= CCAP and W.c5_dd_bitsize(vals) < 31


def _raw_eligible(f: np.ndarray, vals: np.ndarray) -> bool:
    """Taken by the raw-DD kernel: bigger than the coded kernel's cap, DD raw
    (BWR(256) windows: a power of two, <= 320 windows)."""
    return f.size > CCAP and W.c5_dd_bitsize(vals) >= 31


def raw_window_values(kinds, rng) -> np.ndarray:
    """int32 tile values whose C5 encoding stores DoubleDelta raw and whose
    256-B BWR windows over DD's output have (mostly) the given kinds: DD's
    output bytes [26, 65562) are the byteshuffled values, so designing the
    BWR elements (bytes [4e, 4e + 4) of that output) designs the values.
    kinds cycle over windows: 8 (range < 127), 16 (range < 32767), 32 (random)."""
    nel = 65562 // 4 + 1
    v = np.empty(nel, dtype=np.int64)
    for wi in range(nel // 64 + 1):
        a, b = 64 * wi, min(64 * wi + 64, nel)
        if a >= b:
            break
        k = kinds[wi % len(kinds)]
        base = int(rng.integers(-2**30, 2**30))
        if k == 8:
            v[a:b] = base + rng.integers(0, 100, b - a)
        elif k == 16:
            v[a:b] = base + rng.integers(0, 30000, b - a)
        else:
            v[a:b] = rng.integers(-2**31, 2**31, b - a)
    out = v.astype(np.int64).astype("<i8").astype(np.int32).view(np.uint8)
    s = out[26:26 + 65536].view("<i4")
    return unshuffle(s)


@pytest.mark.parametrize("align", [1, 16])
def test_c5tile_coded_active_tiles(eng, ctx, oracle_mod, align):
    """C5 'active' tiles: every one taken by the streaming kernel."""
    pool, vals = W.c5_pool("active", 24, seed=21)
    case = Case("c5_active", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case, align)
    assert fb == 0 and fused == len(enc)
    assert st == len(enc), f"streaming kernel took {st} of {len(enc)} tiles"


def test_c5tile_coded_every_code_width(eng, ctx, oracle_mod):
    """DD bitsize 1..30 (code widths 2..31, every instantiation), two tiles each."""
    rng = np.random.default_rng(22)
    vals = [step_values(b, rng) for b in range(1, 31) for _ in range(2)]
    bs = sorted({W.c5_dd_bitsize(v) for v in vals})
    assert bs[0] <= 1 and bs[-1] >= 30, bs
    case = Case("c5_steps", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    want = sum(_eligible(e[0], v) for e, v in zip(enc, vals * (len(enc) // len(vals))))
    assert want >= len(enc) - 4 * (len(enc) // len(vals))
    assert fb == 0 and fused == len(enc)
    assert st == want, f"streaming kernel took {st}, expected {want}"


def slope_values(rng, n: int = 16384) -> np.ndarray:
    """Values whose byteshuffled stream is piecewise linear with nonzero
    slopes: DD codes are zero along each segment (whole waves of them, which
    the kernel's all-zero-codes path skips) while the running delta they
    carry is not -- the skipped waves' values come from the fold alone."""
    d = np.empty(n, dtype=np.int64)
    i = 0
    while i < n:
        run = int(rng.integers(1500, 6000))
        d[i:i + run] = int(rng.integers(-4000, 4000))
        i += run
    d[int(rng.integers(1, n))] = int(rng.integers(-50, 50))  # one isolated kink
    s = np.cumsum(d) + int(rng.integers(-2**20, 2**20))
    return unshuffle(s.astype(np.int32))


def test_c5tile_coded_zero_code_waves(eng, ctx, oracle_mod):
    """Whole waves of zero DD codes inside nonzero-slope segments, UINT32 and
    INT32, next to step tiles: bit-exact, every tile taken by the kernel."""
    rng = np.random.default_rng(27)
    vals = [slope_values(rng) for _ in range(12)]
    assert all(W.c5_dd_bitsize(v) < 31 for v in vals)
    case = Case("c5_slopes", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and fused == len(enc)
    assert st == len(enc), f"streaming kernel took {st} of {len(enc)} tiles"
    case = Case("c5_slopes_u32", _pipe(), Datatype.UINT32, 4, [as_u8(v.view(np.uint32)) for v in vals[:4]])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and st == len(enc)


def test_c5tile_coded_dense_codes(eng, ctx, oracle_mod):
    """The bench's 'walk' tiles (c5_dense_codes leg): nonzero DD codes in
    every wave, BWR windows raw; every tile taken, bit-exact."""
    pool, vals = W.c5_pool("walk", 16, seed=28)
    assert all(W.c5_dd_bitsize(v) < 31 for v in vals)
    case = Case("c5_walk", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and fused == len(enc)
    assert st == len(enc), f"streaming kernel took {st} of {len(enc)} tiles"


def test_c5tile_coded_uint32(eng, ctx, oracle_mod):
    """UINT32 (BWR zero-extends its 8/16-bit windows: spec 20)."""
    rng = np.random.default_rng(23)
    vals = [step_values(b, rng).view(np.uint32) for b in (3, 9, 17, 28)]
    vals += [v.view(np.uint32) for v in W.c5_pool("active", 4, seed=24)[1]]
    case = Case("c5_u32", _pipe(), Datatype.UINT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and fused == len(enc)
    assert st >= len(enc) - 2 * (len(enc) // len(vals))


def test_c5tile_coded_mixed_and_declined(eng, ctx, oracle_mod):
    """Active, ramp (DD raw), rand (DD and BWR raw) and step tiles interleaved
    back to back: each streaming kernel takes exactly its eligible tiles, the
    fused kernel the rest, all bit-exact."""
    rng = np.random.default_rng(25)
    act = W.c5_pool("active", 6, seed=26)[1]
    vals = []
    for k in range(6):
        vals += [act[k], W.c5_values("ramp", k, rng), step_values(int(rng.integers(1, 31)), rng),
                 W.c5_values("rand", k, rng)]
    case = Case("c5_mixed", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    r0 = ctx.stream_raw_tiles()
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    rep = vals * (len(enc) // len(vals))
    want = sum(_eligible(e[0], v) for e, v in zip(enc, rep))
    want_raw = sum(_raw_eligible(e[0], v) for e, v in zip(enc, rep))
    assert want_raw >= len(enc) // 2
    assert fb == 0 and fused == len(enc)
    assert ctx.stream_raw_tiles() - r0 == want_raw
    assert st == want + want_raw


def _run_raw(eng, ctx, O, case, align=1):
    r0 = ctx.stream_raw_tiles()
    enc, fused, fb, st = _run(eng, ctx, O, case, align)
    return enc, fused, fb, st, ctx.stream_raw_tiles() - r0


@pytest.mark.parametrize("variant", ["rand", "ramp"])
@pytest.mark.parametrize("align", [1, 16])
def test_c5tile_raw_tiles(eng, ctx, oracle_mod, variant, align):
    """SURVEY's C5 'rand' (DD and BWR raw) and 'ramp' (DD raw, raw and 8-bit
    windows) tiles: every one taken by the raw-DD streaming kernel."""
    pool, vals = W.c5_pool(variant, 16, seed=31)
    assert all(W.c5_dd_bitsize(v) >= 31 for v in vals)
    case = Case(f"c5_{variant}", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st, raw = _run_raw(eng, ctx, oracle_mod, case, align)
    assert fb == 0 and fused == len(enc)
    assert raw == len(enc) and st == len(enc), f"raw kernel took {raw} of {len(enc)}"


@pytest.mark.parametrize("kinds", [(8, 8, 8, 32), (16, 32), (8, 16, 32), (32, 8), (16, 16, 16, 8, 32)],
                         ids=lambda k: "w" + "_".join(map(str, k)))
def test_c5tile_raw_window_decoders(eng, ctx, oracle_mod, kinds):
    """Raw-DD tiles whose BWR windows are 8-bit, 16-bit and raw in runs:
    job planes over all-raw, all-8-bit and mixed / 16-bit windows (the raw
    kernel's three decoders), including window-boundary minimum changes."""
    rng = np.random.default_rng(sum(kinds) + 7 * len(kinds))
    vals = [raw_window_values(kinds, rng) for _ in range(8)]
    assert all(W.c5_dd_bitsize(v) >= 31 for v in vals)
    case = Case("c5_rawwin", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st, raw = _run_raw(eng, ctx, oracle_mod, case)
    want = sum(_raw_eligible(e[0], v) for e, v in zip(enc, vals * (len(enc) // len(vals))))
    assert want == len(enc)
    assert fb == 0 and fused == len(enc) and raw == want


def test_c5tile_raw_uint32(eng, ctx, oracle_mod):
    """UINT32: the raw kernel zero-extends 8/16-bit windows."""
    rng = np.random.default_rng(33)
    vals = [raw_window_values((8, 16, 32), rng).view(np.uint32) for _ in range(4)]
    vals += [W.c5_values("ramp", k, rng).view(np.uint32) for k in range(4)]
    case = Case("c5_raw_u32", _pipe(), Datatype.UINT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st, raw = _run_raw(eng, ctx, oracle_mod, case)
    assert fb == 0 and fused == len(enc) and raw == len(enc)


@pytest.mark.parametrize("window", [512, 1024, 4096, 128, 384])
def test_c5tile_raw_window_sizes(eng, ctx, oracle_mod, window):
    """BWR windows of 512..4096 B are taken; 128 B (513 windows > 320) and a
    window that is not a power of two (384) are declined to the fused kernel."""
    rng = np.random.default_rng(window)
    vals = [W.c5_values("rand", k, rng) for k in range(4)] + [W.c5_values("ramp", k, rng) for k in range(4)]
    case = Case(f"c5_raw_w{window}", P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(window)),
                Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st, raw = _run_raw(eng, ctx, oracle_mod, case)
    taken = window in (512, 1024, 4096)
    if taken:
        assert fb == 0 and fused == len(enc)
    assert raw == (len(enc) if taken else 0)  # (declined ones: parity checked, any path)


def test_c5tile_raw_corrupted_tiles(eng, ctx, oracle_mod):
    """Corruptions of raw-DD tiles (tile and chunk headers, BWR metadata,
    compression frame, both DD headers, data, truncation) get the oracle's
    status and bytes; intact tiles beside them are taken by the raw kernel."""
    from tests.test_gpu_parity import check_parity
    rng = np.random.default_rng(35)
    pool = W.c5_pool("ramp", 2, seed=36)[0] + W.c5_pool("rand", 2, seed=37)[0]
    tiles = []
    for f in pool:
        f = np.frombuffer(f, dtype=np.uint8)
        tiles.append(f.copy())
        ml = int(f[16:20].view("<u4")[0])
        nwin = int(f[24:28].view("<u4")[0])
        data0 = 20 + ml
        for pos in (0, 8, 12, 16, 20, 24, 28, 32, 33, 37, 28 + 9 * (nwin - 1) + 5, 20 + ml - 24, 20 + ml - 12,
                    20 + ml - 4, data0, data0 + 1, data0 + 9, data0 + 13, data0 + 17, data0 + 18, data0 + 24,
                    data0 + 300, f.size - 3):
            g = f.copy()
            g[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
            tiles.append(g)
        tiles.append(f[: f.size - 1].copy())
        tiles.append(f[: f.size // 2].copy())
    case = Case("c5_raw_corrupt", _pipe(), Datatype.INT32, 4, [])
    tiles = tiles * -(-MIN_TILES // len(tiles))
    r0 = ctx.stream_raw_tiles()
    check_parity(eng, ctx, oracle_mod, case, tiles, [W.TILE_BYTES] * len(tiles))
    assert ctx.stream_raw_tiles() > r0


def test_c5tile_raw_wrong_sizes_and_offsets(eng, ctx, oracle_mod):
    """Raw-DD tiles with a wrong output size, and as offsets tiles, are
    declined by the raw kernel and get the oracle's status."""
    from tests.test_gpu_parity import check_parity
    pool = W.c5_pool("rand", 4, seed=38)[0]
    tiles = [np.frombuffer(f, dtype=np.uint8) for f in pool]
    tiles = tiles * -(-MIN_TILES // len(tiles))
    case = Case("c5_raw_sizes", _pipe(), Datatype.INT32, 4, [])
    sizes = [W.TILE_BYTES + (8 if i % 3 == 1 else -4 if i % 3 == 2 else 0) for i in range(len(tiles))]
    check_parity(eng, ctx, oracle_mod, case, tiles, sizes)


def test_c5tile_coded_corrupted_tiles(eng, ctx, oracle_mod):
    """Corruptions of active tiles (headers, metadata, DD header, truncation)
    get the oracle's status; untouched tiles beside them stay exact."""
    from tests.test_gpu_parity import check_parity
    pool, vals = W.c5_pool("active", 4, seed=27)
    rng = np.random.default_rng(28)
    tiles = []
    for f in pool:
        f = np.frombuffer(f, dtype=np.uint8)
        tiles.append(f.copy())
        ml = int(f[16:20].view("<u4")[0])
        data0 = 20 + ml
        for pos in (0, 8, 12, 16, 20, 24, 28, 33, 20 + ml - 24, 20 + ml - 4, data0, data0 + 17, data0 + 18,
                    data0 + 26, data0 + 300, f.size - 3):
            g = f.copy()
            g[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
            tiles.append(g)
        tiles.append(f[: f.size - 1].copy())
        tiles.append(f[: f.size // 2].copy())
    case = Case("c5_corrupt", _pipe(), Datatype.INT32, 4, [])
    tiles = tiles * -(-MIN_TILES // len(tiles))
    s0 = ctx.stream_tiles()
    check_parity(eng, ctx, oracle_mod, case, tiles, [W.TILE_BYTES] * len(tiles))
    assert ctx.stream_tiles() > s0  # the intact tiles (and harmless flips) streamed
