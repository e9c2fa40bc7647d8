"""GPU parity of the streaming kernel for the headline pipeline
[BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION(256)] on INT32 / UINT32
(tiledb_amd/csrc/tdbg_stream.hip), through the C-ABI.

Bit-exact against the oracle, with the streaming kernel proven to have taken
the tiles it is built for (tdbg_context_stream_stats) and every DD code
width cb = 2..31 exercised; tiles it declines (too big, DD raw, corrupted)
must come out exactly as the oracle says through the fused kernel and the
general interpreter behind it.
"""
from __future__ import annotations

import numpy as np
import pytest

import workloads as W
from tests.cases import Case, DD, P, as_u8
from tiledb_amd.filter_pipeline import BitWidthReductionFilter, ByteshuffleFilter, Datatype

pytestmark = pytest.mark.gpu

CCAP = 22016  # tdbg_stream.hip: tile image bytes staged in LDS


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
    return f.size + 15 <= CCAP and W.c5_dd_bitsize(vals) < 31


@pytest.mark.parametrize("align", [1, 16])
def test_stream_active_tiles(eng, ctx, oracle_mod, align):
    """C5 'active' tiles: every one taken by the streaming kernel."""
    pool, vals = W.c5_pool("active", 24, seed=21)
    case = Case("c5_active", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case, align)
    assert fb == 0 and fused == len(enc)
    assert st == len(enc), f"streaming kernel took {st} of {len(enc)} tiles"


def test_stream_every_code_width(eng, ctx, oracle_mod):
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


def test_stream_uint32(eng, ctx, oracle_mod):
    """UINT32 (BWR zero-extends its 8/16-bit windows: spec 20)."""
    rng = np.random.default_rng(23)
    vals = [step_values(b, rng).view(np.uint32) for b in (3, 9, 17, 28)]
    vals += [v.view(np.uint32) for v in W.c5_pool("active", 4, seed=24)[1]]
    case = Case("c5_u32", _pipe(), Datatype.UINT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    assert fb == 0 and fused == len(enc)
    assert st >= len(enc) - 2 * (len(enc) // len(vals))


def test_stream_mixed_and_declined(eng, ctx, oracle_mod):
    """Active, ramp (DD raw), rand (too big) and step tiles interleaved back to
    back: the streaming kernel takes exactly the eligible ones, the fused
    kernel the rest, all bit-exact."""
    rng = np.random.default_rng(25)
    act = W.c5_pool("active", 6, seed=26)[1]
    vals = []
    for k in range(6):
        vals += [act[k], W.c5_values("ramp", k, rng), step_values(int(rng.integers(1, 31)), rng),
                 W.c5_values("rand", k, rng)]
    case = Case("c5_mixed", _pipe(), Datatype.INT32, 4, [as_u8(v) for v in vals])
    enc, fused, fb, st = _run(eng, ctx, oracle_mod, case)
    want = sum(_eligible(e[0], v) for e, v in zip(enc, vals * (len(enc) // len(vals))))
    assert fb == 0 and fused == len(enc)
    assert st == want


def test_stream_corrupted_tiles(eng, ctx, oracle_mod):
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
