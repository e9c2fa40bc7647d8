"""GPU parity of the C2 / C2i tile kernel (tdbg_c2tile.hip): [BITSHUFFLE]
(+ BIT_WIDTH_REDUCTION on FLOAT32, a pass-through, bit_width_reduction_filter
.cc:166-176) and [BITSHUFFLE, BIT_WIDTH_REDUCTION(w)] on INT32 / UINT32, one
64 KiB chunk per tile (bitshuffle_filter.cc:128-212, bit_width_reduction_
filter.cc:288-380).

Bit-exact against the oracle (statuses and bytes), with the kernel's counters
proving which tiles it took: every one-chunk 64 KiB tile whose BWR windows are
a power of two in [256, 4096] B; other sizes and multi-chunk tiles are left to
the fused kernel in the same launch.  The BWR windows see the bitshuffled
stream, so the windows' kinds (8-bit, 16-bit, raw; negative minima) are set
by crafting that stream S and taking the values whose bitshuffle is S.
"""
from __future__ import annotations

import numpy as np
import pytest

import workloads as W
from tests.cases import Case, P, as_u8
from tiledb_amd.filter_pipeline import BitshuffleFilter, BitWidthReductionFilter, Datatype

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


def unbitshuffle4(s: bytes) -> np.ndarray:
    """The 4-byte elements whose bitshuffle (whole 8,192-B blocks) is s."""
    b = np.frombuffer(s, dtype=np.uint8).reshape(-1, 32, 256)
    bits = np.unpackbits(b, axis=2, bitorder="little")            # (blk, 32 rows, 2048 elems)
    x = np.packbits(bits.transpose(0, 2, 1), axis=2, bitorder="little")  # (blk, 2048, 4)
    return x.reshape(-1).view("<i4").copy()


def crafted(kinds: str, rng, nbytes: int = 65536, window: int = 256) -> np.ndarray:
    """Values whose bitshuffled stream has, window by window (cycling over
    `kinds`): '8' dwords in a 127 range, 'h' a 32,767 range, 'r' full range,
    'n' an 8-bit range at a negative base, 'z' zeros, 'm' -1."""
    nw = nbytes // window
    per = window // 4
    out = []
    for i in range(nw):
        k = kinds[i % len(kinds)]
        if k == "8":
            v = int(rng.integers(-2**31, 2**31 - 300)) + rng.integers(0, 128, per)
        elif k == "h":
            v = int(rng.integers(-2**31, 2**31 - 70000)) + rng.integers(0, 32768, per)
        elif k == "r":
            v = rng.integers(-2**31, 2**31, per)
        elif k == "n":
            v = -1000 + rng.integers(0, 100, per)
        elif k == "z":
            v = np.zeros(per, dtype=np.int64)
        else:
            v = -np.ones(per, dtype=np.int64)
        out.append(np.asarray(v, dtype=np.int64).astype(np.int32))
    s = np.concatenate(out).astype("<i4").tobytes()
    v = unbitshuffle4(s)
    assert W.bitshuffle_fwd(v.tobytes(), 4)[1] == s
    return v


def c2_taken(f: np.ndarray, bwr: bool) -> bool:
    """The C2 tile kernel decodes this tile: one chunk of 256..65,536 bytes
    (a multiple of 4) and, with BWR, window 0 a power of two in [256, 4096]."""
    nch = int(np.frombuffer(f[:8].tobytes(), dtype="<u8")[0])
    orig = int(np.frombuffer(f[8:12].tobytes(), dtype="<u4")[0])
    if nch != 1 or orig < 256 or orig > 65536 or orig % 4:
        return False
    if not bwr:
        return True
    ws = int(np.frombuffer(f[20 + 13:20 + 17].tobytes(), dtype="<u4")[0])
    return 256 <= ws <= 4096 and ws & (ws - 1) == 0


def _tile_mode(eng, ctx, O, case, align=1, bwr=None):
    """Tile-mode launch of >= MIN_TILES tiles cycling over the case's tiles:
    bit-exact vs the oracle; returns (n, fused, fallback, taken by the kernel,
    tiles it should take)."""
    from tests.test_gpu_parity import check_parity_replicated, encode
    _, enc = encode(O, case)
    assert len(enc) == len(case.tiles)
    n = max(MIN_TILES, len(enc))
    f0, b0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    st = check_parity_replicated(eng, ctx, O, case, enc, n, align=align)
    assert not st.any()
    f1, b1, _ = ctx.path_stats()
    if bwr is None:
        bwr = len(case.pipeline.filters) == 2 and int(case.dtype) != int(Datatype.FLOAT32)
    want = sum(c2_taken(enc[i % len(enc)][0], bwr) for i in range(n))
    return n, f1 - f0, b1 - b0, ctx.stream_tiles() - s0, want


@pytest.mark.parametrize("align", [1, 16])
@pytest.mark.parametrize("dtype", [Datatype.FLOAT32, Datatype.INT32])
@pytest.mark.parametrize("bwr", [False, True])
def test_c2_tiles(eng, ctx, oracle_mod, dtype, bwr, align):
    """BASELINE C2 (FLOAT32) and C2i (INT32) tiles, with and without the BWR
    stage: every tile taken, bit-exact, at every input alignment class."""
    rng = np.random.default_rng(11 + int(dtype) + 2 * bwr)
    vals = [W.c2_values(k, rng) for k in range(6)]
    if dtype == Datatype.INT32:
        vals = [v.view(np.int32) for v in vals]
    pipe = P(BitshuffleFilter(), BitWidthReductionFilter(256)) if bwr else P(BitshuffleFilter())
    case = Case(f"c2_{int(dtype)}_{bwr}", pipe, dtype, 4, [as_u8(v) for v in vals])
    n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case, align)
    assert want == n and fb == 0 and fused == n
    assert st == n, f"C2 tile kernel took {st} of {n}"


@pytest.mark.parametrize("window", [256, 1024, 4096])
@pytest.mark.parametrize("dtype", [Datatype.INT32, Datatype.UINT32])
def test_c2i_window_kinds(eng, ctx, oracle_mod, dtype, window):
    """C2i with 8-bit, 16-bit and raw BWR windows (negative minima, zeros, -1)
    in every order, windows of 256 / 1024 / 4096 B, signed and unsigned."""
    rng = np.random.default_rng(31 + window + int(dtype))
    kinds = ["8", "h", "r", "n", "z", "m", "8h", "hr8", "r8n", "zmh8r"]
    vals = [crafted(k, rng, window=window) for k in kinds]
    if dtype == Datatype.UINT32:
        vals = [v.view(np.uint32) for v in vals]
    case = Case(f"c2i_{window}_{int(dtype)}", P(BitshuffleFilter(), BitWidthReductionFilter(window)), dtype, 4,
                [as_u8(v) for v in vals])
    n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case)
    assert want == n and fb == 0
    assert st == n, f"C2i tile kernel took {st} of {n}"


@pytest.mark.parametrize("bwr", [False, True])
def test_c2_declined_shapes(eng, ctx, oracle_mod, bwr):
    """Tiles the kernel leaves to the fused kernel in the same launch (8 B;
    two chunks: 128 KiB) mixed with ones it takes (64 KiB, 40,000 B, 65,532 B;
    outputs back to back: at every 4-B alignment): bit-exact, and it took
    exactly the one-chunk tiles of 256 B or more (the fused kernel passes one
    of the odd shapes on to the general interpreter)."""
    rng = np.random.default_rng(41 + bwr)
    vals = [crafted("8hr", rng), rng.integers(-2**31, 2**31, 10000).astype(np.int32),
            crafted("r", rng), rng.integers(-5, 5, 16383).astype(np.int32),
            np.concatenate([crafted("hz", rng), crafted("n8", rng)]), np.array([7, -7], dtype=np.int32)]
    pipe = P(BitshuffleFilter(), BitWidthReductionFilter(256)) if bwr else P(BitshuffleFilter())
    case = Case(f"c2_declined_{bwr}", pipe, Datatype.INT32, 4, [as_u8(v) for v in vals])
    n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case)
    assert 0 < want < n and fb <= n // 6 + 1
    assert st == want, f"C2 tile kernel took {st}, expected {want}"


# every size class of a one-chunk tile: whole 8,192-B blocks or a partial last
# block (rows of R < 256 bytes, R % 4 = 0 or 2), os % 8 = 4 (a second,
# copied bitshuffle part), short tiles down to 256 B
_SIZES = [256, 260, 1000, 1004, 4100, 8192, 8196, 12288, 12292, 40000, 40004, 40960, 65528, 65532, 65536]


@pytest.mark.parametrize("dtype,window", [(Datatype.FLOAT32, 0), (Datatype.INT32, 0), (Datatype.INT32, 256),
                                          (Datatype.UINT32, 1024)])
def test_c2_every_size_class(eng, ctx, oracle_mod, dtype, window):
    """One launch of tiles of every size class back to back (outputs at every
    4-B alignment), [BITSHUFFLE] or [BITSHUFFLE, BWR(window)]: bit-exact, and
    the kernel takes exactly the tiles it decodes (BWR: window 0 a power of
    two >= 256 B, so a tile under the window size is left unless it is one)."""
    rng = np.random.default_rng(77 + window + int(dtype))
    vals = []
    for k, nb in enumerate(_SIZES):
        v = crafted("8hrnzm"[k % 6] + "8r", rng)[: nb // 4] if window else rng.normal(0, 1e3, nb // 4).astype(np.float32)
        vals.append(v.view(np.uint32) if dtype == Datatype.UINT32 else v.view(np.int32) if dtype == Datatype.INT32 else v)
    pipe = P(BitshuffleFilter(), BitWidthReductionFilter(window)) if window else P(BitshuffleFilter())
    case = Case(f"c2_sizes_{int(dtype)}_{window}", pipe, dtype, 4, [as_u8(v) for v in vals])
    n, fused, fb, st, want = _tile_mode(eng, ctx, oracle_mod, case, bwr=bool(window))
    assert want >= n // 2, want
    assert fb <= n - want  # (the fused kernel may pass a declined odd shape on to the general interpreter)
    assert st == want, f"C2 tile kernel took {st}, expected {want}"


@pytest.mark.parametrize("bwr", [False, True])
def test_c2_malformed_tiles(eng, ctx, oracle_mod, bwr):
    """Valid 64 KiB tiles with one header or metadata field corrupted (chunk
    count, orig, bitshuffle part count / size, BWR window bytes / bits, a
    truncated image): the tile kernel declines each, and the statuses and
    bytes of the whole launch equal the oracle's."""
    import struct
    from tests.test_gpu_parity import check_parity_replicated
    rng = np.random.default_rng(91 + bwr)
    pipe = P(BitshuffleFilter(), BitWidthReductionFilter(256)) if bwr else P(BitshuffleFilter())
    dtype = Datatype.INT32
    op = oracle_mod.OraclePipeline(pipe.serialize(), 23, int(dtype), 4)
    good = [np.frombuffer(op.filter_tile(as_u8(crafted("8hr", rng))), dtype=np.uint8) for _ in range(3)]
    bad = []
    m = 20
    bmd = m + (8 + 9 * 256 if bwr else 0)  # the bitshuffle md (256 BWR windows of 256 B)

    def patch(t, off, fmt, val):
        b = bytearray(t.tobytes())
        struct.pack_into(fmt, b, off, val)
        return np.frombuffer(bytes(b), dtype=np.uint8)

    bad.append(patch(good[0], 0, "<Q", 2))             # chunk count
    bad.append(patch(good[0], 8, "<I", 65532))         # orig
    bad.append(patch(good[1], bmd, "<I", 2))           # bitshuffle parts
    bad.append(patch(good[1], bmd + 4, "<I", 65528))   # bitshuffle part size
    if bwr:
        bad.append(patch(good[2], m + 8 + 5, "<I", 252))   # window 0 bytes
        bad.append(patch(good[2], m + 8 + 9 * 7 + 4, "<B", 12))  # window 7 bits
    bad.append(good[2][: len(good[2]) - 100].copy())   # truncated
    enc = [(t, None, 65536) for t in good + bad]
    case = Case(f"c2_malformed_{bwr}", pipe, dtype, 4, [])
    f0, b0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    st = check_parity_replicated(eng, ctx, oracle_mod, case, enc, MIN_TILES)
    taken = ctx.stream_tiles() - s0
    n_good = sum(1 for i in range(MIN_TILES) if i % len(enc) < len(good))
    assert taken == n_good, f"C2 tile kernel took {taken}, expected {n_good}"
    assert (st != 0).sum() > 0
