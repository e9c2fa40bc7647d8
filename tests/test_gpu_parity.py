"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

Bit-exact for every byte and identical status codes, on the BASELINE configs
at test sizes, the SURVEY A.5 edge cases, random pipelines and corrupted
tiles; plus full-size round-trip properties at the BASELINE tile counts.
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


def encode(O, case):
    op = O.OraclePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    enc = []
    for i, t in enumerate(case.tiles):
        offs = case.offsets[i] if case.offsets else None
        try:
            f = op.filter_tile(t, offs, case.max_chunk)
        except O.OracleError:
            continue
        osz = t.size + (8 if case.offsets_tile else 0)
        enc.append((np.frombuffer(f, dtype=np.uint8), t, osz))
    return op, enc


def check_parity(eng, ctx, O, case, filtered, out_sizes, originals=None, fill=0, align=1):
    """Tiles packed back to back by default (align=1): arbitrary tile starts,
    as FilteredData::data_at hands them over (filtered_data.h:100-101)."""
    op = O.OraclePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    assert dp.supported
    batch = eng.TileBatch.from_host(filtered, out_sizes, fill=fill, align=align)
    st = ctx.unfilter(dp, batch, offsets_tiles=case.offsets_tile)
    out = batch.outputs_host()
    for i, f in enumerate(filtered):
        rc, ref = op.unfilter_tile(f, out_sizes[i], case.offsets_tile, fill=fill)
        assert int(st[i]) == rc, f"{case.name} tile {i}: gpu status {st[i]} oracle {rc}"
        if rc == 0:
            o = int(batch.out_off[i])
            got = out[o:o + out_sizes[i]]
            if not np.array_equal(got, ref):
                bad = np.nonzero(got != ref)[0]
                raise AssertionError(f"{case.name} tile {i}: {bad.size} bytes differ, first at "
                                     f"{bad[0]} gpu {got[bad[0]]} oracle {ref[bad[0]]}")
            if originals is not None and originals[i] is not None:
                n = originals[i].size
                if np.array_equal(ref[:n], originals[i]):
                    assert np.array_equal(got[:n], originals[i])
    return st


_CONFIG = config_cases(4)
_EDGE = edge_cases()
_RANDOM = random_cases(120)


_SPECS = fused_spec_cases(3)


@pytest.mark.parametrize("align", [1, 16])
@pytest.mark.parametrize("case", _CONFIG, ids=[c.name for c in _CONFIG])
def test_config_parity(eng, ctx, oracle_mod, case, align):
    """BASELINE configs, back-to-back and 16-B aligned tile starts; every tile
    is taken by the fused kernel (fallback counter unchanged)."""
    _, enc = encode(oracle_mod, case)
    assert enc
    f0, b0, _ = ctx.path_stats()
    check_parity(eng, ctx, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc],
                 [e[1] for e in enc], align=align)
    f1, b1, _ = ctx.path_stats()
    assert b1 - b0 == 0, f"{case.name}: {b1 - b0} tiles fell back to the general path"
    assert f1 - f0 == len(enc)


@pytest.mark.parametrize("align", [1, 16])
@pytest.mark.parametrize("case", _SPECS, ids=[c.name for c in _SPECS])
def test_fused_spec_no_fallback(eng, ctx, oracle_mod, case, align):
    """One case per fused-kernel spec (tdbg_fast.hip SPECS): bit-exact, and
    the fused kernel handled every tile (fallback == 0)."""
    _, enc = encode(oracle_mod, case)
    assert len(enc) == len(case.tiles)
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    f0, b0, _ = ctx.path_stats()
    check_parity(eng, ctx, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc],
                 [e[1] for e in enc], align=align)
    f1, b1, _ = ctx.path_stats()
    assert b1 - b0 == 0, f"{case.name}: {b1 - b0} tiles fell back to the general path"
    assert f1 - f0 == len(enc)
    del dp


def check_parity_replicated(eng, ctx, O, case, enc, n, align=1, chunk_parallel=False):
    """n tiles cycling over the unique encoded tiles `enc` (the oracle runs
    once per unique tile): a launch of more tiles than the GPU has CUs, so it
    takes the tile-serial path (fused kernel: cross-tile prefetch and the
    load hook; or the streaming kernels), not the chunk-parallel one."""
    op = O.OraclePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    refs = [op.unfilter_tile(e[0], e[2], case.offsets_tile) for e in enc]
    idx = np.arange(n) % len(enc)
    batch = eng.TileBatch.from_host([enc[i][0] for i in idx], [enc[i][2] for i in idx], align=align)
    st = ctx.unfilter(dp, batch, offsets_tiles=case.offsets_tile, chunk_parallel=chunk_parallel)
    out = batch.outputs_host()
    for k, i in enumerate(idx):
        rc, ref = refs[i]
        assert int(st[k]) == rc, f"{case.name} tile {k}: gpu status {st[k]} oracle {rc}"
        if rc == 0:
            o = int(batch.out_off[k])
            assert np.array_equal(out[o:o + enc[i][2]], ref), f"{case.name} tile {k} differs from the oracle"
    return st


# the tile-serial launch of the fused kernel (tdbg_fast.hip: one tile per
# workgroup iteration, next tile prefetched, stage hooks) and the streaming
# kernels run only when a launch has at least one tile per CU
_SERIAL_N = 320


@pytest.mark.parametrize("case", _CONFIG + _SPECS, ids=[c.name for c in _CONFIG + _SPECS])
def test_tile_serial_launch_parity(eng, ctx, oracle_mod, case):
    """Every BASELINE config and one case per fused spec at 320 tiles:
    bit-exact vs the oracle, every tile taken by the fused/streaming kernels
    (fallback == 0, fused == 320)."""
    import torch
    assert _SERIAL_N >= torch.cuda.get_device_properties(0).multi_processor_count
    _, enc = encode(oracle_mod, case)
    assert enc
    f0, b0, _ = ctx.path_stats()
    st = check_parity_replicated(eng, ctx, oracle_mod, case, enc, _SERIAL_N)
    assert not st.any()
    f1, b1, _ = ctx.path_stats()
    assert b1 - b0 == 0, f"{case.name}: {b1 - b0} tiles fell back to the general path"
    assert f1 - f0 == _SERIAL_N


@pytest.mark.parametrize("case", _EDGE, ids=[c.name for c in _EDGE])
def test_edge_parity(eng, ctx, oracle_mod, case):
    _, enc = encode(oracle_mod, case)
    if not enc:
        pytest.skip("reference encoder rejects this input")
    check_parity(eng, ctx, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc],
                 [e[1] for e in enc])


def test_random_pipelines_parity(eng, ctx, oracle_mod):
    n = 0
    for case in _RANDOM:
        _, enc = encode(oracle_mod, case)
        if not enc:
            continue
        check_parity(eng, ctx, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc],
                     [e[1] for e in enc])
        n += 1
    assert n > 60


def _mutations(f: np.ndarray, rng):
    """Corruptions of an on-disk tile: truncation, header/metadata byte flips."""
    out = []
    out.append(f[: max(0, f.size - 1)])
    out.append(f[: f.size // 2])
    out.append(f[:7])
    g = f.copy(); g[0] ^= 3; out.append(g)                          # nchunks
    if f.size > 12:
        g = f.copy(); g[8] ^= 1; out.append(g)                      # orig size
        g = f.copy(); g[12] ^= 0x40; out.append(g)                  # filtered size
        g = f.copy(); g[16] ^= 0x10; out.append(g)                  # md size
    for _ in range(6):
        if f.size > 24:
            g = f.copy()
            k = int(rng.integers(20, min(f.size, 120)))
            g[k] ^= np.uint8(1 << int(rng.integers(8)))
            out.append(g)
    return out


@pytest.mark.parametrize("case", _CONFIG + [c for c in _EDGE if c.name.startswith(("dd_", "rle_run_65535",
                                                                                    "bwr_window_437",
                                                                                    "pd_", "bwr_then",
                                                                                    "byte_bit", "xor_", "fscale_",
                                                                                    "delta_"))],
                         ids=lambda c: c.name)
def test_corrupt_tiles_status_parity(eng, ctx, oracle_mod, case):
    rng = np.random.default_rng(7)
    _, enc = encode(oracle_mod, case)
    if not enc:
        pytest.skip("reference encoder rejects this input")
    f, t, osz = enc[0]
    muts = _mutations(f, rng)
    check_parity(eng, ctx, oracle_mod, case, muts, [osz] * len(muts), fill=0x5A)


def test_wrong_output_size(eng, ctx, oracle_mod):
    case = _CONFIG[-2]
    _, enc = encode(oracle_mod, case)
    f, t, osz = enc[0]
    check_parity(eng, ctx, oracle_mod, case, [f, f, f], [osz - 4, osz + 4, 0])


@pytest.mark.parametrize("align", [1, 16])
def test_full_size_c5_roundtrip(eng, ctx, oracle_mod, align):
    """BASELINE C5 per-GPU shard (12,500 tiles x 64 KiB), ramp+rand+active
    mixed, tiles back to back (align=1) or 16-B aligned: size-independent
    property = the unfiltered bytes equal the written tiles; every tile taken
    by the fused kernel."""
    import workloads as W
    from tests.cases import c5_tiles, P, DD
    from tiledb_amd.filter_pipeline import ByteshuffleFilter, BitWidthReductionFilter, Datatype
    case_p = P(ByteshuffleFilter(), DD(), BitWidthReductionFilter(256))
    op = oracle_mod.OraclePipeline(case_p.serialize(), 23, int(Datatype.INT32), 4)
    rng = np.random.default_rng(9)
    uniq = (c5_tiles(40, "ramp") + c5_tiles(16, "rand") +
            [W.c5_values("active", k, rng).view(np.uint8) for k in range(16)])
    enc = [np.frombuffer(op.filter_tile(t), dtype=np.uint8) for t in uniq]
    ntiles = 12500
    idx = np.arange(ntiles) % len(enc)
    tiles = [enc[i] for i in idx]
    dp = eng.DevicePipeline(case_p.serialize(), 23, int(Datatype.INT32), 4)
    batch = eng.TileBatch.from_host(tiles, [65536] * ntiles, align=align)
    f0, b0, _ = ctx.path_stats()
    st = ctx.unfilter(dp, batch)
    f1, b1, _ = ctx.path_stats()
    assert not st.any()
    assert b1 - b0 == 0 and f1 - f0 == ntiles
    out = batch.outputs_host().reshape(ntiles, 65536)
    for k in range(len(enc)):
        rows = out[idx == k]
        assert (rows == uniq[k][None, :]).all()


def test_two_contexts_two_threads(eng, oracle_mod):
    """Two host threads, each with its own context and stream, unfilter
    concurrently through the C-ABI (the reference is re-entrant,
    reader_base.cc:929-934)."""
    import threading
    import torch
    errs = []

    def run(case):
        try:
            c = eng.Context(0)
            s = torch.cuda.Stream()
            _, enc = encode(oracle_mod, case)
            for _ in range(4):
                with torch.cuda.stream(s):
                    check_parity(eng, c, oracle_mod, case, [e[0] for e in enc] * 8, [e[2] for e in enc] * 8)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(c,)) for c in (_CONFIG[0], _CONFIG[-1], _CONFIG[6])]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


def test_one_context_two_streams(eng, oracle_mod):
    """Async launches of one context on two streams: the context serializes
    them (its scratch slots and fallback queue are shared), so both batches
    come out right, including a batch whose tiles all fall back."""
    import torch
    c = eng.Context(0)
    case = _CONFIG[-2]
    _, enc = encode(oracle_mod, case)
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    mc = next(x for x in _EDGE if x.name == "multichunk_c5_small_chunks")
    _, enc2 = encode(oracle_mod, mc)
    dp2 = eng.DevicePipeline(mc.serialized, mc.version, int(mc.dtype), mc.cell_size)
    b1 = eng.TileBatch.from_host([e[0] for e in enc] * 64, [e[2] for e in enc] * 64)
    b2 = eng.TileBatch.from_host([e[0] for e in enc2] * 16, [e[2] for e in enc2] * 16)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        c.unfilter_async(dp, b1, stream=s1.cuda_stream)
        c.unfilter_async(dp2, b2, stream=s2.cuda_stream)
        c.unfilter_async(dp, b1, stream=s2.cuda_stream)
    torch.cuda.synchronize()
    assert not b1.d_status.cpu().numpy().any() and not b2.d_status.cpu().numpy().any()
    o1, o2 = b1.outputs_host(), b2.outputs_host()
    for i in range(b1.ntiles):
        e = enc[i % len(enc)]
        assert np.array_equal(o1[int(b1.out_off[i]):int(b1.out_off[i]) + e[1].size], e[1])
    for i in range(b2.ntiles):
        e = enc2[i % len(enc2)]
        assert np.array_equal(o2[int(b2.out_off[i]):int(b2.out_off[i]) + e[1].size], e[1])


def test_scratch_retry_does_not_inflate_context(eng, oracle_mod):
    """An oversized chunk (1 MiB RLE chunk: TDBG_E_SCRATCH, retried with
    bigger retry-only slots), then a normal BASELINE-size launch on the same
    context: both succeed."""
    c = eng.Context(0)
    big = next(x for x in _EDGE if x.name == "rle_run_70030")
    check_parity(eng, c, oracle_mod, big, *[[e[i] for e in encode(oracle_mod, big)[1]] for i in (0, 2)])
    case = _CONFIG[-1]
    _, enc = encode(oracle_mod, case)
    n = 3000
    check_parity(eng, c, oracle_mod, case, [enc[i % len(enc)][0] for i in range(n)],
                 [enc[i % len(enc)][2] for i in range(n)])


def test_host_end_to_end_and_multi_gpu(eng, ctx, oracle_mod):
    import torch
    case = _CONFIG[-1]
    _, enc = encode(oracle_mod, case)
    filtered = [e[0] for e in enc] * 8
    origs = [e[1] for e in enc] * 8
    osz = [e[2] for e in enc] * 8
    # pinned host buffers, contiguous (FilteredData-style batch)
    sizes = np.array([f.size for f in filtered], dtype=np.uint64)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    hin = torch.empty(int(sizes.sum()), dtype=torch.uint8).pin_memory()
    hin_np = hin.numpy()
    for f, o in zip(filtered, offs):
        hin_np[int(o):int(o) + f.size] = f
    osz_a = np.array(osz, dtype=np.uint64)
    ooff = np.zeros_like(osz_a)
    ooff[1:] = np.cumsum(osz_a)[:-1]
    hout = torch.zeros(int(osz_a.sum()), dtype=torch.uint8).pin_memory()
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    in_ptrs = offs + np.uint64(hin.data_ptr())
    out_ptrs = ooff + np.uint64(hout.data_ptr())
    for contiguous in (True, False):
        hout.zero_()
        st = ctx.unfilter_host(dp, in_ptrs, sizes, out_ptrs, osz_a, batch_bytes=3 * 65536,
                               contiguous_input=contiguous, contiguous_output=contiguous)
        assert not st.any()
        res = hout.numpy()
        for i, o in enumerate(origs):
            assert np.array_equal(res[int(ooff[i]):int(ooff[i]) + o.size], o)
    hout.zero_()
    st = eng.unfilter_multi_gpu(dp, in_ptrs, sizes, out_ptrs, osz_a, [0, 0], batch_bytes=1 << 20,
                                contiguous_input=True, contiguous_output=True)
    assert not st.any()
    res = hout.numpy()
    for i, o in enumerate(origs):
        assert np.array_equal(res[int(ooff[i]):int(ooff[i]) + o.size], o)


def test_host_end_to_end_padded_layouts(eng, ctx, oracle_mod):
    """Host tiles with alignment padding (coalesced H2D incl. padding), a
    large gap and an out-of-order tile (separate copies), and padded outputs
    whose padding bytes must survive the D2H untouched."""
    import torch
    case = _CONFIG[-1]
    _, enc = encode(oracle_mod, case)
    filtered = [e[0] for e in enc] * 6
    origs = [e[1] for e in enc] * 6
    n = len(filtered)
    sizes = np.array([f.size for f in filtered], dtype=np.uint64)
    gaps = np.array([(16 - int(s) % 16) % 16 for s in sizes], dtype=np.uint64)
    gaps[n // 3] = 4096  # too large to copy across
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes + gaps)[:-1]
    # swap two tiles' host positions: tile 5 lies before tile 4
    perm_offs = offs.copy()
    span = int((sizes + gaps).sum())
    perm_offs[5], perm_offs[4] = span, span + int(sizes[5]) + 8
    hin = torch.full((span + 512 + int(sizes.max()) * 2,), 0x5A, dtype=torch.uint8).pin_memory()
    hin_np = hin.numpy()
    for f, o in zip(filtered, perm_offs):
        hin_np[int(o):int(o) + f.size] = f
    osz = np.array([e[2] for e in enc] * 6, dtype=np.uint64)
    ooff = np.zeros_like(osz)
    ooff[1:] = np.cumsum(osz + np.uint64(32))[:-1]
    hout = torch.full((int(ooff[-1] + osz[-1]) + 32,), 0xAB, dtype=torch.uint8).pin_memory()
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    st = ctx.unfilter_host(dp, perm_offs + np.uint64(hin.data_ptr()), sizes,
                           ooff + np.uint64(hout.data_ptr()), osz, batch_bytes=5 * 65536,
                           contiguous_input=True, contiguous_output=True)
    assert not st.any()
    res = hout.numpy()
    mask = np.ones(res.size, dtype=bool)
    for i, o in enumerate(origs):
        assert np.array_equal(res[int(ooff[i]):int(ooff[i]) + o.size], o)
        mask[int(ooff[i]):int(ooff[i]) + int(osz[i])] = False
    assert (res[mask] == 0xAB).all()


@pytest.mark.parametrize("case", _CONFIG, ids=lambda c: c.name)
def test_async_api_and_timing(eng, ctx, oracle_mod, case):
    """Armed launches time their kernels with events bound to the dispatches
    (tdbg_launch.h): per launch, kernel time > 0 and launch time >= it, on the
    streamed (C1, C3-C5), fused-only (C2) and chunk-parallel paths alike."""
    import torch
    _, enc = encode(oracle_mod, case)
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    batch = eng.TileBatch.from_host([e[0] for e in enc], [e[2] for e in enc])
    ctx.time_launches(2)  # events only on armed launches
    ctx.unfilter_async(dp, batch)
    ctx.unfilter_async(dp, batch, chunk_parallel=True)
    torch.cuda.synchronize()
    assert not batch.d_status.cpu().numpy().any()
    assert ctx.last_kernel_ms() > 0
    kern, total = ctx.launch_times()
    assert len(kern) == 2 and (kern > 0).all() and (total >= kern).all(), (kern, total)
    out = batch.outputs_host()
    for i, e in enumerate(enc):
        o = int(batch.out_off[i])
        assert np.array_equal(out[o:o + e[1].size], e[1])
    ctx.unfilter_async(dp, batch)  # unarmed: no events
    torch.cuda.synchronize()
    assert len(ctx.launch_times()[0]) == 0  # reading the times disarmed the context


def test_filter_pipeline_run_reverse_api(eng, oracle_mod):
    """FilterPipeline.run_reverse mirror raises FilterStatusException like the reference."""
    from tiledb_amd.filter_pipeline import FilterStatusException
    case = _CONFIG[4]
    _, enc = encode(oracle_mod, case)
    f, t, osz = enc[0]
    batch = case.pipeline.run_reverse([f], [osz], case.dtype, case.cell_size)
    assert np.array_equal(batch.output(0), t)
    with pytest.raises(FilterStatusException):
        case.pipeline.run_reverse([f[:100]], [osz], case.dtype, case.cell_size)


def _offsets_cases():
    return [c for c in config_cases(2) + edge_cases() if c.offsets_tile]


def test_add_extra_offset_device(eng, ctx, oracle_mod):
    """Tile::add_extra_offset (tile.h:144-146) after a TDBG_TILE_OFFSETS
    unfilter: the tile's values, then its var tile's size in the last u64;
    an errored tile is left alone."""
    rng = np.random.default_rng(7)
    cases = _offsets_cases()
    assert cases
    for case in cases:
        op, enc = encode(oracle_mod, case)
        if not enc:
            continue
        filt = [e[0] for e in enc]
        osz = [e[2] for e in enc]
        # one corrupted copy: its status is an error, its slot keeps the fill
        bad = filt[0].copy()
        bad[:8] = 0xff
        filt2, osz2 = filt + [bad], osz + [osz[0]]
        dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
        batch = eng.TileBatch.from_host(filt2, osz2, fill=0x5a)
        var = rng.integers(0, 2**40, len(filt2)).astype(np.uint64)
        ctx.unfilter_async(dp, batch, offsets_tiles=True)
        ctx.add_extra_offsets(batch, var)
        st = batch.d_status[: batch.ntiles].cpu().numpy()
        for i, f in enumerate(filt2):
            rc, ref = op.unfilter_tile(f, osz2[i], True, fill=0x5a)
            assert int(st[i]) == rc
            got = batch.output(i)
            if rc:
                assert np.all(got[-8:] == 0x5a), "an errored tile's extra slot was written"
                continue
            assert np.array_equal(got[:-8], ref[:-8])
            assert int(got[-8:].view(np.uint64)[0]) == int(var[i])


def test_add_extra_offset_host_fused(eng, ctx, oracle_mod):
    """tdbg_unfilter_offsets_host: the extra offset is written on the device
    before the D2H, so the host result holds the complete offsets tile."""
    rng = np.random.default_rng(8)
    for case in _offsets_cases():
        op, enc = encode(oracle_mod, case)
        if not enc:
            continue
        filt = [e[0] for e in enc] * 3
        osz = np.array([e[2] for e in enc] * 3, dtype=np.uint64)
        var = rng.integers(0, 2**40, len(filt)).astype(np.uint64)
        sizes = np.array([f.size for f in filt], dtype=np.uint64)
        offs = eng.pack_offsets(sizes, 1)
        packed = np.zeros(int(offs[-1] + sizes[-1]), dtype=np.uint8)
        for f, o in zip(filt, offs):
            packed[int(o):int(o) + f.size] = f
        out = np.zeros(int(osz.sum()), dtype=np.uint8)
        oo = np.zeros_like(osz)
        oo[1:] = np.cumsum(osz)[:-1]
        st = ctx.unfilter_host(dp := eng.DevicePipeline(case.serialized, case.version, int(case.dtype),
                                                        case.cell_size),
                               offs + np.uint64(packed.ctypes.data), sizes, oo + np.uint64(out.ctypes.data), osz,
                               var_size=var, batch_bytes=1 << 20, contiguous_input=True,
                               contiguous_output=True)
        assert not st.any()
        for i, f in enumerate(filt):
            rc, ref = op.unfilter_tile(f, int(osz[i]), True)
            assert rc == 0
            got = out[int(oo[i]):int(oo[i] + osz[i])]
            assert np.array_equal(got[:-8], ref[:-8])
            assert int(got[-8:].view(np.uint64)[0]) == int(var[i])
        del dp


@pytest.mark.parametrize("ntiles,nvalues,max_chunk,flag", [
    (4, 262144, 0, False),        # 4 x 1 MiB tiles, 16 chunks each: fewer tiles than CUs (auto)
    (300, 16384, 8192, True),     # 300 x 64 KiB tiles, 8 chunks each: TDBG_CHUNK_PARALLEL
])
def test_chunk_parallel_multichunk(eng, ctx, oracle_mod, ntiles, nvalues, max_chunk, flag):
    """Chunk-parallel launches (device chunk directory, tdbg_chunkdir.hip):
    bit-exact with the oracle, every tile taken by the fused kernel."""
    import workloads as W
    from tiledb_amd.filter_pipeline import Datatype
    ser = W.c5_pipeline_bytes()
    op = oracle_mod.OraclePipeline(ser, 23, int(Datatype.INT32), 4)
    dp = eng.DevicePipeline(ser, 23, int(Datatype.INT32), 4)
    rng = np.random.default_rng(11)
    vals = [np.concatenate([W.c5_values("active", k, rng) for _ in range(nvalues // 16384)])
            for k in range(min(ntiles, 8))]
    enc = [np.frombuffer(op.filter_tile(v.view(np.uint8), None, max_chunk), dtype=np.uint8) for v in vals]
    filt = [enc[i % len(enc)] for i in range(ntiles)]
    osz = [vals[i % len(vals)].nbytes for i in range(ntiles)]
    batch = eng.TileBatch.from_host(filt, osz)
    f0, b0, _ = ctx.path_stats()
    st = ctx.unfilter(dp, batch, chunk_parallel=flag)
    f1, b1, _ = ctx.path_stats()
    assert not st.any()
    assert b1 - b0 == 0 and f1 - f0 == ntiles
    out = batch.outputs_host()
    for i in range(ntiles):
        o = int(batch.out_off[i])
        assert np.array_equal(out[o:o + osz[i]], vals[i % len(vals)].view(np.uint8)), f"tile {i}"


def test_chunk_parallel_corrupt_mix(eng, ctx, oracle_mod):
    """Chunk mode with corrupted tiles among good ones: statuses as the
    oracle's (header errors from the directory pass, chunk errors through the
    general interpreter), good tiles bit-exact."""
    import workloads as W
    from tiledb_amd.filter_pipeline import Datatype
    ser = W.c5_pipeline_bytes()
    op = oracle_mod.OraclePipeline(ser, 23, int(Datatype.INT32), 4)
    dp = eng.DevicePipeline(ser, 23, int(Datatype.INT32), 4)
    rng = np.random.default_rng(12)
    v = np.concatenate([W.c5_values("active", k, rng) for k in range(4)])
    good = np.frombuffer(op.filter_tile(v.view(np.uint8), None, 0), dtype=np.uint8)
    tiles = []
    for k in range(24):
        t = good.copy()
        if k % 4 == 1:
            t[:8] = 0x7f                      # chunk count: header walk fails
        elif k % 4 == 2:
            t[8 + 12 + 4 * (k % 5)] ^= 0x5a   # chunk metadata byte
        elif k % 4 == 3:
            t[len(t) // 2] ^= 0xff            # data byte
        tiles.append(t)
    osz = [v.nbytes] * len(tiles)
    batch = eng.TileBatch.from_host(tiles, osz)
    st = ctx.unfilter(dp, batch, chunk_parallel=True)
    out = batch.outputs_host()
    for i, t in enumerate(tiles):
        rc, ref = op.unfilter_tile(t, osz[i])
        assert int(st[i]) == rc, f"tile {i}: gpu {st[i]} oracle {rc}"
        if rc == 0:
            o = int(batch.out_off[i])
            assert np.array_equal(out[o:o + osz[i]], ref)


@pytest.mark.parametrize("variant", ["active", "ramp", "rand"])
def test_chunk_stream_multichunk(eng, ctx, oracle_mod, variant):
    """Multi-chunk C5 tiles (1 MiB minus a few values: 16 chunks, the last
    one short) in a chunk-parallel launch: the C5 tile kernel
    (tdbg_c5tile.hip) takes every chunk from the device chunk directory --
    the short last ones and the chunks of tiles whose outputs start only
    4-B aligned included; bit-exact vs the oracle, no fallback."""
    import workloads as W
    from tiledb_amd.filter_pipeline import Datatype
    ser = W.c5_pipeline_bytes()
    op = oracle_mod.OraclePipeline(ser, 23, int(Datatype.INT32), 4)
    dp = eng.DevicePipeline(ser, 23, int(Datatype.INT32), 4)
    rng = np.random.default_rng(21)
    vals = [np.concatenate([W.c5_values(variant, 16 * k + c, rng) for c in range(16)])[: 262144 - 9 * k - 1]
            for k in range(6)]
    enc = [np.frombuffer(op.filter_tile(v.view(np.uint8)), dtype=np.uint8) for v in vals]
    assert all(int(np.frombuffer(e[:8].tobytes(), dtype=np.uint64)[0]) == 16 for e in enc)
    n = 40
    batch = eng.TileBatch.from_host([enc[i % 6] for i in range(n)], [vals[i % 6].nbytes for i in range(n)])
    f0, b0, _ = ctx.path_stats()
    c0 = ctx.stream_chunks()
    st = ctx.unfilter(dp, batch, chunk_parallel=True)
    f1, b1, _ = ctx.path_stats()
    assert not st.any()
    assert b1 - b0 == 0 and f1 - f0 == n
    # (the outputs are packed back to back and these tiles' sizes are 4 mod
    # 16 apart: most tiles' chunks start only 4-B aligned)
    aligned = sum(int(batch.out_off[i]) % 16 == 0 for i in range(n))
    assert 0 < aligned < n
    assert ctx.stream_chunks() - c0 == 16 * n
    out = batch.outputs_host()
    for i in range(n):
        o = int(batch.out_off[i])
        assert np.array_equal(out[o:o + vals[i % 6].nbytes], vals[i % 6].view(np.uint8)), f"tile {i}"


def _chunk_headers(t):
    """(offset, orig, fl, ml) of every chunk header of a filtered tile (tile.cc:280-313)."""
    n = int(np.frombuffer(t[:8].tobytes(), dtype=np.uint64)[0])
    o, hs = 8, []
    for _ in range(n):
        orig, fl, ml = (int(x) for x in np.frombuffer(t[o:o + 12].tobytes(), dtype=np.uint32))
        hs.append((o, orig, fl, ml))
        o += 12 + ml + fl
    return hs


@pytest.mark.parametrize("variant", ["active", "rand"])
def test_chunk_stream_walk_rejects(eng, ctx, oracle_mod, variant):
    """Chunk mode: tiles whose chunk walk fails (a chunk's data or metadata
    size past the tile end, a chunk count one too high or one too low, an
    unfiltered size that no longer sums to the tile) among good 16-chunk
    tiles.  The directory counts chunks from the tile header and rejects on
    its single walk (tdbg_chunkdir.hip): statuses are the oracle's, a
    rejected tile's output keeps the fill bytes (no kernel takes its
    records), good tiles are bit-exact and all their full chunks stream."""
    import workloads as W
    from tiledb_amd.filter_pipeline import Datatype
    ser = W.c5_pipeline_bytes()
    op = oracle_mod.OraclePipeline(ser, 23, int(Datatype.INT32), 4)
    dp = eng.DevicePipeline(ser, 23, int(Datatype.INT32), 4)
    rng = np.random.default_rng(33)
    v = np.concatenate([W.c5_values(variant, c, rng) for c in range(16)])
    good = np.frombuffer(op.filter_tile(v.view(np.uint8)), dtype=np.uint8)
    hs = _chunk_headers(good)
    assert len(hs) == 16

    def put32(t, o, x):
        t[o:o + 4] = np.frombuffer(np.uint32(x).tobytes(), dtype=np.uint8)

    def mutate(k):
        t = good.copy()
        if k == 1:
            put32(t, hs[5][0] + 4, 0x7fffffff)      # chunk 5's data size past the end
        elif k == 2:
            put32(t, hs[9][0] + 8, 0x7fffffff)      # chunk 9's metadata size past the end
        elif k == 3:
            t[:8] = np.frombuffer(np.uint64(17).tobytes(), dtype=np.uint8)  # one chunk too many
        elif k == 4:
            t[:8] = np.frombuffer(np.uint64(15).tobytes(), dtype=np.uint8)  # one too few
        elif k == 5:
            put32(t, hs[7][0], hs[7][1] + 4)         # chunk 7's unfiltered size
        return t

    tiles = [mutate(k % 6) for k in range(36)]
    osz = [v.nbytes] * len(tiles)
    batch = eng.TileBatch.from_host(tiles, osz, fill=0x5A, align=16)
    c0 = ctx.stream_chunks()
    st = ctx.unfilter(dp, batch, chunk_parallel=True)
    out = batch.outputs_host()
    for i, t in enumerate(tiles):
        rc, ref = op.unfilter_tile(t, osz[i], fill=0x5A)
        assert int(st[i]) == rc, f"tile {i} (mutation {i % 6}): gpu {st[i]} oracle {rc}"
        o = int(batch.out_off[i])
        if i % 6 == 0:
            assert rc == 0 and np.array_equal(out[o:o + osz[i]], ref), f"tile {i}"
        else:
            assert rc != 0
            assert (out[o:o + osz[i]] == 0x5A).all(), f"tile {i}: a rejected tile's output was written"
    assert ctx.stream_chunks() - c0 == 16 * (len(tiles) // 6)


@pytest.mark.parametrize("case", _CONFIG, ids=[c.name for c in _CONFIG])
def test_chunk_parallel_many_tiles(eng, ctx, oracle_mod, case):
    """A chunk-parallel launch of more than 4,096 tiles (the directory's
    parallel header-count launch, tdbg_chunkdir.hip) with corrupted tiles
    among them (a chunk count past the tile, a chunk data size past the
    end): statuses and bytes as the oracle's."""
    _, enc = encode(oracle_mod, case)
    assert enc
    f = np.frombuffer(bytes(enc[0][0]), dtype=np.uint8).copy()
    bad_count = f.copy()
    bad_count[:8] = 0x7f
    bad_fl = f.copy()
    bad_fl[12:16] = 0xff  # chunk 0's filtered size
    enc = list(enc) + [(bad_count, None, enc[0][2]), (bad_fl, None, enc[0][2])]
    st = check_parity_replicated(eng, ctx, oracle_mod, case, enc, 4500, chunk_parallel=True)
    assert (st != 0).sum() >= 2 * (4500 // len(enc))
