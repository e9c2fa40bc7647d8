"""Edge cases of the dense-read step after the path, through
the C-ABI: subarray cells in no given space tile, launches without tiles,
fragments without validity tiles, offsets outside their var tile, and var
tiles whose unfilter needs the scratch retry.

The reference iterates every space tile of the subarray (DenseReader,
dense_reader.cc:1555-2007) and writes the fill value where no fragment has
data (:1610-1735); the async entries give every result cell the fill value
first, and the host var entry refuses a tile set that does not cover the
subarray exactly once, as tdbg_dense_read_host does.  Expected values come
from the oracle's restatements (oracle/oracle.py dense_copy_fragments,
dense_var_read)."""
from __future__ import annotations

import numpy as np
import pytest

from tiledb_amd.filter_pipeline import (BitWidthReductionFilter, CompressionFilter, Compressor, Datatype,
                                        FilterPipeline, PositiveDeltaFilter)

from .test_adjacent_steps import _frag_layout, _var_tiles

pytestmark = pytest.mark.gpu


def _dev(a, keep):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a)).to(torch.device("cuda", 0))
    keep.append(t)
    return t.data_ptr()


def _ptr_table(ptrs, keep):
    return _dev(np.array(ptrs or [0], dtype=np.uint64).view(np.int64), keep)


@pytest.mark.parametrize("drop", ["some", "all"])
def test_dense_copy_fragments_cells_outside_given_tiles_get_fill(oracle_mod, drop):
    """Space tiles left out of the launch (or no tiles at all): their cells
    of the subarray hold the fill value and fill validity, as if the tile had
    no fragment data."""
    import torch
    from tiledb_amd import engine
    rng = np.random.default_rng(41)
    shape_tiles, ext, lo, hi, nfrag = (3, 4), (8, 16), (2, 3), (21, 60), 2
    doms, starts, present = _frag_layout(rng, shape_tiles, ext, nfrag)
    ncell_t, cs = int(np.prod(ext)), 4
    keep_t = [i for i in range(len(starts)) if drop == "some" and i % 3 != 1]
    tiles = [[rng.integers(0, 256, ncell_t * cs, dtype=np.uint8) if present[t][f] else None
              for f in range(nfrag)] for t in range(len(starts))]
    # fragment 1 comes without validity tiles (NULL entries): its cells count
    # as valid
    vt = [[(rng.integers(0, 2, ncell_t, dtype=np.uint8) if f == 0 else np.ones(ncell_t, np.uint8))
           if present[t][f] else None for f in range(nfrag)] for t in range(len(starts))]
    # the oracle sees every space tile; the left-out ones have no fragment data
    o_tiles = [tiles[t] if t in keep_t else [None] * nfrag for t in range(len(starts))]
    o_vt = [vt[t] if t in keep_t else [None] * nfrag for t in range(len(starts))]
    fill = bytes([5, 6, 7, 8])
    want, wantv = oracle_mod.dense_copy_fragments(o_tiles, starts, ext, cs, lo, hi, doms, fill, 0, 0,
                                                  validity=o_vt, fill_validity=1)
    keep = []
    tp = _ptr_table([0 if tiles[t][f] is None else _dev(tiles[t][f], keep) for t in keep_t for f in range(nfrag)], keep)
    vp = _ptr_table([0 if (vt[t][f] is None or f == 1) else _dev(vt[t][f], keep) for t in keep_t for f in range(nfrag)],
                    keep)
    d_start = _dev(starts[keep_t].reshape(-1) if keep_t else np.zeros(1, np.int64), keep)
    d_dom = _dev(np.array(doms, dtype=np.int64).reshape(-1), keep)
    d_fill = _dev(np.frombuffer(fill, dtype=np.uint8).copy(), keep)
    fc = engine.dense_frag_config(cs, ext, lo, hi, nfrag, cs, 0, 0, nullable=True, fill_validity=1)
    ncell = int(np.prod([h - l + 1 for l, h in zip(lo, hi)]))
    d_res = torch.full((ncell * cs,), 0xEE, dtype=torch.uint8, device="cuda:0")
    d_resv = torch.full((ncell,), 0xEE, dtype=torch.uint8, device="cuda:0")
    ctx = engine.Context(0)
    engine.dense_copy_fragments_async(ctx, fc, len(keep_t), d_start, d_dom, tp, d_fill, d_res.data_ptr(), vp,
                                      d_resv.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(d_res.cpu().numpy(), want)
    assert np.array_equal(d_resv.cpu().numpy(), wantv)


def test_dense_var_offsets_without_tiles_are_fill(oracle_mod):
    """tdbg_dense_var_offsets_async with no space tiles: every result cell is
    the fill value (offsets 0, f, 2 f, ...; total = cells x f)."""
    import torch
    from tiledb_amd import engine
    ext, lo, hi = (8, 16), (2, 3), (21, 60)
    fill = bytes([9, 9, 9])
    keep = []
    fc = engine.dense_frag_config(8, ext, lo, hi, 1, len(fill), 0, 0)
    ncell = int(np.prod([h - l + 1 for l, h in zip(lo, hi)]))
    d_off = torch.full((ncell,), 7, dtype=torch.int64, device="cuda:0")
    d_tot = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    d_fill = _dev(np.frombuffer(fill, dtype=np.uint8).copy(), keep)
    ctx = engine.Context(0)
    engine.dense_var_offsets_async(ctx, fc, 0, None, None, None, None, d_fill, d_off.data_ptr(), d_tot.data_ptr())
    d_var = torch.zeros(ncell * len(fill), dtype=torch.uint8, device="cuda:0")
    engine.dense_var_copy_async(ctx, fc, d_off.data_ptr(), d_tot.data_ptr(), d_var.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(d_off.cpu().numpy(), np.arange(ncell, dtype=np.int64) * len(fill))
    assert int(d_tot.item()) == ncell * len(fill)
    assert bytes(d_var.cpu().numpy()) == fill * ncell


def _var_inputs(oracle_mod, rng, starts, ext, nfrag, present, offp, varp, vdt, maxlen):
    oo = oracle_mod.OraclePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    ov = oracle_mod.OraclePipeline(varp.serialize(), 23, int(vdt), 1)
    ncell_t = int(np.prod(ext))
    off_f, var_f, var_u, off_unf, var_unf = [], [], [], [], []
    for t in range(len(starts)):
        ou, vu = [], []
        for f in range(nfrag):
            if not present[t][f]:
                off_f.append(None)
                var_f.append(None)
                var_u.append(0)
                ou.append(None)
                vu.append(None)
                continue
            o_w, o_x, var = _var_tiles(rng, ncell_t, maxlen)
            off_f.append(np.frombuffer(oo.filter_tile(o_w.view(np.uint8)), dtype=np.uint8))
            var_f.append(np.frombuffer(ov.filter_tile(var, None, varp.max_chunk_size), dtype=np.uint8))
            var_u.append(var.size)
            ou.append(o_x.tobytes())
            vu.append(var.tobytes())
        off_unf.append(ou)
        var_unf.append(vu)
    return off_f, var_f, var_u, off_unf, var_unf


def test_dense_read_var_host_refuses_uncovered_subarray(oracle_mod):
    """tdbg_dense_read_var_host: a space tile of the subarray left out, a tile
    given twice, or no tiles at all: TDBG_E_ARG (nothing read from device
    memory that no tile wrote)."""
    from tiledb_amd import engine
    rng = np.random.default_rng(5)
    shape_tiles, ext, lo, hi, nfrag = (3, 4), (8, 16), (2, 3), (21, 60), 1
    doms, starts, present = _frag_layout(rng, shape_tiles, ext, nfrag)
    offp = FilterPipeline(65536, [PositiveDeltaFilter(1024), BitWidthReductionFilter(256)])
    varp = FilterPipeline(65536, [BitWidthReductionFilter(256)])
    off_f, var_f, var_u, _, _ = _var_inputs(oracle_mod, rng, starts, ext, nfrag, present, offp, varp,
                                            Datatype.UINT8, 6)
    ctx = engine.Context(0)
    dpo = engine.DevicePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    dpv = engine.DevicePipeline(varp.serialize(), 23, int(Datatype.UINT8), 1)
    fill = b"\x01\x02"
    fc = engine.dense_frag_config(8, ext, lo, hi, nfrag, len(fill), 0, 0)
    dom = np.array(doms, dtype=np.int64)
    # all tiles: fine
    rc, _, _, st = engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, dom, off_f, var_f, var_u, fill, 1 << 20)
    assert rc == 0 and not st.any()
    n = len(starts)
    for name, sel in (("dropped", [i for i in range(n) if i != 4]), ("twice", list(range(n)) + [0]), ("none", [])):
        with pytest.raises(engine.EngineError) as ei:
            engine.dense_read_var_host(ctx, dpo, dpv, fc, starts[sel] if sel else np.zeros((0, 2), np.int64), dom,
                                       [off_f[i] for i in sel], [var_f[i] for i in sel], [var_u[i] for i in sel],
                                       fill, 1 << 20)
        assert ei.value.code == 1, name  # TDBG_E_ARG


def test_dense_read_var_host_scratch_retry(oracle_mod):
    """Var tiles filtered with RLE on UINT8 cells in chunks of 1 MiB: the
    unfilter's stages outgrow the default scratch slots (TDBG_E_SCRATCH
    inside the launch) and are redone through the retry, so the read matches
    the oracle instead of failing."""
    from tiledb_amd import engine
    rng = np.random.default_rng(17)
    shape_tiles, ext, lo, hi, nfrag = (2, 2), (4, 16), (1, 2), (6, 29), 1
    doms, starts, present = _frag_layout(rng, shape_tiles, ext, nfrag)
    offp = FilterPipeline(65536, [PositiveDeltaFilter(1024), BitWidthReductionFilter(256)])
    varp = FilterPipeline(1 << 20, [CompressionFilter(Compressor.RLE, -1)])
    off_f, var_f, var_u, off_unf, var_unf = _var_inputs(oracle_mod, rng, starts, ext, nfrag, present, offp, varp,
                                                        Datatype.UINT8, 4000)
    assert max(var_u) > 120_000  # (a chunk bigger than the default slots)
    fill = b"\x05"
    want_o, want_d = oracle_mod.dense_var_read(off_unf, var_unf, starts, ext, lo, hi, doms, fill, 0, 0)
    ctx = engine.Context(0)
    dpo = engine.DevicePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    dpv = engine.DevicePipeline(varp.serialize(), 23, int(Datatype.UINT8), 1)
    fc = engine.dense_frag_config(8, ext, lo, hi, nfrag, len(fill), 0, 0)
    rc, got_o, got_d, st = engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, np.array(doms, dtype=np.int64),
                                                      off_f, var_f, var_u, fill, len(want_d) + 64)
    assert rc == 0 and not st.any(), st
    assert np.array_equal(got_o, want_o)
    assert got_d == want_d


def test_dense_read_var_host_offsets_outside_var_tile(oracle_mod):
    """An offsets tile whose offsets decrease, or pass the var tile's size:
    TDBG_E_DATA_READ, and the device reads nothing outside the var tile."""
    from tiledb_amd import engine
    rng = np.random.default_rng(23)
    shape_tiles, ext, lo, hi, nfrag = (1, 2), (4, 8), (0, 0), (3, 15), 1
    _, starts, _ = _frag_layout(rng, shape_tiles, ext, nfrag)
    doms, present = [[(0, 3), (0, 15)]], [[True], [True]]  # one fragment over the whole subarray
    offp = FilterPipeline(65536, [BitWidthReductionFilter(256)])  # (no PD: decreasing offsets encode)
    varp = FilterPipeline(65536, [BitWidthReductionFilter(256)])
    oo = oracle_mod.OraclePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    ov = oracle_mod.OraclePipeline(varp.serialize(), 23, int(Datatype.UINT8), 1)
    ctx = engine.Context(0)
    dpo = engine.DevicePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    dpv = engine.DevicePipeline(varp.serialize(), 23, int(Datatype.UINT8), 1)
    fc = engine.dense_frag_config(8, ext, lo, hi, nfrag, 1, 0, 0)
    for bad in ("decreasing", "past_end"):
        off_f, var_f, var_u = [], [], []
        for t in range(len(starts)):
            o_w, o_x, var = _var_tiles(rng, 32, 5)
            if t == 1:
                if bad == "decreasing":
                    o_w[7], o_w[8] = o_w[8] + 3, o_w[7]
                else:
                    o_w[31] = var.size + 40
            off_f.append(np.frombuffer(oo.filter_tile(o_w.view(np.uint8)), dtype=np.uint8))
            var_f.append(np.frombuffer(ov.filter_tile(var), dtype=np.uint8))
            var_u.append(var.size)
        with pytest.raises(engine.EngineError) as ei:
            engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, np.array(doms, dtype=np.int64), off_f, var_f, var_u,
                                       b"\x00", 1 << 16)
        assert ei.value.code == 5, bad  # TDBG_E_DATA_READ
    # the context works normally afterwards (the flag was cleared)
    off_f, var_f, var_u, off_unf, var_unf = _var_inputs(oracle_mod, rng, starts, ext, nfrag, present, offp, varp,
                                                        Datatype.UINT8, 5)
    want_o, want_d = oracle_mod.dense_var_read(off_unf, var_unf, starts, ext, lo, hi, doms, b"\x00", 0, 0)
    rc, got_o, got_d, st = engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, np.array(doms, dtype=np.int64),
                                                      off_f, var_f, var_u, b"\x00", 1 << 16)
    assert rc == 0 and np.array_equal(got_o, want_o) and got_d == want_d


def test_dense_var_offsets_async_flag_is_per_call(oracle_mod):
    """the async offsets entry clears the context's data flag on
    the caller's stream at every call, and tdbg_dense_var_status reports it.
    Bad offsets -> TDBG_E_DATA_READ from the status query; the next async call
    with good offsets -> TDBG_OK; a host read on the same context then
    matches the oracle (the flag no longer outlives its call)."""
    import torch
    from tiledb_amd import engine
    rng = np.random.default_rng(29)
    ext, lo, hi = (4, 8), (0, 0), (3, 15)
    starts = np.array([(0, 0), (0, 8)], dtype=np.int64)
    doms = [[(0, 3), (0, 15)]]
    fc = engine.dense_frag_config(8, ext, lo, hi, 1, 1, 0, 0)
    keep = []
    ctx = engine.Context(0)

    def run(bad):
        offs_t, var_t, want_tot = [], [], 0
        for t in range(2):
            _, o_x, var = _var_tiles(rng, 32, 5)
            if bad and t == 1:
                o_x[20] = var.size + 40  # past the var tile's end
            want_tot += var.size
            offs_t.append(_dev(o_x.view(np.int64), keep))
            var_t.append(_dev(var if var.size else np.zeros(1, np.uint8), keep))
        d_off = torch.zeros(64, dtype=torch.int64, device="cuda:0")
        d_tot = torch.zeros(1, dtype=torch.int64, device="cuda:0")
        d_fill = _dev(np.zeros(1, np.uint8), keep)
        engine.dense_var_offsets_async(ctx, fc, 2, _dev(starts.reshape(-1), keep),
                                       _dev(np.array(doms, dtype=np.int64).reshape(-1), keep),
                                       _ptr_table(offs_t, keep), _ptr_table(var_t, keep), d_fill,
                                       d_off.data_ptr(), d_tot.data_ptr())
        return engine.dense_var_status(ctx), int(d_tot.item()), want_tot

    st, _, _ = run(True)
    assert st == 5  # TDBG_E_DATA_READ
    st, tot, want = run(False)
    assert st == 0 and tot == want
    st, _, _ = run(True)
    assert st == 5
    # a good host read on the same context right after a flagged async call
    nfrag, present = 1, [[True], [True]]
    offp = FilterPipeline(65536, [PositiveDeltaFilter(1024), BitWidthReductionFilter(256)])
    varp = FilterPipeline(65536, [BitWidthReductionFilter(256)])
    off_f, var_f, var_u, off_unf, var_unf = _var_inputs(oracle_mod, rng, starts, ext, nfrag, present, offp, varp,
                                                        Datatype.UINT8, 5)
    want_o, want_d = oracle_mod.dense_var_read(off_unf, var_unf, starts, ext, lo, hi, doms, b"\x00", 0, 0)
    dpo = engine.DevicePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    dpv = engine.DevicePipeline(varp.serialize(), 23, int(Datatype.UINT8), 1)
    rc, got_o, got_d, st = engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, np.array(doms, dtype=np.int64),
                                                      off_f, var_f, var_u, b"\x00", 1 << 16)
    assert rc == 0 and np.array_equal(got_o, want_o) and got_d == want_d
