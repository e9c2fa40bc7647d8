"""The steps either side of the path, through the C-ABI.

* FilteredData-style reads (tdbg_filtered_data_blocks / tdbg_read_unfilter_tiles):
  the block rule against the oracle's restatement of
  FilteredData::make_new_block_if_required (filtered_data.h:531-575) on the CPU,
  and on the GPU tiles read from fragment files by IO threads into
  NUMA-local pinned blocks, unfiltered, bit-exact against the oracle.
* Dense cell-slab copy fused with the D2H (tdbg_dense_read_host /
  tdbg_dense_copy_async): the subarray's cells against the oracle's
  restatement of DenseReader::copy_fixed_tiles (dense_reader.cc:1555-1750)
  for row/col-major cell orders and layouts, 1-3 dimensions, partial tiles.
"""
from __future__ import annotations

import os
import tempfile

import numpy as np
import pytest

import workloads as W
from tiledb_amd.filter_pipeline import ByteshuffleFilter, Datatype, FilterPipeline


# ---------------------------------------------------------------------------
# CPU: the block rule
# ---------------------------------------------------------------------------
def _random_layout(rng, ntiles, nfiles):
    fi = np.sort(rng.integers(0, nfiles, ntiles)).astype(np.uint32)
    size = rng.integers(1, 5000, ntiles).astype(np.uint64)
    off = np.zeros(ntiles, dtype=np.uint64)
    pos = {}
    for i in range(ntiles):
        f = int(fi[i])
        gap = int(rng.choice([0, 0, 7, 300, 5000, 200000]))
        off[i] = pos.get(f, 0) + gap
        pos[f] = int(off[i] + size[i])
    return fi, off, size


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("params", [(20971520, 104857600, 512000), (3000, 20000, 10), (0, 8000, 0),
                                    (10**9, 10**9, 10**9), (100, 100, 0)])
def test_filtered_data_blocks_match_reference_rule(oracle_mod, seed, params):
    from tiledb_amd import engine
    rng = np.random.default_rng(seed)
    fi, off, size = _random_layout(rng, 200, 3)
    got = engine.filtered_data_blocks(fi, off, size, *params)
    want = oracle_mod.filtered_data_blocks(fi, off, size, *params)
    assert got.tolist() == want


def test_filtered_data_blocks_edge_cases(oracle_mod):
    from tiledb_amd import engine
    assert engine.filtered_data_blocks([], [], []).tolist() == [0]
    assert engine.filtered_data_blocks([0], [5], [10]).tolist() == [0, 1]
    # overlapping / out-of-order offsets: the reference's unsigned gap wraps
    fi, off, size = [0, 0, 0], [100, 50, 400], [10, 10, 10]
    assert engine.filtered_data_blocks(fi, off, size, 30, 1000, 5).tolist() == \
        oracle_mod.filtered_data_blocks(fi, off, size, 30, 1000, 5)


# ---------------------------------------------------------------------------
# GPU: read + unfilter from fragment files
# ---------------------------------------------------------------------------
def _c5_pipe():
    return W.c5_pipeline_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_kind", ["default", "small_blocks", "zero_gap"])
def test_read_unfilter_tiles_from_files(oracle_mod, cfg_kind):
    import torch
    assert torch.cuda.is_available()
    from tiledb_amd import _native, engine
    rng = np.random.default_rng(41)
    pools = []
    for var in ("active", "ramp", "rand"):
        pools += list(zip(*W.c5_pool(var, 6, seed=42)))
    # three fragment files; tiles at their offsets with gaps between some
    nfiles = 3
    tiles, vals, fidx, foff = [], [], [], []
    with tempfile.TemporaryDirectory() as tmp:
        paths = [os.path.join(tmp, f"frag{f}.tdb") for f in range(nfiles)]
        blobs = [bytearray() for _ in range(nfiles)]
        order = rng.permutation(len(pools) * 3)
        for k in order:
            f = int(k % nfiles)
            t, v = pools[int(k) % len(pools)]
            blobs[f] += bytes(int(rng.choice([0, 0, 16, 3000, 700000])))
            fidx.append(f)
            foff.append(len(blobs[f]))
            blobs[f] += t
            tiles.append(t)
            vals.append(v)
        for pth, b in zip(paths, blobs):
            with open(pth, "wb") as fh:
                fh.write(bytes(b))
        # result-tile order: by fragment, then offset
        srt = sorted(range(len(tiles)), key=lambda i: (fidx[i], foff[i]))
        tiles = [tiles[i] for i in srt]
        vals = [vals[i] for i in srt]
        fidx = np.array([fidx[i] for i in srt], dtype=np.uint32)
        foff = np.array([foff[i] for i in srt], dtype=np.uint64)
        size = np.array([len(t) for t in tiles], dtype=np.uint64)
        fds = [os.open(pth, os.O_RDONLY) for pth in paths]
        try:
            ctx = engine.Context(0)
            dp = engine.DevicePipeline(_c5_pipe(), 23, int(Datatype.INT32), 4)
            res = engine.HostBuffer(0, len(tiles) * W.TILE_BYTES)
            out_ptrs = res.ptr + np.arange(len(tiles), dtype=np.uint64) * np.uint64(W.TILE_BYTES)
            cfg = _native.ReadConfig()
            if cfg_kind == "small_blocks":
                cfg.min_batch_size, cfg.max_batch_size, cfg.min_batch_gap = 100000, 300000, 100
                cfg.io_threads, cfg.slots = 2, 2
            elif cfg_kind == "zero_gap":
                cfg.min_batch_size, cfg.flags = 1, 0x1  # TDBG_READ_ZERO_GAP
            st = ctx.read_unfilter(dp, fds, fidx, foff, size, out_ptrs,
                                   np.full(len(tiles), W.TILE_BYTES, dtype=np.uint64), cfg=cfg)
            assert not st.any(), np.unique(st)
            op = oracle_mod.OraclePipeline(_c5_pipe(), 23, int(Datatype.INT32), 4)
            for i, t in enumerate(tiles):
                got = res.array[i * W.TILE_BYTES:(i + 1) * W.TILE_BYTES]
                rc, ref = op.unfilter_tile(np.frombuffer(t, dtype=np.uint8), W.TILE_BYTES)
                assert rc == 0 and np.array_equal(got, ref), f"tile {i}"
                assert np.array_equal(got, vals[i].view(np.uint8))
            # a file too short for its last block: those tiles get TDBG_E_IO
            st2 = ctx.read_unfilter(dp, fds, fidx, foff + np.uint64(10**9), size, out_ptrs,
                                    np.full(len(tiles), W.TILE_BYTES, dtype=np.uint64), cfg=cfg)
            assert (st2 == 18).all()
        finally:
            for fd in fds:
                os.close(fd)


@pytest.mark.gpu
def test_read_unfilter_statuses_after_device_failure():
    """A device error in block 1 (injected: TDBG_DEBUG_IO_FAIL_BLOCK) after a
    block holding a corrupt tile: block 0 keeps its real statuses (the corrupt
    tile's error, OK for the rest), every tile of block 1 and after says
    TDBG_E_NOT_RUN -- never OK for output that was not written -- and the call
    raises the device error although some tiles carry statuses.  The fault
    injection exists only in the experiments library (tdbg_hooks.h), so the
    case runs in a child process that loads it (TDBG_LIB)."""
    import subprocess
    import sys
    from tiledb_amd import build as B
    assert os.path.exists(B.EXP_LIB), "experiments library missing: __graft_entry__.build() builds it"
    env = dict(os.environ, TDBG_LIB=os.path.basename(B.EXP_LIB))
    code = ("import sys; sys.path.insert(0, %r); from oracle import oracle as O; O.build(); "
            "from tests.test_adjacent_steps import _device_failure_case; _device_failure_case(O)" % B.ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


def test_product_library_ignores_hooks():
    """The product library reads no TDBG_* timing, ablation or fault hook
    (tdbg_hooks.h compiles them out): none of their names is left in it,
    while the experiments library keeps them."""
    from tiledb_amd import build as B
    names = (b"TDBG_DEBUG_STOP", b"TDBG_NO_STREAM", b"TDBG_DEBUG_SKIP_FUSED", b"TDBG_DEBUG_SKIP_FIXUP",
             b"TDBG_DEBUG_IO_FAIL_BLOCK", b"TDBG_C5T_ABL", b"TDBG_DEBUG_TILE_MODE", b"TDBG_C5_OLD_RAW")
    with open(B.LIB, "rb") as fh:
        blob = fh.read()
    for name in names:
        assert name not in blob, name
    if os.path.exists(B.EXP_LIB):
        with open(B.EXP_LIB, "rb") as fh:
            assert b"TDBG_DEBUG_IO_FAIL_BLOCK" in fh.read()


def _device_failure_case(oracle_mod):
    import torch
    assert torch.cuda.is_available()
    monkeypatch = pytest.MonkeyPatch()
    from tiledb_amd import _native, engine
    tiles, vals = W.c5_pool("active", 8, seed=7)
    tiles = [bytearray(t) for t in tiles]
    tiles[1][8:12] = (70000).to_bytes(4, "little")  # chunk orig size != tile size
    with tempfile.TemporaryDirectory() as tmp:
        pth = os.path.join(tmp, "frag.tdb")
        blob, foff = bytearray(), []
        for t in tiles:
            foff.append(len(blob))
            blob += t
        with open(pth, "wb") as fh:
            fh.write(bytes(blob))
        fd = os.open(pth, os.O_RDONLY)
        try:
            ctx = engine.Context(0)
            dp = engine.DevicePipeline(_c5_pipe(), 23, int(Datatype.INT32), 4)
            n = len(tiles)
            res = engine.HostBuffer(0, n * W.TILE_BYTES)
            out_ptrs = res.ptr + np.arange(n, dtype=np.uint64) * np.uint64(W.TILE_BYTES)
            cfg = _native.ReadConfig()
            # blocks of 2 tiles: [0, 1], [2, 3], ...
            cfg.min_batch_size, cfg.max_batch_size, cfg.min_batch_gap = 1, 2 * max(len(t) for t in tiles), 0
            cfg.flags = 0x1  # TDBG_READ_ZERO_GAP
            size = np.array([len(t) for t in tiles], dtype=np.uint64)
            fidx = np.zeros(n, dtype=np.uint32)
            nb = oracle_mod.filtered_data_blocks(fidx, np.array(foff, dtype=np.uint64), size,
                                                                  cfg.min_batch_size, cfg.max_batch_size, 0)
            assert list(nb[:3]) == [0, 2, 4], nb
            monkeypatch.setenv("TDBG_DEBUG_IO_FAIL_BLOCK", "1")
            st = np.full(n, -1, dtype=np.int32)
            with pytest.raises(engine.EngineError) as ei:
                ctx.read_unfilter(dp, [fd], fidx, np.array(foff, dtype=np.uint64), size, out_ptrs,
                                  np.full(n, W.TILE_BYTES, dtype=np.uint64), cfg=cfg, status_out=st)
            assert ei.value.code == 14  # TDBG_E_DEVICE
            assert st[0] == 0 and st[1] == 3  # TDBG_E_TILE_SIZE (tile.cc:308)
            assert (st[2:] == engine.E_NOT_RUN).all(), st
            assert np.array_equal(res.array[:W.TILE_BYTES], vals[0].view(np.uint8))
            monkeypatch.delenv("TDBG_DEBUG_IO_FAIL_BLOCK")
            st = ctx.read_unfilter(dp, [fd], fidx, np.array(foff, dtype=np.uint64), size, out_ptrs,
                                   np.full(n, W.TILE_BYTES, dtype=np.uint64), cfg=cfg)
            assert st[1] == 3 and (np.delete(st, 1) == 0).all(), st
        finally:
            os.close(fd)


# ---------------------------------------------------------------------------
# GPU: dense cell-slab copy fused with the D2H
# ---------------------------------------------------------------------------
def _dense_tiles(shape_tiles, ext, cell_order, rng, dtype=np.int32):
    """A dense array of whole tiles (the domain is tile-aligned) and its tiles'
    cell bytes in the given cell order."""
    nd = len(ext)
    full = tuple(t * e for t, e in zip(shape_tiles, ext))
    A = rng.integers(-2**31, 2**31, full, dtype=np.int64).astype(dtype)
    tiles, starts = [], []
    for idx in np.ndindex(*shape_tiles):
        s = tuple(i * e for i, e in zip(idx, ext))
        blk = A[tuple(slice(s[d], s[d] + ext[d]) for d in range(nd))]
        cells = blk.reshape(-1) if cell_order == 0 else np.asfortranarray(blk).T.reshape(-1)
        tiles.append(np.ascontiguousarray(cells).view(np.uint8))
        starts.append(s)
    return A, tiles, np.array(starts, dtype=np.int64)


_DENSE = [
    ((4, 5), (16, 32), (3, 7), (60, 150), 0, 0),
    ((4, 5), (16, 32), (3, 7), (60, 150), 0, 1),
    ((4, 5), (16, 32), (0, 0), (63, 159), 1, 0),
    ((4, 5), (16, 32), (17, 40), (17, 140), 1, 1),
    ((3,), (1000,), (5,), (2990,), 0, 0),
    ((2, 3, 4), (8, 4, 16), (1, 2, 3), (14, 10, 60), 0, 0),
    ((2, 3, 4), (8, 4, 16), (1, 2, 3), (14, 10, 60), 1, 1),
    ((2, 3, 4), (8, 4, 16), (0, 0, 0), (0, 11, 63), 0, 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", _DENSE, ids=lambda c: f"t{'x'.join(map(str, c[0]))}_o{c[4]}l{c[5]}")
def test_dense_read_fused_copy(oracle_mod, case):
    import torch
    assert torch.cuda.is_available()
    from tiledb_amd import engine
    shape_tiles, ext, lo, hi, cell_order, layout = case
    rng = np.random.default_rng(sum(ext) + cell_order + 2 * layout)
    A, raw, starts = _dense_tiles(shape_tiles, ext, cell_order, rng)
    # C1's pipeline ([BYTESHUFFLE] on INT32) and C5's
    for ser in (FilterPipeline(65536, [ByteshuffleFilter()]).serialize(), _c5_pipe()):
        op = oracle_mod.OraclePipeline(ser, 23, int(Datatype.INT32), 4)
        filt = [np.frombuffer(op.filter_tile(t), dtype=np.uint8) for t in raw]
        ctx = engine.Context(0)
        dp = engine.DevicePipeline(ser, 23, int(Datatype.INT32), 4)
        cfg = engine.dense_config(4, ext, lo, hi, cell_order, layout)
        nb = engine.dense_result_bytes(cfg)
        result = np.full(nb, 0xAB, dtype=np.uint8)
        st = ctx.dense_read(dp, filt, starts, cfg, result, batch_bytes=1 << 20)
        assert not st.any()
        want = oracle_mod.dense_subarray_cells(raw, starts, ext, 4, lo, hi, cell_order, layout)
        assert np.array_equal(result, want)
        sub = A[tuple(slice(l, h + 1) for l, h in zip(lo, hi))]
        ref = (sub.reshape(-1) if layout == 0 else np.asfortranarray(sub).T.reshape(-1)).view(np.uint8)
        assert np.array_equal(result, ref)


@pytest.mark.gpu
def test_dense_read_rejects_uncovered_subarray():
    """tdbg_dense_read_host has no fill value: a tile set that leaves result
    cells uncovered (a missing tile, a tile given twice, a start off the tile
    grid) is an argument error, and the result buffer is left untouched."""
    from tiledb_amd import engine
    rng = np.random.default_rng(77)
    ext, shape_tiles, lo, hi = (16, 32), (3, 3), (2, 5), (40, 90)
    _, raw, starts = _dense_tiles(shape_tiles, ext, 0, rng)
    ser = FilterPipeline(65536, [ByteshuffleFilter()]).serialize()
    ctx = engine.Context(0)
    dp = engine.DevicePipeline(ser, 23, int(Datatype.INT32), 4)
    cfg = engine.dense_config(4, ext, lo, hi, 0, 0)
    nb = engine.dense_result_bytes(cfg)
    off = starts.copy()
    off[4] += (1, 0)
    for tiles, st in ((raw[:-1], starts[:-1]), (raw + raw[:1], np.vstack([starts, starts[:1]])), (raw, off)):
        result = np.full(nb, 0xAB, dtype=np.uint8)
        with pytest.raises(engine.EngineError) as ei:
            ctx.dense_read(dp, tiles, st, cfg, result)
        assert ei.value.code == 1  # TDBG_E_ARG
        assert (result == 0xAB).all()


@pytest.mark.gpu
def test_dense_copy_async_skips_failed_tiles(oracle_mod):
    """Device-resident copy: a tile whose status is not OK leaves its cells
    untouched; the others land where copy_fixed_tiles puts them."""
    import torch
    from tiledb_amd import engine
    rng = np.random.default_rng(51)
    ext, shape_tiles, lo, hi = (16, 32), (3, 3), (2, 5), (40, 90)
    A, raw, starts = _dense_tiles(shape_tiles, ext, 0, rng)
    dev = torch.device("cuda", 0)
    d_tiles = [torch.from_numpy(t.copy()).to(dev) for t in raw]
    ptrs = torch.tensor([t.data_ptr() for t in d_tiles], dtype=torch.int64, device=dev)
    d_start = torch.from_numpy(starts.reshape(-1)).to(dev)
    status = torch.zeros(len(raw), dtype=torch.int32, device=dev)
    status[4] = 5
    cfg = engine.dense_config(4, ext, lo, hi)
    d_res = torch.full((engine.dense_result_bytes(cfg),), 7, dtype=torch.uint8, device=dev)
    ctx = engine.Context(0)
    ctx.dense_copy_async(cfg, len(raw), d_start.data_ptr(), ptrs.data_ptr(), d_res.data_ptr(),
                         d_status=status.data_ptr())
    torch.cuda.synchronize()
    got = d_res.cpu().numpy()
    want = oracle_mod.dense_subarray_cells(raw, starts, ext, 4, lo, hi)
    # which result bytes come from tile 4: mark its cells and copy the marks
    marks = [np.full(t.size, 1 if i == 4 else 0, np.uint8) for i, t in enumerate(raw)]
    mask = oracle_mod.dense_subarray_cells(marks, starts, ext, 4, lo, hi).astype(bool)
    assert mask.any() and not mask.all()
    assert np.array_equal(got[~mask], want[~mask])
    assert (got[mask] == 7).all()


# ---------------------------------------------------------------------------
# Several fragments, fill values, var-sized cells (dense_reader.cc:1199-2000)
# ---------------------------------------------------------------------------
def _frag_layout(rng, shape_tiles, ext, nfrag):
    """Fragment domains (random boxes over the array, overlapping) and, per
    (space tile, fragment), whether the fragment has a tile there (it must
    when its domain meets the tile; a few that do not meet it get one too)."""
    nd = len(ext)
    full = [t * e for t, e in zip(shape_tiles, ext)]
    doms = []
    for _ in range(nfrag):
        lo = [int(rng.integers(0, full[d])) for d in range(nd)]
        hi = [int(rng.integers(lo[d], full[d])) for d in range(nd)]
        doms.append([(lo[d], hi[d]) for d in range(nd)])
    starts = [tuple(i * e for i, e in zip(idx, ext)) for idx in np.ndindex(*shape_tiles)]
    present = []
    for s in starts:
        row = []
        for dom in doms:
            meets = all(dom[d][0] <= s[d] + ext[d] - 1 and dom[d][1] >= s[d] for d in range(nd))
            row.append(meets or bool(rng.integers(0, 4) == 0))
        present.append(row)
    return doms, np.array(starts, dtype=np.int64), present


def test_oracle_dense_var_single_fragment_is_concatenation(oracle_mod):
    """The var restatement with one fragment covering the subarray and whole
    tiles equals the cells' bytes in result order (no fill involved)."""
    rng = np.random.default_rng(3)
    ext = (4, 6)
    starts = [(0, 0), (0, 6), (4, 0), (4, 6)]
    cells, offs_t, var_t = {}, [], []
    for s in starts:
        lens = rng.integers(0, 9, 24)
        blob, offs = b"", []
        for k in range(24):
            r, c = divmod(k, 6)
            b = bytes(rng.integers(0, 256, int(lens[k]), dtype=np.uint8))
            cells[(s[0] + r, s[1] + c)] = b
            offs.append(len(blob))
            blob += b
        offs_t.append([np.array(offs + [len(blob)], dtype=np.uint64).tobytes()])
        var_t.append([blob])
    o, data = oracle_mod.dense_var_read(offs_t, var_t, starts, ext, (1, 2), (6, 10), [[(0, 7), (0, 11)]], b"xy")
    want = [cells[(r, c)] for r in range(1, 7) for c in range(2, 11)]
    assert data == b"".join(want)
    assert list(o) == list(np.cumsum([0] + [len(w) for w in want[:-1]]))


_FRAGS = [((3, 4), (8, 16), (2, 3), (21, 60), 3, 0, 0, False),
          ((3, 4), (8, 16), (0, 0), (23, 63), 2, 1, 0, True),
          ((3, 4), (8, 16), (5, 9), (20, 50), 4, 0, 1, True),
          ((2, 2, 3), (4, 8, 8), (1, 0, 3), (7, 14, 20), 3, 1, 1, False),
          ((5,), (512,), (100,), (2400,), 0, 0, 0, True),
         # one fragment: slab copies where its domain holds a tile's whole
         # region in the result's order, cell copies elsewhere
         ((3, 4), (8, 16), (2, 3), (21, 60), 1, 0, 0, True),
         ((3, 4), (8, 16), (0, 0), (23, 63), 1, 1, 1, False),
         ((3, 4), (8, 16), (1, 2), (22, 61), 1, 0, 1, True),
         ((2, 2, 3), (4, 8, 8), (1, 0, 3), (7, 14, 20), 1, 1, 1, True),
         ((5,), (512,), (100,), (2400,), 1, 0, 0, False)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", _FRAGS, ids=lambda c: f"f{c[4]}_t{'x'.join(map(str, c[0]))}_o{c[5]}l{c[6]}")
def test_dense_copy_fragments(oracle_mod, case):
    """copy_fixed_tiles with several overlapping fragments, absent tiles, the
    fill value and validity (nullable), on device tiles: bit-exact against
    the oracle's restatement (dense_reader.cc:1555-1750)."""
    _check_fragments(oracle_mod, case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in _FRAGS if c[4] == 1], ids=lambda c: f"t{'x'.join(map(str, c[0]))}_o{c[5]}l{c[6]}")
@pytest.mark.parametrize("cover", ["whole", "most"])
def test_dense_copy_one_fragment_slabs(oracle_mod, case, cover):
    """One fragment whose domain holds the whole array (every tile's region
    goes through the slab copier when the orders agree) or all of it but the
    last cell row / column of every dimension (the edge tiles fall back to
    cell copies, the fill value beyond the domain): bit-exact."""
    shape_tiles, ext = case[0], case[1]
    full = [t * e for t, e in zip(shape_tiles, ext)]
    hi = [f - 1 - (1 if cover == "most" else 0) for f in full]
    _check_fragments(oracle_mod, case, doms=[[(0, h) for h in hi]])


def _check_fragments(oracle_mod, case, doms=None):
    import torch
    from tiledb_amd import engine
    shape_tiles, ext, lo, hi, nfrag, cell_order, layout, nullable = case
    rng = np.random.default_rng(nfrag * 7 + cell_order + 3 * layout + len(ext))
    rdoms, starts, present = _frag_layout(rng, shape_tiles, ext, nfrag)
    if doms is not None:  # (every tile present)
        present = [[True] * nfrag for _ in present]
    else:
        doms = rdoms
    ncell_t = int(np.prod(ext))
    cs = 8
    tiles = [[rng.integers(0, 256, ncell_t * cs, dtype=np.uint8) if present[t][f] else None
              for f in range(nfrag)] for t in range(len(starts))]
    vtiles = [[rng.integers(0, 2, ncell_t, dtype=np.uint8) if present[t][f] else None for f in range(nfrag)]
              for t in range(len(starts))]
    fill = bytes(range(100, 100 + cs))
    want = oracle_mod.dense_copy_fragments(tiles, starts, ext, cs, lo, hi, doms, fill, cell_order, layout,
                                           validity=vtiles if nullable else None, fill_validity=1)
    dev = torch.device("cuda", 0)
    keep = []

    def dptr(a):
        if a is None:
            return 0
        t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        keep.append(t)
        return t.data_ptr()

    tp = torch.from_numpy(np.array([dptr(tiles[t][f]) for t in range(len(starts)) for f in range(nfrag)] or [0],
                                   dtype=np.uint64).view(np.int64)).to(dev)
    vp = torch.from_numpy(np.array([dptr(vtiles[t][f]) for t in range(len(starts)) for f in range(nfrag)] or [0],
                                   dtype=np.uint64).view(np.int64)).to(dev)
    d_start = torch.from_numpy(starts.reshape(-1)).to(dev)
    d_dom = torch.from_numpy(np.array(doms, dtype=np.int64).reshape(-1) if nfrag else np.zeros(1, np.int64)).to(dev)
    d_fill = torch.from_numpy(np.frombuffer(fill, dtype=np.uint8).copy()).to(dev)
    fc = engine.dense_frag_config(cs, ext, lo, hi, nfrag, cs, cell_order, layout, nullable=nullable, fill_validity=1)
    ncell = int(np.prod([h - l + 1 for l, h in zip(lo, hi)]))
    d_res = torch.full((ncell * cs,), 0xEE, dtype=torch.uint8, device=dev)
    d_resv = torch.full((ncell,), 0xEE, dtype=torch.uint8, device=dev)
    ctx = engine.Context(0)
    engine.dense_copy_fragments_async(ctx, fc, len(starts), d_start.data_ptr(), d_dom.data_ptr(), tp.data_ptr(),
                                      d_fill.data_ptr(), d_res.data_ptr(), vp.data_ptr() if nullable else None,
                                      d_resv.data_ptr() if nullable else None)
    torch.cuda.synchronize()
    if nullable:
        res, val = want
        assert np.array_equal(d_res.cpu().numpy(), res)
        assert np.array_equal(d_resv.cpu().numpy(), val)
    else:
        assert np.array_equal(d_res.cpu().numpy(), want)


def _var_tiles(rng, ncell_t, maxlen):
    """One var tile: cells of 0..maxlen bytes; its offsets tile as TileDB
    writes it (cell byte offsets, no extra offset) and the unfiltered offsets
    tile with the extra offset (tile.h:144-146)."""
    lens = rng.integers(0, maxlen + 1, ncell_t)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    var = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    return offs[:-1].copy(), offs, var


_VAR = [((3, 4), (8, 16), (2, 3), (21, 60), 3, 0, 0, False),
        ((3, 4), (8, 16), (0, 0), (23, 63), 1, 1, 0, False),
        ((2, 2, 3), (4, 8, 8), (1, 0, 3), (7, 14, 20), 3, 1, 1, True),
        ((5,), (512,), (100,), (2400,), 2, 0, 0, True),
        ((3, 4), (8, 16), (5, 9), (20, 50), 0, 0, 1, False)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", _VAR, ids=lambda c: f"f{c[4]}_t{'x'.join(map(str, c[0]))}_o{c[5]}l{c[6]}_e{int(c[7])}")
def test_dense_read_var_host(oracle_mod, case):
    """A var-sized attribute's dense read (copy_offset_tiles +
    fix_offsets_buffer + copy_var_tiles) from FILTERED offsets and var tiles
    of several fragments: offsets unfiltered with the extra offset fused on
    the device, the var bytes gathered there, one D2H of each result buffer;
    bit-exact against the oracle's restatement, elements mode included."""
    import torch
    assert torch.cuda.is_available()
    from tiledb_amd import engine
    from tiledb_amd.filter_pipeline import (BitshuffleFilter, BitWidthReductionFilter, PositiveDeltaFilter)
    shape_tiles, ext, lo, hi, nfrag, cell_order, layout, elements = case
    tsz = 4 if elements else 1  # elements mode: INT32 cells counted in elements
    rng = np.random.default_rng(nfrag * 13 + cell_order + 5 * layout + len(ext))
    doms, starts, present = _frag_layout(rng, shape_tiles, ext, nfrag) if nfrag else \
        ([], np.array([tuple(i * e for i, e in zip(idx, ext)) for idx in np.ndindex(*shape_tiles)]), [[]] * int(np.prod(shape_tiles)))
    ncell_t = int(np.prod(ext))
    offp = FilterPipeline(65536, [PositiveDeltaFilter(1024), BitWidthReductionFilter(256)])
    varp = FilterPipeline(65536, [BitshuffleFilter()])
    oo = oracle_mod.OraclePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    vdt = Datatype.INT32 if elements else Datatype.UINT8
    ov = oracle_mod.OraclePipeline(varp.serialize(), 23, int(vdt), 4 if elements else 1)
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
            o_w, o_x, var = _var_tiles(rng, ncell_t, 12)
            if elements:  # whole INT32 elements per cell
                o_w, o_x = o_w * 4, o_x * 4
                var = rng.integers(0, 256, int(o_x[-1]), dtype=np.uint8)
            off_f.append(np.frombuffer(oo.filter_tile(o_w.view(np.uint8)), dtype=np.uint8))
            var_f.append(np.frombuffer(ov.filter_tile(var), dtype=np.uint8))
            var_u.append(var.size)
            ou.append(o_x.tobytes())
            vu.append(var.tobytes())
        off_unf.append(ou)
        var_unf.append(vu)
    fill = bytes([7, 8, 9, 10, 11, 12, 13, 14])
    want_o, want_d = oracle_mod.dense_var_read(off_unf, var_unf, starts, ext, lo, hi, doms, fill, cell_order, layout,
                                               elements_mode=elements, type_size=tsz)
    ctx = engine.Context(0)
    dpo = engine.DevicePipeline(offp.serialize(), 23, int(Datatype.UINT64), 8)
    dpv = engine.DevicePipeline(varp.serialize(), 23, int(vdt), 4 if elements else 1)
    fc = engine.dense_frag_config(8, ext, lo, hi, nfrag, len(fill), cell_order, layout, elements_mode=elements,
                                  data_type_size=tsz)
    rc, got_o, got_d, st = engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, np.array(doms, dtype=np.int64),
                                                      off_f, var_f, var_u, fill, len(want_d) + 64)
    assert rc == 0 and not st.any()
    assert np.array_equal(got_o, want_o)
    assert got_d == want_d
    if len(want_d) > 1:  # a result buffer one byte short: TDBG_E_OUT_FULL, nothing copied
        with pytest.raises(engine.EngineError) as ei:
            engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, np.array(doms, dtype=np.int64), off_f, var_f, var_u,
                                       fill, len(want_d) - 1)
        assert ei.value.code == 6
