"""CPU entry parity (no GPU): tdbg_unfilter_tiles_cpu, the C-ABI's host-thread
unfilter, against the oracle -- bit-exact bytes and identical
statuses on the BASELINE configs, the SURVEY A.5 edge cases, random pipelines,
corrupted tiles and wrong output sizes, with the reference's tile x chunk-range
split (reader_base.cc:929-989) exercised by multi-chunk tiles on many threads.
"""
from __future__ import annotations

import threading

import numpy as np
import pytest

from tests.cases import config_cases, edge_cases, random_cases


@pytest.fixture(scope="module")
def eng():
    from tiledb_amd import engine
    return engine


def _encode(O, case):
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
    return enc


def cpu_unfilter(eng, case, filtered, out_sizes, nthreads=4, fill=0, align=1):
    """Packs tiles back to back (arbitrary starts) and outputs back to back."""
    dp = eng.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    sizes = np.array([f.size for f in filtered], dtype=np.uint64)
    offs = eng.pack_offsets(sizes, align)
    hin = np.zeros(int(offs[-1] + sizes[-1]) + 1 if sizes.size else 1, dtype=np.uint8)
    for f, o in zip(filtered, offs):
        hin[int(o):int(o) + f.size] = f
    osz = np.array(out_sizes, dtype=np.uint64)
    ooff = eng.pack_offsets(osz, 1)
    hout = np.full(int(osz.sum()) + 1, fill, dtype=np.uint8)
    st = eng.unfilter_cpu(dp, offs + np.uint64(hin.ctypes.data), sizes, ooff + np.uint64(hout.ctypes.data),
                          osz, nthreads=nthreads, offsets_tiles=case.offsets_tile)
    outs = [hout[int(o):int(o) + int(n)] for o, n in zip(ooff, osz)]
    return st, outs


def check(eng, O, case, filtered, out_sizes, fill=0, nthreads=4):
    op = O.OraclePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
    st, outs = cpu_unfilter(eng, case, filtered, out_sizes, nthreads=nthreads, fill=fill)
    for i, f in enumerate(filtered):
        rc, ref = op.unfilter_tile(f, out_sizes[i], case.offsets_tile, fill=fill)
        assert int(st[i]) == rc, f"{case.name} tile {i}: cpu status {st[i]} oracle {rc}"
        if rc == 0:
            got = outs[i]
            if not np.array_equal(got, ref):
                bad = np.nonzero(got != ref)[0]
                raise AssertionError(f"{case.name} tile {i}: {bad.size} bytes differ, first at {bad[0]}")


_CONFIG = config_cases(3)
_EDGE = edge_cases()


@pytest.mark.parametrize("case", _CONFIG + _EDGE, ids=[c.name for c in _CONFIG + _EDGE])
def test_cpu_entry_parity(eng, oracle_mod, case):
    enc = _encode(oracle_mod, case)
    if not enc:
        pytest.skip("reference encoder rejects this input")
    check(eng, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc])


def test_cpu_entry_random_pipelines(eng, oracle_mod):
    n = 0
    for case in random_cases(60):
        enc = _encode(oracle_mod, case)
        if not enc:
            continue
        check(eng, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc])
        n += 1
    assert n > 30


def _mutations(f: np.ndarray, rng):
    out = [f[: max(0, f.size - 1)], f[: f.size // 2], f[:7]]
    g = f.copy(); g[0] ^= 3; out.append(g)
    if f.size > 12:
        for k, m in ((8, 1), (12, 0x40), (16, 0x10)):
            g = f.copy(); g[k] ^= m; out.append(g)
    for _ in range(8):
        if f.size > 24:
            g = f.copy()
            k = int(rng.integers(20, min(f.size, 160)))
            g[k] ^= np.uint8(1 << int(rng.integers(8)))
            out.append(g)
    return out


@pytest.mark.parametrize("case", _CONFIG + [c for c in _EDGE if c.name.startswith(
    ("dd_", "rle_", "bwr_", "pd_", "byte_bit", "xor_", "fscale_", "delta_", "multichunk"))],
    ids=lambda c: c.name)
def test_cpu_entry_corrupt_status_parity(eng, oracle_mod, case):
    rng = np.random.default_rng(3)
    enc = _encode(oracle_mod, case)
    if not enc:
        pytest.skip("reference encoder rejects this input")
    f, t, osz = enc[0]
    muts = _mutations(f, rng)
    check(eng, oracle_mod, case, muts, [osz] * len(muts), fill=0x5A)


def test_cpu_entry_wrong_output_size(eng, oracle_mod):
    case = _CONFIG[-2]
    f, t, osz = _encode(oracle_mod, case)[0]
    check(eng, oracle_mod, case, [f, f, f], [osz - 4, osz + 4, 0])


@pytest.mark.parametrize("nthreads", [1, 3, 16, 64])
def test_cpu_entry_range_threads(eng, oracle_mod, nthreads):
    """Fewer tiles than threads: each tile's chunks split over range threads
    (compute_chunk_min_max); the outputs are the same at any thread count."""
    case = next(c for c in _EDGE if c.name == "multichunk_c5_small_chunks")
    enc = _encode(oracle_mod, case)
    check(eng, oracle_mod, case, [e[0] for e in enc] * 2, [e[2] for e in enc] * 2, nthreads=nthreads)


def test_cpu_entry_concurrent_callers(eng, oracle_mod):
    """Two host threads in the C-ABI at once (the reference is re-entrant,
    reader_base.cc:929-934)."""
    cases = [_CONFIG[0], _CONFIG[-1]]
    errs = []

    def run(case):
        try:
            enc = _encode(oracle_mod, case)
            for _ in range(5):
                check(eng, oracle_mod, case, [e[0] for e in enc], [e[2] for e in enc], nthreads=3)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(c,)) for c in cases]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


def test_cpu_entry_rejects_unsupported(eng):
    from tiledb_amd.engine import EngineError
    from tiledb_amd.filter_pipeline import CompressionFilter, Compressor, Datatype, FilterPipeline
    ser = FilterPipeline(65536, [CompressionFilter(Compressor.GZIP, 6)]).serialize()
    dp = eng.DevicePipeline(ser, 23, int(Datatype.INT32), 4)
    x = np.zeros(64, dtype=np.uint8)
    with pytest.raises(EngineError) as ei:
        eng.unfilter_cpu(dp, np.array([x.ctypes.data], np.uint64), np.array([64], np.uint64),
                         np.array([x.ctypes.data], np.uint64), np.array([64], np.uint64))
    assert ei.value.code == 10
