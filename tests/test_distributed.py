"""World-size-2 CPU (gloo) rehearsal of the multi-GPU path.

The path shards: each rank unfilters a contiguous,
byte-balanced range of tiles (tdbg_shard_tiles) with no collective on the
data path; the only collectives are the bench's barrier and max-over-ranks
timing.  Here each rank unfilters its shard with the product's C++ CPU entry
(tdbg_unfilter_tiles_cpu, the same C-ABI the GPU ranks drive), checks every
tile against the generator's source values, and rank 0 verifies that the
gathered shards cover every tile exactly once.
"""
from __future__ import annotations

import argparse
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tiles():
    import workloads as W
    pool_r, vals_r = W.c5_pool("rand", 5, seed=11)
    pool_m, vals_m = W.c5_pool("ramp", 6, seed=12)
    tiles = pool_r + pool_m
    vals = vals_r + vals_m
    return tiles, vals


def _worker(rank: int, world: int, port: int, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import workloads as W
        from tiledb_amd import engine
        from tiledb_amd.engine import shard_tiles
        tiles, vals = _tiles()
        isz = np.array([len(t) for t in tiles], dtype=np.uint64)
        osz = np.full(len(tiles), W.TILE_BYTES, dtype=np.uint64)
        cuts = shard_tiles(isz, osz, world)
        lo, hi = int(cuts[rank]), int(cuts[rank + 1])
        dp = engine.DevicePipeline(W.c5_pipeline_bytes(), 23, 0, 4)
        bufs = [np.frombuffer(tiles[i], dtype=np.uint8).copy() for i in range(lo, hi)]
        outs = [np.zeros(W.TILE_BYTES, dtype=np.uint8) for _ in range(lo, hi)]
        t0 = time.perf_counter()
        st = engine.unfilter_cpu(dp, [b.ctypes.data for b in bufs], isz[lo:hi],
                                 [o.ctypes.data for o in outs], osz[lo:hi], nthreads=2)
        el = time.perf_counter() - t0
        assert not st.any()
        digests = np.zeros(len(tiles), dtype=np.int64)
        for k, i in enumerate(range(lo, hi)):
            assert np.array_equal(outs[k], vals[i].view(np.uint8))
            digests[i] = int(np.frombuffer(outs[k], dtype=np.uint32).astype(np.uint64).sum()) + 1
        t = torch.from_numpy(digests)
        dist.all_reduce(t)  # disjoint shards: the sum is a gather
        slow = bench.max_over_ranks(dist, float(rank + 1), "cpu")
        # the bench's N = 2 line, from this rank's shard timed on the CPU
        # entry (stand-in for the GPU timing): max-over-ranks time, total
        # bytes over ranks, roofline, and rank 0's cpu_baseline
        packed = np.concatenate(bufs)
        offs = np.concatenate([[0], np.cumsum(isz[lo:hi])[:-1]]).astype(np.uint64)
        elapsed = bench.max_over_ranks(dist, el, "cpu")
        r = dict(elapsed=elapsed, ev_elapsed=elapsed, kern_ms=el * 1e3, launch_ms=el * 1e3, b_alg=float(isz[lo:hi].sum() + osz[lo:hi].sum()),
                 unf=float(osz[lo:hi].sum()), unf_job=bench.sum_over_ranks(dist, float(osz[lo:hi].sum()), "cpu"),
                 out_bytes=W.TILE_BYTES, fused=hi - lo, fallback=0, streamed=hi - lo,
                 packed=packed, offs=offs, sizes=isz[lo:hi], steps=1, ntiles=hi - lo)
        args = argparse.Namespace(config="c5", warmup=0, unique=len(tiles), align=1, e2e_batch_mb=64,
                                  tiles_per_gpu=0)
        line = bench.headline_line(args, W, ["rand"], {"rand": r}, world)
        if rank == 0:
            # (bench.py times the CPU baseline at N = 1 only: here its line
            # builder on this rank's shard, beside the N = 2 line)
            cb = bench.cpu_line(engine, dp, r, "c5", "rand", 2, 0.2)
            q.put((t.numpy().tolist(), cuts.tolist(), slow, line, cb))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_cover_every_tile_once():
    import sys
    sys.path.insert(0, ROOT)
    from tiledb_amd import _native  # noqa: F401  (the ranks drive the library)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    digests, cuts, slow, line, cb = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    tiles, vals = _tiles()
    assert cuts[0] == 0 and cuts[-1] == len(tiles) and cuts[0] < cuts[1] < cuts[2]
    for i in range(len(tiles)):
        assert digests[i] == int(vals[i].view(np.uint32).astype(np.uint64).sum()) + 1
    assert slow == 2.0
    # the N = 2 line: whole-job value over both ranks, roofline; the CPU
    # baseline's line shape
    # C5's 100k tiles sharded over the ranks: strong scaling, the whole job's bytes
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["value"] > 0
    job = sum(len(v) * 4 for v in vals)
    assert abs(line["value"] - job / (line["ms_per_step"] * 1e-3) / 2**30) < 1e-3 * line["value"] + 0.01
    assert line["roofline"]["bound"] == "hbm" and 0 < line["roofline"]["frac"]
    assert "cpu_baseline" not in line
    # the rank's HBM traffic is its own shard's (the 100k-tile PMC pass's
    # traffic / B_alg ratio applied to this rank's B_alg), not the 100k figure
    rf = line["roofline"]
    assert rf["traffic"] and 0.99 < rf["traffic"] / rf["algorithmic_bytes_per_launch"] < 1.05
    assert "scaled" in rf["traffic_source"]
    # the last stdout line the driver parses stays compact
    import json
    import bench
    c = bench.compact_line(line, None)
    assert len(json.dumps(c)) < 6000
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "roofline"):
        assert k in c
    assert c["config"]["workload"] and c["config"]["tiles_per_gpu"] == line["config"]["tiles_per_gpu"]
    assert c["roofline"]["traffic"] == rf["traffic"]
    assert cb["kind"] == "port" and cb["cores"] == 2 and cb["value"] > 0 and cb["unit"] == "GiB/s"


class _FakeCuda:
    def __init__(self, n):
        self.n, self.dev = n, None

    def device_count(self):
        return self.n

    def set_device(self, d):
        self.dev = d


class _FakeTorch:
    def __init__(self, n):
        self.cuda = _FakeCuda(n)

    @staticmethod
    def device(kind, idx):
        return (kind, idx)


class _FakeDist:
    def __init__(self):
        self.calls = []

    def init_process_group(self, backend, **kw):
        self.calls.append((backend, kw))


def test_init_dist_binds_each_rank_to_its_gpu():
    """bench.py's RCCL path: one process per GPU, init_process_group('nccl',
    device_id=cuda:LOCAL_RANK) after set_device(LOCAL_RANK); the gloo
    rehearsal shares the box's GPUs round-robin and reduces on the CPU."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    d, t = _FakeDist(), _FakeTorch(8)
    assert bench.init_dist(d, t, {}, 5) == "cuda"
    assert t.cuda.dev == 5 and d.calls == [("nccl", {"device_id": ("cuda", 5)})]
    d, t = _FakeDist(), _FakeTorch(1)
    assert bench.init_dist(d, t, {"TDBG_DIST_BACKEND": "gloo"}, 3) == "cpu"
    assert t.cuda.dev == 0 and d.calls == [("gloo", {})]
