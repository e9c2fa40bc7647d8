#!/usr/bin/env python3
"""Benchmark: device-resident unfilter of the BASELINE 3-stage pipeline.

Workload (BASELINE.json configs[4]): dense int32 tiles of
64 KiB (one chunk each), pipeline [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION(256)],
the config's 100,000 tiles sharded over the N GPUs (strong scaling: at N = 1
all 100,000 are resident on the one GPU, at N = 8 each GPU holds 12,500).
The other configs run with --config c1|c2|c2i|c3a|c3b|c4 (one JSON line each).
A step is one unfilter pass (one tdbg_unfilter_tiles_async launch) over the
rank's resident tiles, packed back to back in HBM at arbitrary byte offsets
(as FilteredData hands them over, filtered_data.h:100-101).

Three data variants: "rand" (DD and BWR raw: two stages are views) and
"ramp" (DD raw) are SURVEY's; "active" makes all three stages work
(DoubleDelta bit-packed, BWR windows 8-bit, byteshuffle).  `value` is the
minimum over the three.  Every timed launch's statuses and every output tile
are checked after the timed region.

Run:  python bench.py [--gpus N --steps K --warmup W]
      torchrun --nproc-per-node N bench.py --gpus N   (one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

# BASELINE.json configs; per-GPU tile counts at the GPU
# counts the configs name (weak scaling: the same per-GPU work at any N)
CONFIGS = {
    "c1": dict(tiles_per_gpu=256, variants="ramp,rand", dtype="int32",
               workload="C1: 2D int32 dense, [BYTESHUFFLE], 256 tiles x 64 KiB"),
    "c2": dict(tiles_per_gpu=10000, variants="sin", dtype="float32",
               workload="C2: dense float32, [BITSHUFFLE, BIT_WIDTH_REDUCTION(256)] (BWR pass-through "
                        "on float), 10k tiles x 64 KiB"),
    "c2i": dict(tiles_per_gpu=10000, variants="sin", dtype="int32",
                workload="C2i: C2's bytes typed INT32 (BWR active), 10k tiles x 64 KiB"),
    "c3a": dict(tiles_per_gpu=10000, variants="coords", dtype="uint64",
                workload="C3a: sparse uint64 coords, [DOUBLE_DELTA], 10k tiles x 64 KiB"),
    "c3b": dict(tiles_per_gpu=10000, variants="coords", dtype="uint64",
                workload="C3b: sparse uint64 coords, [RLE] (cell 8), 10k tiles x 64 KiB"),
    "c4": dict(tiles_per_gpu=12500, variants="offsets", dtype="uint64",
               workload="C4: var-length offsets uint64, [POSITIVE_DELTA(1024), BIT_WIDTH_REDUCTION(256)], "
                        "50k tiles / 4 GPUs"),
    # the metric's config: 100,000 tiles in all, sharded over the N GPUs
    # (strong scaling; at N = 1 the whole config is resident on the one GPU)
    "c5": dict(tiles_per_gpu=12500, total_tiles=100000, variants="active,rand,ramp", dtype="int32",
               workload="C5: dense int32, [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION(256)], "
                        "64 KiB tiles (1 chunk), device-resident, 100k tiles sharded over the GPUs"),
    "c5s": dict(tiles_per_gpu=163840, variants="active,rand,ramp", dtype="int32",
                workload="C5 pipeline on 40,000-B tiles (10,000 int32 values, one chunk), 163,840 tiles "
                         "per GPU (the c5 leg's 6.55 GB of output)"),
    "c5big": dict(tiles_per_gpu=512, variants="active,rand,ramp", dtype="int32", unique=12,
                  workload="C5 pipeline, 4 MiB tiles (64 chunks of 64 KiB), 512 tiles per GPU: tile mode "
                           "(TDBG_MULTI_CHUNK: one workgroup walks a tile's chunks)"),
    # XOR / DELTA / FLOAT_SCALE pipelines (not BASELINE configs; tiles encoded
    # on the device by tdbg_filter_tiles, checked against the values)
    "xor": dict(tiles_per_gpu=10000, variants="sin", dtype="float32",
                workload="XOR: dense float32, [XOR, BIT_WIDTH_REDUCTION(256)], 10k tiles x 64 KiB"),
    "delta": dict(tiles_per_gpu=12500, variants="active", dtype="int32",
                  workload="DELTA: C5's values, [BYTESHUFFLE, DELTA, BIT_WIDTH_REDUCTION(256)], "
                           "12.5k tiles x 64 KiB"),
    "fscale": dict(tiles_per_gpu=10000, variants="sin", dtype="float64",
                   workload="FLOAT_SCALE: dense float64, [FLOAT_SCALE(1e-3, 0, 4 B), "
                            "BIT_WIDTH_REDUCTION(256)], 10k tiles x 64 KiB"),
}


def build_batch(engine, cfg: str, variant: str, ntiles: int, nunique: int, device: int, seed: int,
                align: int = 1, ctx=None, dp=None, use_arena: bool = True):
    """(use_arena: the batch lives on the run's one device arena -- so only
    one such batch may be alive at a time; c3_combined keeps two)"""
    import workloads as W

    def encode(vals):
        st, tiles = ctx.filter(dp, vals)
        if st.any():
            raise SystemExit(f"{cfg}: device forward encode failed: {np.unique(st)}")
        return [t.tobytes() for t in tiles]

    pool, vals = W.pool(cfg, variant, min(nunique, CONFIGS.get(cfg, {}).get("unique", nunique)), seed,
                        encode=encode)
    nunique = len(vals)
    vals = [W.expected(cfg, v) for v in vals]
    idx = np.arange(ntiles) % nunique
    sizes = np.array([len(pool[i]) for i in idx], dtype=np.uint64)
    offs = engine.pack_offsets(sizes, align)
    total = int(offs[-1] + sizes[-1])
    pool_np = [np.frombuffer(p, dtype=np.uint8) for p in pool]
    if ntiles > nunique:
        # tile k sits at (k // nunique) * period + offs[k % nunique]: pack one
        # period of the unique tiles, then repeat it
        period = int(offs[nunique])
        blk = np.zeros(period, dtype=np.uint8)
        for i in range(nunique):
            blk[int(offs[i]):int(offs[i]) + pool_np[i].size] = pool_np[i]
        packed = np.tile(blk, -(-total // period))[:total]
        assert int(offs[-1]) == (ntiles - 1) // nunique * period + int(offs[(ntiles - 1) % nunique])
    else:
        packed = np.zeros(total, dtype=np.uint8)
        for i, o in zip(idx, offs):
            packed[int(o):int(o) + pool_np[i].size] = pool_np[i]
    out_sizes = [vals[i].nbytes for i in idx]
    batch = engine.TileBatch.from_packed(packed, offs, sizes, out_sizes, device=device,
                                         arena=(bench_arena(engine, packed.size, int(sum(out_sizes)), device)
                                                if use_arena else None),
                                         in_first=bool(int(os.environ.get("TDBG_BENCH_IN_FIRST", "0"))),
                                         gap=int(os.environ.get("TDBG_BENCH_GAP", "0")))
    return batch, pool, vals, idx, packed, offs, sizes


_ARENA = None


def bench_arena(engine, in_bytes: int, out_bytes: int, device: int):
    """One device arena for every timed batch of the run (outputs first, the
    filtered tiles after them): each leg's tiles sit on the same device pages
    whatever ran before.  With a fresh allocation per leg, a variant's rate
    depended on the legs before it (C5 ramp 0.667 first vs 0.693 after rand,
    rand 0.734 first vs 0.775 after ramp, same kernel and tiles) while the
    address-translation misses (~1e3 per launch) and the DRAM read requests
    stayed the same (profiles/r05/order_pmc.txt): the buffers' physical
    placement, not the TLB.  Grown (reallocated) only when a bigger batch
    comes; the default run's first batch (C5, 100,000 tiles) is the biggest."""
    global _ARENA
    import torch
    need = engine.TileBatch.arena_bytes(in_bytes, out_bytes) + int(os.environ.get("TDBG_BENCH_GAP", "0"))
    if _ARENA is None or _ARENA.numel() < need or _ARENA.device.index != device:
        _ARENA = None
        torch.cuda.empty_cache()
        _ARENA = torch.empty(need, dtype=torch.uint8, device=torch.device("cuda", device))
    return _ARENA


def verify(batch, vals, idx) -> None:
    """Every output tile equals its source values (compared on the device)."""
    import torch
    nb = int(vals[0].nbytes)
    if any(int(v.nbytes) != nb for v in vals) or (batch.out_size != nb).any():
        raise SystemExit("bench verification assumes equal tile sizes")
    uniq = torch.from_numpy(np.stack([v.view(np.uint8) for v in vals])).to(batch.d_out.device)
    got = batch.d_out[: batch.ntiles * nb].view(batch.ntiles, nb)
    exp_idx = torch.from_numpy(np.asarray(idx, dtype=np.int64)).to(batch.d_out.device)
    bad = (got != uniq[exp_idx]).any(dim=1)
    if bool(bad.any()):
        t = int(torch.nonzero(bad)[0])
        raise SystemExit(f"bench verification failed: tile {t} differs from its source values")


def time_device(engine, ctx, dp, batch, steps: int, warmup: int, dist, world: int):
    """Wall time of `steps` unfilter launches (barrier + synchronize on both
    sides, max over ranks; nothing but the launches on the stream), then the
    same `steps` launches again with HIP events bound to their kernel
    dispatches (tdbg_context_time_launches): each launch's kernel time (the
    streaming + fused kernels) and kernel + fixup time.  The events stay out
    of the first pass because each one ends its dispatch with a system-scope
    release (an L2 write-back): ~7 us per launch, 2 % of a 12,500-tile C5
    step."""
    import torch
    stream = torch.cuda.current_stream()
    for _ in range(warmup):
        ctx.unfilter_async(dp, batch, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    st = batch.d_status[: batch.ntiles].cpu().numpy()
    if st.any():
        raise SystemExit(f"device status nonzero: {np.unique(st)}")
    fused0, fb0, _ = ctx.path_stats()
    s0 = ctx.stream_tiles()
    c0 = ctx.stream_chunks() + ctx.tile_chunks()
    batch.d_status.fill_(-1)

    def timed(events: bool) -> float:
        if events:
            ctx.time_launches(steps)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.unfilter_async(dp, batch, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        return time.perf_counter() - t0

    elapsed = timed(False)
    # after the timed region: every launch wrote status OK for every tile,
    # and the fast kernels took every tile of every timed launch
    st = batch.d_status[: batch.ntiles].cpu().numpy()
    if st.any():
        raise SystemExit(f"timed launches: device status nonzero: {np.unique(st)}")
    fused1, fb1, _ = ctx.path_stats()
    s1 = ctx.stream_tiles()
    c1 = ctx.stream_chunks() + ctx.tile_chunks()
    batch.d_status.fill_(-1)
    ev_elapsed = timed(True)
    kern_ms, total_ms = ctx.launch_times(steps)
    # (the event-bound pass, whose kernel times `roofline` reports, is checked
    # the same way)
    st = batch.d_status[: batch.ntiles].cpu().numpy()
    if st.any():
        raise SystemExit(f"event-timed launches: device status nonzero: {np.unique(st)}")
    if dist is not None:
        elapsed = max_over_ranks(dist, elapsed, DIST_DEV)
        ev_elapsed = max_over_ranks(dist, ev_elapsed, DIST_DEV)
    return (elapsed, float(np.mean(kern_ms)), float(np.mean(total_ms)), fused1 - fused0, fb1 - fb0, s1 - s0,
            c1 - c0, ev_elapsed)


def time_forward(engine, ctx, dp, vals, idx, pool, steps: int, warmup: int, dist):
    """Forward direction (tdbg_filter_tiles_async) over the same tiles'
    unfiltered values, device-resident: wall time of `steps` launches (barrier
    + synchronize on both sides, max over ranks) and the mean launch time from
    HIP events on the launch stream.  After the timed region every tile's
    statuses are OK and its filtered bytes equal the workload encoder's."""
    import torch
    fb = ctx.filter_batch(dp, [vals[i] for i in idx])
    stream = torch.cuda.current_stream()
    for _ in range(max(1, warmup)):
        ctx.filter_async(dp, fb, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    fb.d_status.fill_(-1)

    def timed(events: bool) -> float:  # (as time_device: the events in a second pass)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for a, b in ev:
            if events:
                a.record(stream)
            ctx.filter_async(dp, fb, stream=stream.cuda_stream)
            if events:
                b.record(stream)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        return time.perf_counter() - t0

    elapsed = timed(False)
    timed(True)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    st = fb.d_status[: fb.ntiles].cpu().numpy()
    if st.any():
        raise SystemExit(f"forward: device status nonzero: {np.unique(st)}")
    lens = fb.lengths()
    want = np.array([len(pool[i]) for i in idx], dtype=np.uint64)
    if not np.array_equal(lens, want):
        raise SystemExit("forward: filtered sizes differ from the encoder's")
    step = 1024
    for a in range(0, fb.ntiles, step):
        b = min(fb.ntiles, a + step)
        lo, hi = int(fb.out_off[a]), int(fb.out_off[b - 1] + lens[b - 1])
        host = fb.d_out[lo:hi].cpu().numpy()
        for k in range(a, b):
            o = int(fb.out_off[k]) - lo
            if host[o:o + int(lens[k])].tobytes() != bytes(pool[idx[k]]):
                raise SystemExit(f"forward: tile {k} differs from the encoder's filtered bytes")
    if dist is not None:
        elapsed = max_over_ranks(dist, elapsed, DIST_DEV)
    b_alg = float(fb.in_size.sum() + lens.sum())
    return elapsed, kern_ms, b_alg, float(fb.in_size.sum())


# Collective device: "cuda" under RCCL; TDBG_DIST_BACKEND=gloo (a rehearsal of
# the multi-rank control flow with several ranks on one GPU) reduces on the CPU.
DIST_DEV = "cuda"


def max_over_ranks(dist, x: float, device: str) -> float:
    """The job's time is its slowest rank's (all_reduce MAX; tests run it on gloo)."""
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x: float, device: str) -> float:
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(engine, dp, packed, offs, sizes, out_bytes, ntiles_sample: int, threads: int,
                 min_seconds: float = 10.0):
    """The engine's CPU entry (tdbg_unfilter_tiles_cpu: C++ restatement of the
    reverse pipeline with the reference's tile x chunk-range thread split,
    reader_base.cc:929-989) on a bounded sample of the same tiles."""
    n = min(ntiles_sample, offs.size)
    out = np.zeros(n * out_bytes, dtype=np.uint8)
    in_ptrs = offs[:n] + np.uint64(packed.ctypes.data)
    out_ptrs = np.arange(n, dtype=np.uint64) * np.uint64(out_bytes) + np.uint64(out.ctypes.data)
    out_size = np.full(n, out_bytes, dtype=np.uint64)
    reps = 0
    t0 = time.perf_counter()
    while True:
        st = engine.unfilter_cpu(dp, in_ptrs, sizes[:n], out_ptrs, out_size, nthreads=threads)
        if st.any():
            raise SystemExit(f"cpu baseline failed: {np.unique(st)}")
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds:
            break
    gib = reps * n * out_bytes / 2**30
    return gib / el, reps * n, el


TRAFFIC_FILE = "profiles/pmc_traffic.json"


def load_traffic(cfg: str, variant: str, b_alg: float | None = None):
    """(HBM bytes per launch, source) for this launch from the committed
    rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes (tools/profile.sh): not
    measured in this run (PMC counters need their own rocprofv3 passes).

    A PMC pass is this launch's only when it ran the same workload at the same
    size: its algorithmic bytes equal `b_alg` (within 0.1 %).  Otherwise (a
    rank's shard at N > 1, a --tiles-per-gpu run) the pass's measured
    traffic / B_alg ratio is applied to this launch's B_alg and labelled
    "scaled"; with no pass of the workload at all, (None, None)."""
    path = os.path.join(ROOT, TRAFFIC_FILE)
    try:
        with open(path) as f:
            e = json.load(f).get(f"{cfg}_{variant}", {})
    except Exception:
        return None, None
    hbm, alg = e.get("hbm_bytes_per_launch"), e.get("algorithmic_bytes_per_launch")
    if hbm is None:
        return None, None
    if b_alg is None or not alg:
        return (hbm, "measured") if b_alg is None else (None, None)
    if abs(alg - b_alg) <= 1e-3 * b_alg:
        return int(hbm), "measured"
    return int(round(hbm / alg * b_alg)), f"scaled: {hbm / alg:.4f} x B_alg (PMC pass at {alg:.4g} B_alg)"


def run_config(engine, ctx, W, args, cfgname, variants, ntiles, steps, warmup, dist, world, rank,
               forward=False, e2e_leg=False, align=1):
    """Build and time one config's variants; returns (DevicePipeline, {variant: result})."""
    import torch
    ser, dt, cs, _, _ = W.config(cfgname)
    dp = engine.DevicePipeline(ser, 23, int(dt), cs)
    # timing-only ablations (outputs unchecked): TDBG_DEBUG_STOP (fused
    # kernel stages) or TDBG_BENCH_NOVERIFY (e.g. TDBG_RAW_ABL, TDBG_STREAM_STORE=3)
    ablation = bool(os.environ.get("TDBG_DEBUG_STOP") or os.environ.get("TDBG_BENCH_NOVERIFY"))
    res = {}
    for vi, var in enumerate(variants):
        batch, pool, vals, idx, packed, offs, sizes = build_batch(
            engine, cfgname, var, ntiles, args.unique, torch.cuda.current_device(),
            seed=5 + 1000 * rank + zlib.crc32(var.encode()) % 997,  # (by name: a --variants run sees the same tiles)
            align=align, ctx=ctx, dp=dp)
        st = ctx.unfilter(dp, batch)  # synchronous first pass (status + retry path)
        if st.any():
            raise SystemExit(f"{cfgname} {var}: first pass status nonzero: {np.unique(st)}")
        if not ablation:
            verify(batch, vals, idx)
        elapsed, kern_ms, launch_ms, fused, fallback, streamed, schunks, ev_elapsed = time_device(
            engine, ctx, dp, batch, steps, warmup, dist, world)
        if not ablation:
            verify(batch, vals, idx)
        unf = float(sum(vals[i].nbytes for i in idx))
        b_alg = float(sizes.sum()) + unf
        unf_job = sum_over_ranks(dist, unf, DIST_DEV) if dist is not None else unf
        res[var] = dict(elapsed=elapsed, ev_elapsed=ev_elapsed, kern_ms=kern_ms, launch_ms=launch_ms, b_alg=b_alg, unf=unf, unf_job=unf_job,
                        out_bytes=int(vals[0].nbytes), fused=fused, fallback=fallback, streamed=streamed,
                        stream_chunks=schunks,
                        packed=packed, offs=offs, sizes=sizes, steps=steps, ntiles=ntiles)
        if forward and vi == 0 and not ablation and cfgname != "fscale":  # (lossy: values differ)
            # (on at most one GPU's shard of C5, 12,500 tiles: the forward leg
            # checks every filtered tile against the encoder's bytes on the host)
            try:
                res[var]["fwd"] = time_forward(engine, ctx, dp, vals, idx[: args.shard_tiles or ntiles], pool, steps,
                                               warmup, dist)
            except SystemExit as ex:
                if cfgname == args.config:
                    raise
                res[var]["fwd_error"] = str(ex)  # (other configs' legs: reported, not fatal)
        if e2e_leg:
            ne = min(ntiles, args.e2e_tiles) if args.e2e_tiles else ntiles
            res[var]["e2e"] = e2e(engine, ctx, dp, packed, offs[:ne], sizes[:ne], int(vals[0].nbytes), args, dist,
                                  world)
        del batch
        torch.cuda.empty_cache()
    return dp, res


def c3_combined(engine, ctx, W, args):
    """the literal [DOUBLE_DELTA, RLE] cannot be built (DESIGN
    7), so C3a [DOUBLE_DELTA] and C3b [RLE] run back to back on the same
    coordinates: one step = the C3a launch then the C3b launch on one stream,
    both batches resident.  Combined rate = both launches' unfiltered bytes /
    the step's wall time; frac = both launches' B_alg / their kernels' time
    (HIP events on the launch stream)."""
    import torch
    parts = []
    for c in ("c3a", "c3b"):
        ser, dt, cs, _, _ = W.config(c)
        dp = engine.DevicePipeline(ser, 23, int(dt), cs)
        batch, pool, vals, idx, packed, offs, sizes = build_batch(
            engine, c, "coords", CONFIGS[c]["tiles_per_gpu"], args.unique, torch.cuda.current_device(), seed=5,
            ctx=ctx, dp=dp, use_arena=False)
        if ctx.unfilter(dp, batch).any():
            raise SystemExit(f"{c}: first pass status nonzero")
        parts.append((c, dp, batch, vals, idx, float(sizes.sum()), float(sum(vals[i].nbytes for i in idx))))
    stream = torch.cuda.current_stream()
    for _ in range(max(1, args.warmup)):
        for _, dp, batch, *_ in parts:
            ctx.unfilter_async(dp, batch, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    for p_ in parts:
        p_[2].d_status.fill_(-1)

    def timed() -> float:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            for _, dp, batch, *_ in parts:
                ctx.unfilter_async(dp, batch, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    el = timed()  # wall time; then the same steps with HIP events (as time_device)
    ctx.time_launches(2 * args.steps)
    timed()
    kern_ms, _ = ctx.launch_times(2 * args.steps)
    for c, dp, batch, vals, idx, _, _ in parts:
        if batch.d_status[: batch.ntiles].cpu().numpy().any():
            raise SystemExit(f"{c}: timed launches: device status nonzero")
        verify(batch, vals, idx)
    unf = sum(p_[6] for p_ in parts)
    b_alg = sum(p_[5] + p_[6] for p_ in parts)
    k_ms = float(np.sum(kern_ms)) / args.steps
    return {"workload": "C3a [DOUBLE_DELTA] then C3b [RLE] on the same uint64 coordinates, back to back on one "
                        "stream (10,000 tiles each)",
            "GiBps": round(unf / (el / args.steps) / 2**30, 2), "ms_per_step": round(el / args.steps * 1e3, 4),
            "kernel_ms": round(k_ms, 4), "algorithmic_bytes_per_step": int(b_alg),
            "roofline_frac": round(b_alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def gibps(r, world):
    # unfiltered bytes of the whole job (every rank's shard) / max-over-ranks time
    return r.get("unf_job", r["unf"] * world) / (r["elapsed"] / r["steps"]) / 2**30


def frac(r):
    return r["b_alg"] / (r["kern_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS


def kernel_name(cfgname, r):
    if cfgname == "c5big" and r.get("stream_chunks"):
        return ("unfilter_c5tile_kernel<MC> (tile mode: one workgroup per tile walks its chunks; or the chunk "
                "directory's records) + unfilter_fused_kernel (queue of declined tiles)")
    if cfgname in ("c5", "c5s", "c5big") and r["streamed"]:
        return "unfilter_c5tile_kernel + unfilter_fused_kernel (queue of declined tiles)"
    if cfgname == "c1" and r["streamed"]:
        return "unfilter_shuffle4_kernel + unfilter_fused_kernel (queue of declined tiles)"
    if cfgname in ("c2", "c2i") and r["streamed"]:
        return "unfilter_c2tile_kernel + unfilter_fused_kernel (queue of declined tiles)"
    if cfgname in ("c3a", "c3b", "c4") and r["streamed"]:
        return "unfilter_stream_small_kernel + unfilter_fused_kernel (queue of declined tiles)"
    return "unfilter_fused_kernel"


def roofline(cfgname, var, r):
    achieved = r["b_alg"] / (r["kern_ms"] * 1e-3) / 1e9
    traffic, tsrc = load_traffic(cfgname, var, r["b_alg"])
    return {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_source": f"{TRAFFIC_FILE} ({tsrc})" if traffic else None,
        # kernel_ms: the launch's unfilter kernels on its stream, HIP events
        "kernel": kernel_name(cfgname, r),
        "kernel_ms": round(r["kern_ms"], 4),
        "launch_ms": round(r["launch_ms"], 4),
        "kernel_ms_source": "HIP events bound to the kernel dispatches (tdbg_launch.h), mean over a second pass of "
                            "the same timed launches; that pass's ms_per_step is ms_per_step_events",
        "ms_per_step_events": round(r["ev_elapsed"] / r["steps"] * 1e3, 4),
        "algorithmic_bytes_per_launch": int(r["b_alg"]),
    }


def variant_line(cfgname, var, r, world):
    return {"GiBps": round(gibps(r, world), 2), "roofline_frac": round(frac(r), 4),
            "kernel_ms": round(r["kern_ms"], 4), "ms_per_step": round(r["elapsed"] / r["steps"] * 1e3, 4),
            "ms_per_step_events": round(r["ev_elapsed"] / r["steps"] * 1e3, 4),
            "fallback_tiles_timed": r["fallback"], "stream_tiles_timed": r["streamed"],
            "stream_chunks_timed": r.get("stream_chunks", 0),
            "algorithmic_bytes_per_launch": int(r["b_alg"]),
            "traffic": load_traffic(cfgname, var, r["b_alg"])[0]}


def cgroup_cpus():
    """The process's CPU quota in CPUs (cgroup v2 cpu.max 'quota period'), or
    None when unlimited / unreadable.  On the GPU boxes the quota is what a
    job may use, not the CPUs in its affinity list."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except Exception:
        return None


def _cpulist(path):
    """'0-7,16,18-19' -> [0..7, 16, 18, 19]; None if unreadable."""
    try:
        out = []
        for part in open(path).read().strip().split(","):
            a, _, b = part.partition("-")
            out += list(range(int(a), int(b or a) + 1))
        return out
    except Exception:
        return None


def spread_cpus(threads):
    """`threads` physical cores of NUMA node 0 within this process's
    affinity, dealt round-robin over the node's L3 domains (CCDs), or None.
    On the GPU host (2 x EPYC 9575F, 8-core CCDs) the CPU entry's rate is
    bound by each CCD's memory link (8 threads on one CCD: 38.8 GiB/s, on
    two: 47.4, 16 threads over four: 51.4; profiles/r05/cpu_curve.txt), so
    the baseline spreads its threads."""
    aff = os.sched_getaffinity(0)
    node0 = _cpulist("/sys/devices/system/node/node0/cpulist") or sorted(aff)
    groups = {}
    for c in node0:
        if c not in aff:
            continue
        sib = _cpulist(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") or [c]
        if min(sib) != c:
            continue  # an SMT sibling
        l3 = _cpulist(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") or [0]
        groups.setdefault(min(l3), []).append(c)
    order, k = [], 0
    lists = [groups[g] for g in sorted(groups)]
    while len(order) < threads and any(k < len(g) for g in lists):
        order += [g[k] for g in lists if k < len(g)]
        k += 1
    return order[:threads] if len(order) >= threads else None


def cpu_timed(engine, dp, r, threads, ntiles_sample, seconds):
    """cpu_baseline with the threads on spread_cpus (the sample copied while
    pinned, so its pages sit on that node); the affinity is restored."""
    old = os.sched_getaffinity(0)
    cpus = spread_cpus(threads)
    try:
        packed = r["packed"]
        if cpus:
            os.sched_setaffinity(0, cpus)
            n = min(ntiles_sample, r["offs"].size)
            packed = packed[: int(r["offs"][n - 1] + r["sizes"][n - 1])].copy()
        v = cpu_baseline(engine, dp, packed, r["offs"], r["sizes"], r["out_bytes"], ntiles_sample, threads, seconds)
    finally:
        os.sched_setaffinity(0, old)
    return v, cpus


def cpu_line(engine, dp, r, cfgname, var, threads, seconds, ntiles_sample=2048, scaling=False):
    (cpu, ntl, el), cpus = cpu_timed(engine, dp, r, threads, ntiles_sample, seconds)
    line = {
        "value": round(cpu, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{ntl} {cfgname.upper()} '{var}' tiles ({min(ntiles_sample, r['offs'].size)}-tile sample, "
                  f"repeated) in {el:.2f}s on {threads} threads of '{cpu_model()}' ({os.cpu_count()} CPUs "
                  f"visible, {len(os.sched_getaffinity(0))} in this process's affinity, cgroup quota "
                  f"{cgroup_cpus() or 'none'} CPUs: the threads used = the quota, every core the job may use), "
                  "tdbg_unfilter_tiles_cpu (the C-ABI's C++ CPU entry, the reference's tile x chunk-range split)",
        "cgroup_cpu_quota": cgroup_cpus(),
        "thread_placement": (f"pinned to physical cores {cpus} of NUMA node 0, round-robin over its L3 domains "
                             "(sample pages first-touched there)") if cpus else "unpinned",
    }
    if scaling:
        # per-thread rate and the thread-scaling curve of the same sample, so
        # the all-cores figure can be read off (the box lends a GPU job 16
        # threads; running on all of them is not allowed there)
        curve = {}
        for t in (1, 2, 4, 8, 12):
            if t < threads:
                (v, _, _), _ = cpu_timed(engine, dp, r, t, min(ntiles_sample, 256 * t), max(1.0, seconds / 5))
                curve[str(t)] = round(v, 3)
        curve[str(threads)] = round(cpu, 3)
        line["thread_scaling_GiBps"] = curve
        if "1" in curve:
            ncpu = os.cpu_count() or threads
            line["per_thread_GiBps"] = curve["1"]
            line["all_cores_linear_estimate_GiBps"] = {
                "cores": ncpu, "value": round(min(curve["1"] * ncpu, cpu * ncpu / threads), 1),
                "note": "not measured: min(1-thread rate x cores, measured rate x cores / threads); "
                        "memory bandwidth would cap it lower"}
    return line


# the other BASELINE configs timed in the default (N = 1) run, per-GPU sizes
OTHER_CONFIGS = ("c1", "c2", "c2i", "c3a", "c3b", "c4")


FORWARD_KERNEL = {
    "c5": "filter_c5tile_kernel (tdbg_forward_stream.hip, one 1,024-thread workgroup per tile) + filter_tiles_kernel on its queue",
    "c3a": "filter_small_kernel<0> (tdbg_forward_small.hip) + filter_tiles_kernel on its queue",
    "c3b": "filter_small_kernel<1> (tdbg_forward_small.hip) + filter_tiles_kernel on its queue",
    "c4": "filter_small_kernel<2> (tdbg_forward_small.hip) + filter_tiles_kernel on its queue",
    "c1": "filter_shuffle4_kernel<0> (tdbg_forward_shuffle.hip) + filter_tiles_kernel on its queue",
    "c2": "filter_shuffle4_kernel<1> (tdbg_forward_shuffle.hip) + filter_tiles_kernel on its queue",
    "c2i": "filter_shuffle4_kernel<2> (tdbg_forward_shuffle.hip) + filter_tiles_kernel on its queue",
}


def forward_line(cfgname, variants, res, world):
    """The forward (filter) leg of a config's first variant, if it ran."""
    fv = variants[0]
    if "fwd_error" in res[fv]:
        return {"variant": fv, "error": res[fv]["fwd_error"]}
    if "fwd" not in res[fv]:
        return None
    r = res[fv]
    el, fk, fb_alg, fin = r["fwd"]
    return {
        "metric": "GiB/s unfiltered tile bytes filtered (device-resident), same tiles and pipeline",
        "variant": fv,
        "tiles_per_gpu": int(round(fin / r["out_bytes"])),
        "value": round(fin * world / (el / r["steps"]) / 2**30, 2),
        "unit": "GiB/s",
        "ms_per_step": round(el / r["steps"] * 1e3, 4),
        "kernel": FORWARD_KERNEL.get(cfgname, "filter_tiles_kernel (general forward kernel)"),
        "kernel_ms": round(fk, 4),
        "algorithmic_bytes_per_launch": int(fb_alg),
        "roofline_frac": round(fb_alg / (fk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
    }


def headline_line(args, W, variants, res, world):
    """The JSON line of the bench's config: `value` is the slowest variant
    (SURVEY 8(d) defines C5's 'ramp' and 'rand'; 'active' makes all three
    stages work), so the headline is a floor over the data variants."""
    cfg = CONFIGS[args.config]
    head = min(variants, key=lambda v: gibps(res[v], world))
    r = res[head]
    line = {
        "metric": "GiB/s unfiltered tile bytes (device-resident), 64 KiB chunks, 3-stage pipeline",
        "value": round(gibps(r, world), 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": r["steps"],
        "warmup": args.warmup,
        "ms_per_step": round(r["elapsed"] / r["steps"] * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if "total_tiles" in cfg and not args.tiles_per_gpu else "weak",
        "vs_baseline": None,
        "dtype": cfg["dtype"],
        "data": f"synthetic {args.config.upper()} tiles, variants {','.join(variants)} ({args.unique} unique each, "
                "replicated), " + ("device-encoded (tdbg_filter_tiles)" if W.config(args.config)[4] is None
                                   else "numpy-encoded (workloads.py)"),
        "config": {
            "workload": cfg["workload"],
            "tiles_per_gpu": r["ntiles"],
            "variant": head if len(variants) == 1 else f"min over {','.join(variants)} = '{head}'",
            "tile_alignment": args.align,
            "parallelism": f"tile-shard x{world} (no collectives)",
            "filtered_bytes_per_gpu": int(r["sizes"].sum()),
            "fused_tiles_timed": r["fused"],
            "fallback_tiles_timed": r["fallback"],
            "stream_tiles_timed": r["streamed"],
            "stream_chunks_timed": r.get("stream_chunks", 0),
        },
        "roofline": roofline(args.config, head, r),
    }
    line["config"]["variants"] = {v: variant_line(args.config, v, res[v], world) for v in variants}
    line["config"]["min_over_variants_GiBps"] = round(min(gibps(res[v], world) for v in variants), 2)
    line["config"]["min_over_variants_roofline_frac"] = round(min(frac(res[v]) for v in variants), 4)
    fl = forward_line(args.config, variants, res, world)
    if fl:
        line["forward"] = fl
    if all("e2e" in res[v] for v in variants):
        line["config"]["e2e_GiBps"] = {v: res[v]["e2e"] for v in variants}
        line["config"]["e2e_note"] = ("pinned host tiles -> H2D -> unfilter -> D2H into a pinned result buffer, "
                                      "TDBG_HOST_CONTIGUOUS_INPUT|OUTPUT (one FilteredData-style block each way), "
                                      f"{args.e2e_batch_mb} MiB batches; PCIe-bound, never `value`")
    return line


def dense_var_leg(engine, ctx, steps: int, tiles_side: int = 32, seed: int = 9, pinned: bool = False):
    """The step after the path for a var-sized attribute (SURVEY 8(f) 4,
    dense_reader.cc:1555-2007): tdbg_dense_read_var_host from host FILTERED
    offsets tiles ([POSITIVE_DELTA(1024), BWR(256)] on uint64) and var tiles
    ([BITSHUFFLE] on uint8) -> H2D -> unfilter (offsets with the extra offset)
    -> cell sizes -> device scan -> byte gather -> D2H of the result offsets
    and bytes.  One fragment over a tiles_side^2 grid of 64 x 128-cell space
    tiles (8,192 cells of U{0..32} bytes each), subarray = the array, row
    major; 16 unique tile pairs (encoded on the device by tdbg_filter_tiles),
    replicated into one host block.  Rate = result bytes (offsets + var
    bytes) / wall time per call; host buffers are pageable, as a reader's
    would be."""
    from tiledb_amd.filter_pipeline import (BitshuffleFilter, BitWidthReductionFilter, Datatype,
                                            FilterPipeline, PositiveDeltaFilter)
    rng = np.random.default_rng(seed)
    ext = (64, 128)
    nct = ext[0] * ext[1]
    offp = FilterPipeline(65536, [PositiveDeltaFilter(1024), BitWidthReductionFilter(256)]).serialize()
    varp = FilterPipeline(65536, [BitshuffleFilter()]).serialize()
    dpo = engine.DevicePipeline(offp, 23, int(Datatype.UINT64), 8)
    dpv = engine.DevicePipeline(varp, 23, int(Datatype.UINT8), 1)
    offs_w, vars_ = [], []
    for _ in range(16):
        lens = rng.integers(0, 33, nct)
        o = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        offs_w.append(o[:-1].copy())
        vars_.append(rng.integers(0, 256, int(o[-1]), dtype=np.uint8))
    st1, fo = ctx.filter(dpo, [x.view(np.uint8) for x in offs_w])
    st2, fv = ctx.filter(dpv, vars_)
    if st1.any() or st2.any():
        raise SystemExit("dense var leg: device encode failed")
    nt = tiles_side * tiles_side
    starts = np.array([(r * ext[0], c * ext[1]) for r in range(tiles_side) for c in range(tiles_side)], dtype=np.int64)
    hi = (tiles_side * ext[0] - 1, tiles_side * ext[1] - 1)
    idx = [t % 16 for t in range(nt)]
    # the filtered tiles back to back in one host block, [offsets tile, var
    # tile] per space tile, as a FilteredData block holds a batch's reads
    import torch
    sz = [(len(fo[i]), len(fv[i])) for i in idx]
    hbytes = lambda nb: (torch.empty(nb, dtype=torch.uint8, pin_memory=True).numpy() if pinned  # noqa: E731
                         else np.empty(nb, dtype=np.uint8))
    blk = hbytes(sum(a + b for a, b in sz))
    off_f, var_f, o = [], [], 0
    for i, (a, b) in zip(idx, sz):
        blk[o:o + a] = fo[i]
        off_f.append(blk[o:o + a])
        blk[o + a:o + a + b] = fv[i]
        var_f.append(blk[o + a:o + a + b])
        o += a + b
    var_u = [vars_[i].size for i in idx]
    fc = engine.dense_frag_config(8, ext, (0, 0), hi, 1, 1, 0, 0)
    dom = np.array([[0, hi[0], 0, hi[1]]], dtype=np.int64)
    cap = sum(var_u) + 64
    ro_buf = hbytes(nt * nct * 8).view(np.uint64)
    rv_buf = hbytes(cap)
    call = lambda: engine.dense_read_var_host(ctx, dpo, dpv, fc, starts, dom, off_f, var_f, var_u, b"\0", cap,  # noqa: E731
                                              out_offsets=ro_buf, out_var=rv_buf)
    rc, ro, rv, st = call()
    rv = bytes(rv)
    if rc or st.any() or len(rv) != sum(var_u):
        raise SystemExit(f"dense var leg failed: rc {rc}")
    # (the result's first cell row -- row 0 of every tile of the first tile
    # row -- must be those cells' source bytes)
    row0 = b"".join(vars_[idx[c]][: int(offs_w[idx[c]][ext[1]])].tobytes() for c in range(tiles_side))
    if not rv.startswith(row0) or int(ro[1]) != int(offs_w[idx[0]][1]):
        raise SystemExit("dense var leg: result bytes differ from the source cells")
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
    el = (time.perf_counter() - t0) / steps
    res_bytes = nt * nct * 8 + len(rv)
    return {"workload": f"dense var-sized attribute, 1 fragment, {nt} space tiles of 64 x 128 cells "
                        f"(U{{0..32}} B each), offsets [PD(1024), BWR(256)] uint64 + var [BITSHUFFLE] uint8, "
                        "host filtered tiles -> result offsets + bytes on the host",
            "entry": "tdbg_dense_read_var_host", "steps": steps,
            "host_buffers": "pinned" if pinned else "pageable",
            "result_bytes": res_bytes, "filtered_bytes": int(sum(len(x) for x in off_f) + sum(len(x) for x in var_f)),
            "ms_per_call": round(el * 1e3, 3), "GiBps_result": round(res_bytes / el / 2**30, 2)}


def compact_line(line: dict, legs_file) -> dict:
    """The headline JSON the driver parses: the contract's fields, the
    headline roofline and cpu_baseline, and one GiB/s + roofline fraction per
    variant and per other leg.  Every leg's detail (kernel names, event
    times, CPU curves, dense var leg, ...) is in the full line / `legs_file`."""
    c = line["config"]
    rf = line["roofline"]
    out = {k: line[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    tr = lambda v: (round(v["traffic"] / v["algorithmic_bytes_per_launch"], 4)  # noqa: E731
                    if v.get("traffic") else None)
    cc = {"workload": c["workload"], "tiles_per_gpu": c["tiles_per_gpu"], "variant": c["variant"],
          "parallelism": c["parallelism"], "fallback_tiles_timed": c["fallback_tiles_timed"],
          "variants": {v: {"GiBps": x["GiBps"], "roofline_frac": x["roofline_frac"], "kernel_ms": x["kernel_ms"],
                           "ms_per_step": x["ms_per_step"], "traffic_over_alg": tr(x)}
                       for v, x in c["variants"].items()},
          "min_over_variants_roofline_frac": c["min_over_variants_roofline_frac"]}
    if "forward" in line:
        f = line["forward"]
        cc["forward"] = {"GiBps": f.get("value"), "roofline_frac": f.get("roofline_frac"), "tiles": f.get("tiles_per_gpu")}
    if "e2e_GiBps" in c:
        cc["e2e_GiBps_pcie_inclusive"] = c["e2e_GiBps"]
    if "other_configs" in c:
        oc = {}
        for k, o in c["other_configs"].items():
            e = {"GiBps": o["value_GiBps"], "roofline_frac": o["roofline"]["frac"],
                 "traffic_over_alg": (round(o["roofline"]["traffic"] / o["roofline"]["algorithmic_bytes_per_launch"], 4)
                                      if o["roofline"].get("traffic") else None)}
            if isinstance(o.get("forward"), dict) and "roofline_frac" in o["forward"]:
                e["forward_frac"] = o["forward"]["roofline_frac"]
            if "cpu_baseline" in o:
                e["cpu_GiBps"] = o["cpu_baseline"]["value"]
            oc[k] = e
        cc["other_configs"] = oc
    if "c3_combined" in c:
        cc["c3_combined"] = {k: c["c3_combined"][k] for k in ("GiBps", "roofline_frac")}
    for leg in ("c5_shard_12500", "c5_40000B_tiles", "c5_4MiB_tiles", "c5_dense_codes"):
        if leg in c:
            cc[leg] = {v: {"GiBps": x["GiBps"], "roofline_frac": x["roofline_frac"],
                           "ms_per_step": x["ms_per_step"], "kernel_ms": x["kernel_ms"]}
                       for v, x in c[leg]["variants"].items()}
    cc["legs_file"] = legs_file or "(the line before this one)"
    out["config"] = cc
    out["roofline"] = {k: rf[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_source",
                                           "kernel", "kernel_ms", "algorithmic_bytes_per_launch")}
    if "cpu_baseline" in line:
        cb = line["cpu_baseline"]
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample") if k in cb}
        if "per_thread_GiBps" in cb:
            out["cpu_baseline"]["per_thread_GiBps"] = cb["per_thread_GiBps"]
    return out


def init_dist(dist_mod, torch, env, local: int) -> str:
    """One process per GPU: RCCL ('nccl') bound to the rank's own device
    (init_process_group(device_id=cuda:local)), or the gloo rehearsal
    (TDBG_DIST_BACKEND=gloo) with ranks sharing the box's GPUs round-robin.
    Returns the device the max-over-ranks reduction runs on."""
    be, dev = dist_backend(env, local, torch.cuda.device_count())
    if dev is None:
        torch.cuda.set_device(local)
        dist_mod.init_process_group(be, device_id=torch.device("cuda", local))
        return "cuda"
    torch.cuda.set_device(dev)
    dist_mod.init_process_group(be)
    return "cpu"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c5", choices=sorted(CONFIGS),
                    help="BASELINE config (default C5, the metric's 3-stage pipeline)")
    ap.add_argument("--tiles-per-gpu", type=int, default=0,
                    help="default: the config's per-GPU tile count (C5: its 100,000 tiles / N)")
    ap.add_argument("--unique", type=int, default=128)
    ap.add_argument("--variants", default="")
    ap.add_argument("--align", type=int, default=1,
                    help="tile start alignment in HBM (1 = back to back, as on disk)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-seconds-other", type=float, default=2.0,
                    help="CPU baseline sample time per other config")
    ap.add_argument("--e2e", action="store_true", default=True,
                    help="also time host-resident end-to-end (default on; every rank, "
                         "total over ranks / max-over-ranks time)")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false")
    ap.add_argument("--forward", action="store_true", default=True,
                    help="also time the forward (filter) direction on the first variant (default on)")
    ap.add_argument("--no-forward", dest="forward", action="store_false")
    ap.add_argument("--e2e-tiles", type=int, default=25000,
                    help="host E2E leg on the first N tiles of the rank's shard (0 = all; PCIe-bound)")
    ap.add_argument("--e2e-batch-mb", type=int, default=64,
                    help="host E2E staging batch (MiB per side; 2 batches in flight)")
    ap.add_argument("--others", action="store_true", default=True,
                    help="N = 1 default C5 run: also time every other BASELINE config (config.other_configs) "
                         "and C5 at 100k tiles on the one GPU")
    ap.add_argument("--no-others", dest="others", action="store_false")
    ap.add_argument("--shard-tiles", type=int, default=12500,
                    help="N = 1 run: also time C5 on one GPU's shard of an 8-GPU node (100k / 8)")
    ap.add_argument("--c5s-tiles", type=int, default=CONFIGS["c5s"]["tiles_per_gpu"],
                    help="N = 1 run: also time the C5 pipeline on 40,000-B tiles (0 = skip)")
    ap.add_argument("--c5big-tiles", type=int, default=CONFIGS["c5big"]["tiles_per_gpu"],
                    help="N = 1 run: also time the C5 pipeline on 4 MiB tiles, tile mode (0 = skip)")
    ap.add_argument("--dense-tiles", type=int, default=100000,
                    help="C5 tiles of dense DoubleDelta codes (variant 'walk') for the c5_dense_codes leg (0: off)")
    ap.add_argument("--legs-file", default="gpurun_out/bench_legs.json",
                    help="every leg's full JSON (also printed on the line before the headline); '' = none")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        global DIST_DEV
        DIST_DEV = init_dist(dist_mod, torch, os.environ, local)
        dist = dist_mod
    else:
        torch.cuda.set_device(0)
    from tiledb_amd import engine
    import workloads as W

    cfg = CONFIGS[args.config]
    if args.tiles_per_gpu:
        ntiles = args.tiles_per_gpu
    elif "total_tiles" in cfg:
        # strong scaling: the config's tiles, sharded over the ranks (rank r
        # takes tiles [r * n, (r + 1) * n) of the job; the last may be short)
        per = -(-cfg["total_tiles"] // world)
        ntiles = max(1, min(per, cfg["total_tiles"] - rank * per))
    else:
        ntiles = cfg["tiles_per_gpu"]
    ctx = engine.Context(torch.cuda.current_device())  # this rank's GPU (set above)
    # the run's one device arena, sized up front for the config's biggest
    # variant (C5 rand: 68,003-B images + 64 KiB outputs per tile)
    tb = W.TILE_BYTES * (64 if args.config == "c5big" else 1)
    bench_arena(engine, int(ntiles * tb * 1.04), ntiles * tb, torch.cuda.current_device())
    variants = [v for v in (args.variants or cfg["variants"]).split(",") if v]
    dp, res = run_config(engine, ctx, W, args, args.config, variants, ntiles, args.steps, args.warmup, dist,
                         world, rank, forward=args.forward, e2e_leg=args.e2e, align=args.align)

    line = headline_line(args, W, variants, res, world)
    head = min(variants, key=lambda v: gibps(res[v], world))
    r = res[head]
    # every core the job may use: the cgroup quota (16 on the GPU boxes), not
    # the affinity list (the whole machine there)
    threads = args.cpu_threads or min(cgroup_cpus() or 16, len(os.sched_getaffinity(0)))
    if world == 1 and args.others and args.config == "c5" and not args.tiles_per_gpu:
        # every other BASELINE config at its per-GPU size, and C5 at 100k tiles
        others = {}
        for c in OTHER_CONFIGS:
            cc = CONFIGS[c]
            cvars = [v for v in cc["variants"].split(",") if v]
            cdp, cres = run_config(engine, ctx, W, args, c, cvars, cc["tiles_per_gpu"], args.steps, args.warmup,
                                   dist, world, rank, forward=args.forward)
            ch = min(cvars, key=lambda v: gibps(cres[v], world))
            o = {"workload": cc["workload"], "tiles_per_gpu": cc["tiles_per_gpu"], "dtype": cc["dtype"],
                 "value_GiBps": round(gibps(cres[ch], world), 2), "variant": ch,
                 "roofline": roofline(c, ch, cres[ch]),
                 "variants": {v: variant_line(c, v, cres[v], world) for v in cvars}}
            fl = forward_line(c, cvars, cres, world)
            if fl:
                o["forward"] = fl
            if not args.no_cpu_baseline:
                o["cpu_baseline"] = cpu_line(engine, cdp, cres[ch], c, ch, threads, args.cpu_seconds_other)
            if c == "c1":
                o["note"] = ("BASELINE names C1 a CPU-path config: cpu_baseline is that path (the C++ CPU entry); "
                             "the GPU line is the same tiles on the device")
            others[c] = o
            for v in cres:  # free the host copies
                cres[v].pop("packed", None)
        line["config"]["other_configs"] = others
        line["config"]["c3_combined"] = c3_combined(engine, ctx, W, args)
        # C5 on one GPU's shard of the 8-GPU config (12,500 tiles): the
        # per-GPU work of the N = 8 line
        if args.shard_tiles and args.shard_tiles != ntiles:
            sh = {}
            _, sres = run_config(engine, ctx, W, args, "c5", variants, args.shard_tiles, args.steps,
                                 args.warmup, dist, world, rank)
            for v in variants:
                sh[v] = variant_line("c5shard", v, sres[v], world)
                sres[v].pop("packed", None)
            line["config"]["c5_shard_12500"] = {
                "tiles": args.shard_tiles, "steps": args.steps, "variants": sh,
                "min_over_variants_GiBps": round(min(x["GiBps"] for x in sh.values()), 2),
                "min_over_variants_roofline_frac": round(min(x["roofline_frac"] for x in sh.values()), 4)}
        line["config"]["dense_read_var_host"] = {
            "pageable": dense_var_leg(engine, ctx, max(2, args.steps // 4)),
            "pinned": dense_var_leg(engine, ctx, max(2, args.steps // 4), pinned=True)}
        # the C5 pipeline on 40,000-B tiles (one chunk of 10,000 values: not
        # 64 KiB, byte planes not 16-B aligned), the same output bytes
        if args.c5s_tiles:
            ss = {}
            _, cres = run_config(engine, ctx, W, args, "c5s", variants, args.c5s_tiles, args.steps, args.warmup,
                                 dist, world, rank)
            for v in variants:
                ss[v] = variant_line("c5s", v, cres[v], world)
                cres[v].pop("packed", None)
            line["config"]["c5_40000B_tiles"] = {
                "workload": CONFIGS["c5s"]["workload"], "tiles": args.c5s_tiles, "steps": args.steps,
                "kernel": kernel_name("c5s", cres[variants[0]]), "variants": ss,
                "min_over_variants_GiBps": round(min(x["GiBps"] for x in ss.values()), 2),
                "min_over_variants_roofline_frac": round(min(x["roofline_frac"] for x in ss.values()), 4)}
        # the C5 pipeline on 4 MiB tiles (64 chunks each): the everyday shape
        # of dense tiles over 64 KiB (tile.cc:87-100), tile mode
        if args.c5big_tiles:
            sb = {}
            _, cres = run_config(engine, ctx, W, args, "c5big", variants, args.c5big_tiles, args.steps,
                                 args.warmup, dist, world, rank)
            for v in variants:
                sb[v] = variant_line("c5big", v, cres[v], world)
                sb[v]["chunks_taken_per_launch"] = cres[v]["stream_chunks"] // max(1, args.steps)
                cres[v].pop("packed", None)
            line["config"]["c5_4MiB_tiles"] = {
                "workload": CONFIGS["c5big"]["workload"], "tiles": args.c5big_tiles, "steps": args.steps,
                "kernel": kernel_name("c5big", cres[variants[0]]), "variants": sb,
                "min_over_variants_roofline_frac": round(min(x["roofline_frac"] for x in sb.values()), 4)}
        # the C5 pipeline with dense DoubleDelta codes (variant 'walk', not a
        # BASELINE variant): the coded path when no wave's codes are all zero
        # (the active tiles skip 11 of 16 waves' code extraction)
        if args.dense_tiles:
            _, dres = run_config(engine, ctx, W, args, "c5", ["walk"], args.dense_tiles, args.steps,
                                 args.warmup, dist, world, rank)
            dv = variant_line("c5", "walk", dres["walk"], world)
            dres["walk"].pop("packed", None)
            line["config"]["c5_dense_codes"] = {
                "workload": "C5 pipeline, 64 KiB tiles whose byteshuffled stream is a random walk (steps "
                            "U{-500..500}): DoubleDelta bit-packed at bitsize 10 with nonzero codes throughout, "
                            "BWR windows over DD's output raw (23,415 B filtered)",
                "tiles": args.dense_tiles, "steps": args.steps, "variants": {"walk": dv}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # after every timed region, at N = 1 only (the N > 1 lines divide the
        # same job over more GPUs; the CPU figure does not change with N)
        line["cpu_baseline"] = cpu_line(engine, dp, r, args.config, head, threads, args.cpu_seconds, scaling=True)
    if rank == 0:
        # every leg in full: a side file and an earlier stdout line; the last
        # line is the compact headline the driver parses (<= ~4 KB)
        full = json.dumps(line)
        legs = args.legs_file
        if legs:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(legs)), exist_ok=True)
                with open(legs, "w") as fh:
                    fh.write(full + "\n")
            except OSError:
                legs = None
        print(full)
        print(json.dumps(compact_line(line, legs)))
    if dist is not None:
        dist.destroy_process_group()


def dist_backend(env, local: int, ndev: int):
    """(backend, device for gloo or None): RCCL ('nccl') with each rank on
    its own GPU, or the gloo rehearsal (TDBG_DIST_BACKEND=gloo) where ranks
    may share the box's GPUs round-robin."""
    if env.get("TDBG_DIST_BACKEND", "nccl") == "gloo":
        return "gloo", local % max(1, ndev)
    return "nccl", None


def e2e(engine, ctx, dp, packed, offs, sizes, out_bytes, args, dist=None, world=1):
    """Host-resident end-to-end: pinned H2D + unfilter + D2H (PCIe-inclusive).
    Every rank moves its own tiles through its own GPU's link; the rate is the
    total over ranks / the slowest rank's time (not `value`: DESIGN.md).  The
    filtered tiles sit back to back in one pinned block (a FilteredData-style
    batch) and the results in one pinned result buffer."""
    import torch
    n = offs.size
    hin = torch.from_numpy(packed[: int(offs[-1] + sizes[-1])]).pin_memory()
    hout = torch.empty(n * out_bytes, dtype=torch.uint8).pin_memory()
    in_ptrs = offs + np.uint64(hin.data_ptr())
    out_ptrs = np.arange(n, dtype=np.uint64) * np.uint64(out_bytes) + np.uint64(hout.data_ptr())
    osz = np.full(n, out_bytes, dtype=np.uint64)
    bb = args.e2e_batch_mb << 20
    kw = dict(batch_bytes=bb, contiguous_input=True, contiguous_output=True)
    ctx.unfilter_host(dp, in_ptrs, sizes, out_ptrs, osz, **kw)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        st = ctx.unfilter_host(dp, in_ptrs, sizes, out_ptrs, osz, **kw)
    el = time.perf_counter() - t0
    assert not st.any()
    if dist is not None:
        el = max_over_ranks(dist, el, DIST_DEV)
    return round(world * reps * n * out_bytes / el / 2**30, 2)


if __name__ == "__main__":
    main()
