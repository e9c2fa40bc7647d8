"""Thread-scaling of the C++ CPU entry (tdbg_unfilter_tiles_cpu) on C5 rand
tiles, on the GPU host: where does the curve flatten, and why?  Unpinned at
1..32 threads (the job's cgroup quota is 16 CPUs), then 8 / 16 threads pinned
to cores of one NUMA node, with the sample's pages first-touched on that node.
usage: python tools/cpu_curve.py [seconds]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import workloads as W  # noqa: E402
from tiledb_amd import engine  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    ser, dt, cs, _, _ = W.config("c5")
    dp = engine.DevicePipeline(ser, 23, int(dt), cs)
    pool, vals = W.pool("c5", "rand", 128, seed=7)
    n = 2048
    idx = np.arange(n) % 128
    sizes = np.array([len(pool[i]) for i in idx], dtype=np.uint64)
    offs = engine.pack_offsets(sizes, 1)
    packed = np.zeros(int(offs[-1] + sizes[-1]), dtype=np.uint8)
    for k, i in enumerate(idx):
        packed[int(offs[k]):int(offs[k]) + len(pool[i])] = np.frombuffer(pool[i], dtype=np.uint8)
    print("cgroup quota CPUs:", bench.cgroup_cpus(), "affinity:", len(os.sched_getaffinity(0)),
          "os.cpu_count:", os.cpu_count(), flush=True)
    all_cpus = sorted(os.sched_getaffinity(0))
    res = {}
    for t in (1, 2, 4, 8, 12, 16, 24, 32):
        v, ntl, el = bench.cpu_baseline(engine, dp, packed, offs, sizes, 65536, n, t, secs)
        res[f"unpinned_{t}"] = round(v, 2)
        print(f"unpinned threads {t:3d}: {v:8.2f} GiB/s", flush=True)
    for t, cpus in ((8, list(range(0, 8))), (16, list(range(0, 16))), (16, list(range(0, 32, 2)))):
        os.sched_setaffinity(0, cpus)
        # the sample re-touched by a pinned thread (pages on that node)
        p2 = packed.copy()
        v, ntl, el = bench.cpu_baseline(engine, dp, p2, offs, sizes, 65536, n, t, secs)
        res[f"pinned_{t}_cpus{cpus[0]}-{cpus[-1]}"] = round(v, 2)
        print(f"pinned threads {t:3d} on CPUs {cpus[0]}..{cpus[-1]} ({len(cpus)}): {v:8.2f} GiB/s", flush=True)
        del p2
    os.sched_setaffinity(0, all_cpus)
    r = {"packed": packed, "offs": offs, "sizes": sizes, "out_bytes": 65536}
    for t in (4, 8, 16):
        (v, _, _), cpus = bench.cpu_timed(engine, dp, r, t, n, secs)
        res[f"spread_{t}"] = round(v, 2)
        print(f"spread threads {t:3d} on {cpus}: {v:8.2f} GiB/s", flush=True)
    print(res)


if __name__ == "__main__":
    main()
