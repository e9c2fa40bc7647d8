"""Summary of tools/profile_all.sh: per (config, variant) the unfilter kernels'
(streaming kernels -- C5: the tile kernel -- + fused on their queue for C3/C4/C5, else fused) rocprofv3 kernel-trace average over the timed launches, per-launch HBM
traffic from the --pmc passes (KiB -> bytes; FETCH_SIZE doubled for gfx950
16-B/lane streaming reads, MI355X_MICROARCH.md "HBM"), the algorithmic bytes
and roofline fraction from the bench line of the same workload."""
import csv
import glob
import json
import os
import statistics
import sys

PEAK = 8000.0


KERNELS = ("unfilter_stream", "unfilter_c5tile", "unfilter_c2tile", "unfilter_shuffle4", "unfilter_fused_kernel")
STARTS = ("unfilter_stream_kernel", "unfilter_c5tile_kernel", "unfilter_c2tile_kernel", "unfilter_stream_small_kernel", "unfilter_shuffle4_kernel")


def _launches(items):
    """items: (order key, kernel name, value) of the unfilter kernels.  A launch
    is a streaming kernel (C5: coded then raw-DD; C3/C4: small-image) plus the
    fused kernel on its queue, or the fused kernel alone; values of one launch
    are summed."""
    out, open_stream = [], False
    for _, name, v in sorted(items):
        if any(k in name for k in STARTS):
            out.append(v)
            open_stream = True
        elif open_stream:
            out[-1] += v
            if "unfilter_fused_kernel" in name:
                open_stream = False
        else:
            out.append(v)
    return out


def pmc(d, counter):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in KERNELS) and r["Counter_Name"] == counter:
                k = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                name, v = per.get(k, (r["Kernel_Name"], 0.0))
                per[k] = (name, v + float(r["Counter_Value"]))
    return _launches([(k, n, v) for k, (n, v) in per.items()])


def trace(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if any(k in r["Kernel_Name"] for k in KERNELS)]
    return _launches([(int(r["Start_Timestamp"]), r["Kernel_Name"],
                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows])


def stats(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main(out):
    res = {}
    for log in sorted(glob.glob(os.path.join(out, "bench_*.log"))):
        cfg = os.path.basename(log)[6:-4]
        lines = [l for l in open(log) if l.startswith("{")]
        if not lines:
            continue
        # (the full line, not the compact one printed after it: its variants
        # carry their own algorithmic bytes)
        line = json.loads(max(lines, key=len))
        variants = line["config"].get("variants") or {line["config"]["variant"]: {}}
        for v in variants:
            key = f"{cfg}_{v}"
            e = {"bench_GiBps": variants[v].get("GiBps", line["value"]) if variants[v] else line["value"]}
            d = trace(os.path.join(out, f"trace_{cfg}_{v}"))
            if len(d) >= 24:
                timed = d[-20:]  # sync pass + warmup first, then the 20 timed launches
                e["rocprof_unfilter_kernels_avg_us"] = round(statistics.mean(timed), 2)
            f = pmc(os.path.join(out, f"pmc_{cfg}_{v}_FETCH_SIZE"), "FETCH_SIZE")
            w = pmc(os.path.join(out, f"pmc_{cfg}_{v}_WRITE_SIZE"), "WRITE_SIZE")
            if f and w:
                fk, wk = statistics.median(f), statistics.median(w)
                e.update({"fetch_size_kib_median": fk, "write_size_kib_median": wk,
                          "hbm_read_bytes_per_launch": int(2 * fk * 1024),
                          "hbm_write_bytes_per_launch": int(wk * 1024),
                          "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
                          "correction": "read = 2 x FETCH_SIZE (gfx950 16B/lane streaming read), KiB -> bytes"})
            res[key] = e
        for v in variants:
            h = f"{cfg}_{v}"
            b_alg = (variants[v] or {}).get("algorithmic_bytes_per_launch") or \
                line["roofline"]["algorithmic_bytes_per_launch"]
            res[h]["algorithmic_bytes_per_launch"] = b_alg
            if "rocprof_unfilter_kernels_avg_us" in res[h]:
                ach = b_alg / (res[h]["rocprof_unfilter_kernels_avg_us"] * 1e-6) / 1e9
                res[h]["rocprof_achieved_GBps"] = round(ach, 1)
                res[h]["rocprof_roofline_frac"] = round(ach / PEAK, 4)
            if "hbm_bytes_per_launch" in res[h]:
                res[h]["traffic_over_algorithmic"] = round(res[h]["hbm_bytes_per_launch"] / b_alg, 4)
        head = line["config"]["variant"]
        head = head.split("'")[1] if "'" in head else head  # "min over a,b = 'a'"
        res[f"{cfg}_{head}"]["bench_line"] = line
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
