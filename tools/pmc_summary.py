"""Per-launch HBM traffic of the fused unfilter kernel from rocprofv3 --pmc
passes (tools/profile.sh).  Corrections per MI355X_MICROARCH.md "HBM":
counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16 B/lane streaming stores.  Output: JSON keyed by data variant."""
import csv
import glob
import json
import os
import statistics
import sys


def per_launch(d: str, counter: str):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "unfilter_fused_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def trace_durations(out: str):
    """Fused-kernel durations (us) per variant from the --kernel-trace pass of
    the default bench command: per variant 1 synchronous + 3 warmup + 20
    timed launches, rand first then ramp; the timed ones are averaged."""
    rows = []
    for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "unfilter_fused_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    if len(d) != 48:
        return {}
    return {"rand": statistics.mean(d[4:24]), "ramp": statistics.mean(d[28:48])}


def main(out: str) -> None:
    res = {}
    tr = trace_durations(out)
    for v in ("rand", "ramp"):
        f = per_launch(os.path.join(out, f"pmc_{v}_FETCH_SIZE"), "FETCH_SIZE")
        w = per_launch(os.path.join(out, f"pmc_{v}_WRITE_SIZE"), "WRITE_SIZE")
        if not f or not w:
            continue
        fk, wk = statistics.median(f), statistics.median(w)
        res[v] = {
            "launches": [len(f), len(w)],
            "fetch_size_kib_median": fk,
            "write_size_kib_median": wk,
            "hbm_read_bytes_per_launch": int(2 * fk * 1024),
            "hbm_write_bytes_per_launch": int(wk * 1024),
            "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
            "correction": "read = 2 x FETCH_SIZE (gfx950 16B/lane streaming read), KiB -> bytes",
        }
        if v in tr:
            res[v]["rocprof_kernel_trace_avg_us"] = round(tr[v], 2)
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
