"""Median per-launch SQ counters of the fused unfilter kernel from
tools/sq_prof.sh passes, with per-tile derived figures.  SQ_*_CYCLES and
SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md)."""
import csv
import glob
import json
import os
import statistics
import sys


def collect(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if os.environ.get("TDBG_KNAME", "unfilter_fused_kernel") not in r["Kernel_Name"]:
                continue
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    by = {}
    for (disp, name), v in per.items():
        by.setdefault(name, []).append(v)
    return {k: statistics.median(v) for k, v in by.items()}


def main(out, cfg, var, tiles=12500):
    c = {}
    dirs = [d for d in sorted(glob.glob(os.path.join(out, "pass*"))) if os.path.isdir(d)] or [out]
    for d in dirs:
        c.update(collect(d))
    res = {"config": cfg, "variant": var, "counters_median_per_launch": c}
    der = {}
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA"):
            if k in c:
                der[k + "_share_of_wave_cycles"] = round(c[k] / w, 4)
    # per CU: SALU issues one instruction per cycle for the whole CU, so
    # SALU instructions / CU vs the kernel's cycles is the scalar unit's load
    if "SQ_INSTS_SALU" in c:
        der["SQ_INSTS_SALU_per_CU"] = round(c["SQ_INSTS_SALU"] / 256, 1)
    if "SQ_INSTS_VALU" in c:
        der["SQ_INSTS_VALU_per_SIMD"] = round(c["SQ_INSTS_VALU"] / 1024, 1)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        if k in c:
            der[k + "_per_tile"] = round(c[k] / tiles, 1)
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
        der["lds_bank_conflict_share"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
    res["derived"] = der
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 12500)
