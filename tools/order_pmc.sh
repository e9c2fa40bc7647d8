#!/bin/bash
# Address-translation counters of the C5 tile kernel in the two leg orders
# whose rates differ (tools/order_probe.sh): ramp then rand, rand then ramp.
# Separate --pmc passes (no traces); per leg the median over its launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/order_pmc_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
P2="GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
P3="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
for ORD in ramp,rand rand,ramp; do
  P=0
  for SET in "$P1" "$P2" "$P3"; do
    P=$((P+1))
    timeout -s KILL 150 rocprofv3 --pmc $SET --output-format csv -d $OUT/${ORD/,/_}_p$P -o run -- python3 $R/bench.py --variants $ORD --steps 10 --warmup 2 --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 --c5s-tiles 0 > $OUT/${ORD/,/_}_p$P.log 2>&1 || { echo "pmc $ORD $P failed"; tail -5 $OUT/${ORD/,/_}_p$P.log; exit 12; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, statistics
out = sys.argv[1]
for ordr in ("ramp_rand", "rand_ramp"):
    per = {}
    for f in glob.glob(os.path.join(out, ordr + "_p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "unfilter_c5tile" not in r["Kernel_Name"]:
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            key = (os.path.basename(os.path.dirname(os.path.dirname(f))) if False else f.split(ordr + "_p")[1][0], d)
            per.setdefault(r["Counter_Name"], {}).setdefault(d, 0.0)
            per[r["Counter_Name"]][d] += float(r["Counter_Value"])
    legs = ordr.split("_")
    for c, m in sorted(per.items()):
        ds = sorted(m)
        h = len(ds) // 2
        a = statistics.median([m[d] for d in ds[:h]]); b = statistics.median([m[d] for d in ds[h:]])
        print(f"{ordr:10s} {c:34s} {legs[0]}(first) {a:16.0f}   {legs[1]}(second) {b:16.0f}")
PY
