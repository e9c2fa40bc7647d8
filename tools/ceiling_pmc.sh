#!/bin/bash
# HBM request counters of the ceiling probe's 1:1 float4 copy (tools/ceiling3,
# "C u4 st-plain ld-plain b256": 6.55 GB read + 6.55 GB written per launch,
# 13 launches): do the bytes the memory system moves equal the algorithmic
# bytes?  Separate --pmc passes (MI355X_MICROARCH.md HBM recipe).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/ceil_pmc_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 60 tools/ceiling3 "C u4 st-plain ld-plain b256" > $OUT/plain.log 2>&1 || exit 11
cat $OUT/plain.log
P=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  P=$((P+1))
  timeout -s KILL 60 rocprofv3 --pmc $SET --output-format csv -d $OUT/pass$P -o run -- tools/ceiling3 "C u4 st-plain ld-plain b256" > $OUT/pass$P.log 2>&1 || { echo "pass $P failed"; tail -5 $OUT/pass$P.log; exit 12; }
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, statistics
out = sys.argv[1]
res = {}
for f in glob.glob(os.path.join(out, "pass*", "**", "*counter_collection.csv"), recursive=True):
    per = {}
    for r in csv.DictReader(open(f)):
        if "k_copy" not in r["Kernel_Name"]:
            continue
        key = (int(r.get("Dispatch_Id") or r.get("Correlation_Id")), r["Counter_Name"])
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (d, c), v in per.items():
        res.setdefault(c, []).append(v)
alg = 6553600000.0
for c, vs in sorted(res.items()):
    m = statistics.median(vs)
    print(f"{c:28s} median per launch {m:16.1f}  launches {len(vs)}")
print(f"algorithmic bytes per launch: read {alg:.0f}, write {alg:.0f}")
PY
