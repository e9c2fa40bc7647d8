#!/bin/bash
# Does a C5 variant's rate depend on what ran before it (warm-up / clocks)
# rather than on the kernel?  100,000 tiles, one box, bench.py legs in order.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/order_${1:-x}
mkdir -p $OUT
cd $R
run() {  # name, bench args... (later flags win: --e2e / --forward turn the legs back on)
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 --c5s-tiles 0 "$@" \
    > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -20 $OUT/$n.err; exit 11; }
  python -c "
import json; d=json.loads([l for l in open('$OUT/$n.json') if l.startswith('{')][-1]); v=d['config']['variants']
print('$n', {k: (v[k]['roofline_frac'], v[k]['kernel_ms']) for k in v})"
}
case ${1:-a} in
a)
run rand_w3 --variants rand
run rand_w300 --variants rand --warmup 300
run ramp_w3 --variants ramp
run ramp_w300 --variants ramp --warmup 300
run ramp_rand_active --variants ramp,rand,active
run active_rand_ramp --variants active,rand,ramp
;;
b)  # the legs between variants: host end-to-end (e2e) and forward
run rr_e2e --variants rand,ramp --e2e
run ramp_rand_e2e --variants ramp,rand --e2e
run ramp_fwd --variants ramp --forward
run arr_e2e_fwd --variants active,rand,ramp --e2e --forward
;;
esac
