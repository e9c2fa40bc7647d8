#!/bin/bash
# wave-uniform pats2-unit stores in partial chunks (40,000-B tiles) A/B
set -o pipefail
mkdir -p gpurun_out/pats2
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pats2/t.log 2>&1 || { tail -30 gpurun_out/pats2/t.log; exit 11; }
tail -1 gpurun_out/pats2/t.log
VARS="ramp rand" CFG=c5s bash tools/ab_lib.sh pats2_c5s && VARS="ramp" bash tools/ab_lib.sh pats2_c5
