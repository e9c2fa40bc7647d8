#!/bin/bash
# wave-uniform s1-unit stores in partial chunks (40,000-B tiles) A/B
set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s1/t.log 2>&1 || { tail -30 gpurun_out/s1/t.log; exit 11; }
tail -1 gpurun_out/s1/t.log
VARS="rand ramp" bash tools/ab_lib.sh s1_c5 && VARS="rand ramp" CFG=c5s bash tools/ab_lib.sh s1_c5s
