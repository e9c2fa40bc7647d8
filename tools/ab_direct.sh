#!/bin/bash
# all-raw tiles without range setup or table lookups (rand): parity + same-box A/B
set -o pipefail
mkdir -p gpurun_out/direct
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py tests/test_gpu_c2tile.py -x -q --timeout 120 --timeout-method thread > gpurun_out/direct/t.log 2>&1 || { tail -30 gpurun_out/direct/t.log; exit 11; }
tail -1 gpurun_out/direct/t.log
VARS="rand ramp" bash tools/ab_lib.sh direct_c5 && VARS="rand" CFG=c5big bash tools/ab_lib.sh direct_c5big
