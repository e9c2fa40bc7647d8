#!/bin/bash
# round-3 block swap A/B (raw path): parity of the raw/shape tests, then
# same-box bench A/B of HEAD's library against the working tree's
set -o pipefail
mkdir -p gpurun_out/rblk
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rblk/t.log 2>&1 || { tail -30 gpurun_out/rblk/t.log; exit 11; }
tail -1 gpurun_out/rblk/t.log
VARS="ramp rand active" bash tools/ab_lib.sh rblk_c5 && VARS="ramp" CFG=c5s bash tools/ab_lib.sh rblk_c5s
