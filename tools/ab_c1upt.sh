#!/bin/bash
# C1 shuffle kernel: 1 (HEAD) vs 2 vs 4 output units per thread, same box
set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "c1 or shuffle" > gpurun_out/c1upt_t.log 2>&1 || { tail -20 gpurun_out/c1upt_t.log; exit 11; }
tail -1 gpurun_out/c1upt_t.log
LIBS="libtiledb_amd_base.so libtiledb_amd_u2.so libtiledb_amd_u4.so" VARS="rand ramp" CFG=c1 bash tools/ab_lib.sh c1upt
