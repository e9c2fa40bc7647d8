#!/bin/bash
# new adjacent-step GPU tests, stream tests, then the driver's default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-l}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_adjacent_steps.py tests/test_gpu_stream.py -p no:cacheprovider > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $OUT/tests.log; exit 10; }
tail -3 $OUT/tests.log
bash tools/r03_k.sh ${1:-l}
