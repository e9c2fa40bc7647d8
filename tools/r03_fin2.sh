#!/bin/bash
# end of round 3: every GPU test, smoke, 2-rank rehearsal, the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/full_check.sh ${1:-fin2} || exit 10
bash tools/r03_k.sh ${1:-fin2} || exit 11
