#!/bin/bash
# round-3 evidence: every GPU test, smoke, the driver's default bench line,
# then rocprofv3 kernel traces + PMC FETCH/WRITE passes of every BASELINE
# config (tools/profile_all.sh), the summary copied next to the logs
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/full_check.sh $TAG || exit 10
bash tools/r03_k.sh $TAG || exit 11
bash tools/profile_all.sh $TAG c5 c1 c2 c2i c3a c3b c4 || exit 12
echo profiles done
