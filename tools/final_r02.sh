#!/bin/bash
# End-of-round pass: all GPU tests, smoke, then C5 bench + rocprofv3 trace +
# PMC traffic (tools/profile_all.sh) for the committed profiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/full_check.sh ${1:-f} || exit $?
bash tools/profile_all.sh ${1:-f} c5 || exit $?
