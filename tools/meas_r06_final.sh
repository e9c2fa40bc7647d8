#!/bin/bash
# Round-6 final profiles: per config (args) rocprofv3 kernel traces and
# separate FETCH_SIZE / WRITE_SIZE passes for every variant
# (tools/profile_all.sh), the bench line of each config alone.
# usage: bash tools/meas_r06_final.sh <tag> <configs...>
set -o pipefail
T=$1; shift
BARGS="--no-cpu-baseline --no-e2e --no-forward --no-others --shard-tiles 0 --c5s-tiles 0 --c5big-tiles 0 --legs-file=" bash tools/profile_all.sh r06final_$T "$@"
