#!/bin/bash
set -o pipefail
BARGS="--no-cpu-baseline --no-e2e --no-forward --no-others --shard-tiles 0 --c5s-tiles 0" bash tools/profile_all.sh r05c c5shard || exit 1
bash tools/ceiling_pmc.sh c || exit 2
VARS="active rand" KN=unfilter_c5tile_kernel bash tools/sq_stream.sh r05/sq_c5t || exit 3
