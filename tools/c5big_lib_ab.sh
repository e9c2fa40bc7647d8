#!/bin/bash
# Multi-chunk tile-mode variants on 4 MiB C5 tiles, one box, 2 reps:
# the product library, round-6 v1 (libtiledb_amd_v1.so: DMA after the stores,
# state publish barrier), and the pipelined DMA (experiments, TDBG_C5T_PIPE).
set -o pipefail
for rep in 1 2; do
  MODES=None bash tools/c5big_ab2.sh ${1:-x}_prod_$rep | sed "s/^/prod  /" || exit 11
  MODES=None ENVS="TDBG_LIB=libtiledb_amd_v1.so" bash tools/c5big_ab2.sh ${1:-x}_v1_$rep | sed "s/^/v1    /" || exit 12
  MODES=None ENVS="TDBG_LIB=libtiledb_amd_exp.so TDBG_C5T_PIPE=1" bash tools/c5big_ab2.sh ${1:-x}_pipe_$rep | sed "s/^/pipe  /" || exit 13
done
