#!/bin/bash
# KMV pass alone at C4 shape for several grid targets (PDEINV_KMV_GRID), two alternating rounds.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/kmvgrid_${1:-x}.txt
: > $OUT
for rep in 1 2; do
  for g in 3072 2048 4096 6144 8192; do
    echo -n "grid $g: " | tee -a $OUT
    PDEINV_KMV_GRID=$g timeout -k 10 120 python3 tools/kmv_time.py 30 2>> gpurun_out/kmvgrid.err | tee -a $OUT || exit 1
  done
done
