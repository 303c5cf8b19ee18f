#!/bin/bash
# KMV pass alone, library variants alternating (tools/kmv_time.py).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}; shift
OUT=gpurun_out/kmvt_${TAG}.txt
: > $OUT
for rep in 1 2 3; do
  for lib in base "$@"; do
    if [ $lib = base ]; then L=pde-inverse-problem_amd/_build/libpdeinv.so; else L=pde-inverse-problem_amd/_build/var/$lib; fi
    PDEINV_LIBRARY=$L timeout -k 10 120 python3 tools/kmv_time.py 30 2>> gpurun_out/kmvt.err | tee -a $OUT || exit 1
  done
done
