#!/bin/bash
# C4 'sim' schedule: library variants A/B (PDEINV_LIBRARY), alternating. Usage: bash tools/r04_c4c.sh <tag> <var.so>...
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}; shift
OUT=gpurun_out/c4c_$TAG.txt
: > $OUT
for rep in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then L=pde-inverse-problem_amd/_build/libpdeinv.so; else L=pde-inverse-problem_amd/_build/var/$lib; fi
    PDEINV_LIBRARY=$L timeout -k 10 200 python3 bench.py --config C4 --c4-schedule sim --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c4c.json 2> gpurun_out/c4c.err || { tail -20 gpurun_out/c4c.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/c4c.json')); print('$lib', round(d['ms_per_step'],4), 'sim', round(d['roofline']['kernel_ms'],4), 'res', round(d['residual']['ms'],4))" | tee -a $OUT
  done
done
