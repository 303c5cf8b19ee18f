#!/bin/bash
# bench.py --config <C> with library variants (PDEINV_LIBRARY), alternating on one box.
# Usage: bash tools/ab_cfg.sh <tag> <config> <var.so>...
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}; CFG=${2:-C3}; shift 2
OUT=gpurun_out/abcfg_${TAG}.txt
: > $OUT
for rep in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then L=pde-inverse-problem_amd/_build/libpdeinv.so; else L=pde-inverse-problem_amd/_build/var/$lib; fi
    PDEINV_LIBRARY=$L timeout -k 10 300 python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abcfg.json 2> gpurun_out/abcfg.err || { tail -20 gpurun_out/abcfg.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abcfg.json')); print('$CFG $lib', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))" | tee -a $OUT
  done
done
