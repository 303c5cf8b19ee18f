#!/bin/bash
# C4 schedule A/B on one box: the next simulate's mean-path sums inside the simulator (sim) vs inside the KMV
# pass (fused, the r03 default) vs separate sums. Usage: bash tools/r04_c4b.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
OUT=gpurun_out/c4b_$TAG.txt
: > $OUT
for rep in 1 2; do
  for sch in sim fused separate; do
    extra="--c4-schedule $sch"
    [ $sch = separate ] && extra="--c4-separate-sums"
    timeout -k 10 200 python3 bench.py --config C4 --steps 30 --warmup 5 --no-cpu-baseline $extra > gpurun_out/c4b_$sch.json 2> gpurun_out/c4b_$sch.err || { tail -20 gpurun_out/c4b_$sch.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/c4b_$sch.json')); print('$sch', round(d['ms_per_step'],4), 'sim', round(d['roofline']['kernel_ms'],4), 'res', round(d['residual']['ms'],4), 'GBps', round(d['residual']['GBps']), 'mean_path', round(d['mean_path']['ms'],4))" | tee -a $OUT
  done
done
