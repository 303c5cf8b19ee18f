#!/bin/bash
# C4 schedule A/B on one box: fused next-simulate sums in the KMV pass vs the unfused pass with the sums
# concurrent on a side stream vs the separate serial sums. Usage: bash tools/r04_c4.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
OUT=gpurun_out/c4ab_$TAG.txt
: > $OUT
for rep in 1 2; do
  for sch in fused concurrent separate; do
    extra="--c4-schedule $sch"
    [ $sch = separate ] && extra="--c4-separate-sums"
    timeout -k 10 200 python3 bench.py --config C4 --steps 30 --warmup 5 --no-cpu-baseline $extra > gpurun_out/c4_$sch.json 2> gpurun_out/c4_$sch.err || { tail -20 gpurun_out/c4_$sch.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/c4_$sch.json')); print('$sch', round(d['ms_per_step'],4), 'sim', round(d['roofline']['kernel_ms'],4), 'res', round(d['residual']['ms'],4), 'GBps', round(d['residual']['GBps']), 'mean_path', round(d['mean_path']['ms'],4))" | tee -a $OUT
  done
done
