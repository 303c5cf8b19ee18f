#!/bin/bash
# C4: the default serial schedule vs the two-stream pipeline, alternating on one box.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/c4pipe_${1:-x}.txt
: > $OUT
for rep in 1 2; do
  for m in "" "--c4-pipeline"; do
    timeout -k 10 300 python3 bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline $m > gpurun_out/c4p.json 2> gpurun_out/c4p.err || { tail -20 gpurun_out/c4p.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c4p.json')); print('C4 ${m:-serial}', round(d['ms_per_step'],4), 'sim', round(d['roofline']['kernel_ms'],4), d.get('kmv_pass_ms', d.get('residual_ms')))" | tee -a $OUT
  done
done
