#!/bin/bash
# C5 residual chunk size A/B (bench.py --chunk-rows), alternating on one box.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/c5chunk_${1:-x}.txt
: > $OUT
for rep in 1 2; do
  for c in 2097152 4194304 5242880; do
    timeout -k 10 300 python3 bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --chunk-rows $c > gpurun_out/c5c.json 2> gpurun_out/c5c.err || { tail -20 gpurun_out/c5c.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c5c.json')); print('C5 chunk $c', round(d['ms_per_step'],3), 'residual', round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],4))" | tee -a $OUT
  done
done
