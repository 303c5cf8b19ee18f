#!/bin/bash
# C4 bench line three times on one box (final code).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/c4rep.txt
: > $OUT
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c4r_$rep.json 2> gpurun_out/c4r.err || { tail -20 gpurun_out/c4r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4r_$rep.json')); print('C4', round(d['ms_per_step'],3), 'sim', round(d['roofline']['kernel_ms'],3), 'kmv', round(d['residual']['ms'],3), round(d['residual']['GBps']))" | tee -a $OUT
done
