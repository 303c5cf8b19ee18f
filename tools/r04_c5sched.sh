#!/bin/bash
# C5 with the rgemm / wgrad2 schedule variants (PDEINV_MLP_SCHED 0 / 1 = default / 3), alternating on one box.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/c5sched.txt
: > $OUT
for rep in 1 2; do
  for v in 1 0 3; do
    PDEINV_MLP_SCHED=$v timeout -k 10 300 python3 bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5s.json 2> gpurun_out/c5s.err || { tail -20 gpurun_out/c5s.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c5s.json')); print('C5 SCHED=$v', round(d['ms_per_step'],3), 'residual', round(d['roofline']['kernel_ms'],3))" | tee -a $OUT
  done
done
