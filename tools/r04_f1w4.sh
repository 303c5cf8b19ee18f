#!/bin/bash
# The 4-wave NI = 4 layer-1-prologue forward (PDEINV_MLP_F1W4=1): MLP residual parity under it, then the C5 A/B
# against the default 8-wave kernel (same library, alternating).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PDEINV_MLP_F1W4=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "residual_mlp" > gpurun_out/f1w4_test.log 2>&1 || { tail -30 gpurun_out/f1w4_test.log; exit 1; }
tail -1 gpurun_out/f1w4_test.log
OUT=gpurun_out/f1w4_ab.txt
: > $OUT
for rep in 1 2; do
  for w in 0 1; do
    PDEINV_MLP_F1W4=$w timeout -k 10 300 python3 bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/f1w4.json 2> gpurun_out/f1w4.err || { tail -20 gpurun_out/f1w4.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/f1w4.json')); print('C5 F1W4=$w', round(d['ms_per_step'],3), 'residual', round(d['roofline']['kernel_ms'],3))" | tee -a $OUT
  done
done
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
PDEINV_MLP_F1W4=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_f1w4 -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_f1w4.log 2>&1 || exit 1
grep -i "rgemm" $R/gpurun_out/prof_f1w4/run_kernel_stats.csv | cut -c1-140
