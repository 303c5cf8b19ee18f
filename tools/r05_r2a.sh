#!/bin/bash
# r05: the K = out_features reverse product (R2a) tile A/B: C5 bench lines and the kernel's traced average per variant.
cd "$GRAFT_REPO_ROOT"; R=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  -k "residual_mlp" > gpurun_out/r05_r2a_tests.txt 2>&1 || { tail -30 gpurun_out/r05_r2a_tests.txt; exit 1; }
tail -1 gpurun_out/r05_r2a_tests.txt
for r in 1 2; do
  for v in 0 1 2 3; do
    PDEINV_MLP_R2A=$v timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline \
      --no-recovery > gpurun_out/r05_r2a_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r05_r2a_$v.json')); r=d['roofline']; print('R2A=$v', round(d['ms_per_step'],2), 'residual', round(r['kernel_ms'],2))"
  done
done 2>&1 | tee gpurun_out/r05_r2a_ab.txt
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 3; do
  PDEINV_MLP_R2A=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2a_prof_$v -o run --output-format csv \
    -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/r2a_prof_$v.log 2>&1 || exit 1
  python3 -c "
import csv,glob
f=glob.glob('$R/gpurun_out/r2a_prof_$v/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'fgemm<3' in r['Name'] and ', 5,' in r['Name']: print('R2A=$v', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms avg')
" | tee -a $R/gpurun_out/r05_r2a_ab.txt
done
