#!/bin/bash
# r05: MLP residual / KMV parity, then C5 with an A/B environment switch off / on (alternating, 3 rounds).
# Usage: bash tools/r05_ab_env.sh <VAR> <tag>
cd "$GRAFT_REPO_ROOT"
VAR=$1; TAG=$2
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_mirror.py tests/test_gpu_meanfield.py -k "residual_mlp or kmv or vs_pairwise_restatement" \
  > gpurun_out/r05_${TAG}_tests.txt 2>&1 || { tail -40 gpurun_out/r05_${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/r05_${TAG}_tests.txt
for r in 1 2 3; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline \
      --no-recovery > gpurun_out/r05_${TAG}_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r05_${TAG}_$v.json')); r=d['roofline']; print('$VAR=$v', round(d['ms_per_step'],2), 'residual', round(r['kernel_ms'],2), 'frac', round(r['frac'],4))"
  done
done 2>&1 | tee gpurun_out/r05_${TAG}_ab.txt
