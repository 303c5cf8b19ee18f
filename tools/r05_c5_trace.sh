#!/bin/bash
# r05: MLP residual parity, a C5 bench line and a C5 kernel trace (per-kernel averages) for the current build.
# Usage: bash tools/r05_c5_trace.sh <tag> [ENV=VAL ...]
cd "$GRAFT_REPO_ROOT"; R=$PWD; TAG=$1; shift
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  -k "residual_mlp" > gpurun_out/r05_${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/r05_${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/r05_${TAG}_tests.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline --no-recovery \
    > gpurun_out/r05_${TAG}_c5.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r05_${TAG}_c5.json')); r=d['roofline']; print('$TAG', round(d['ms_per_step'],2), 'residual', round(r['kernel_ms'],2), 'frac', round(r['frac'],4))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o run --output-format csv \
  -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/prof_${TAG}.log 2>&1 || exit 1
python3 - <<PY
import csv,glob
f=glob.glob('$R/gpurun_out/prof_${TAG}/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e6,3), round(float(r['TotalDurationNs'])/1e6,2))
PY
