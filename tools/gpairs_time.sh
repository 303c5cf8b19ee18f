#!/bin/bash
# Pair kernels: parity tests, recipe timing, kernel-trace stats. Usage: bash tools/gpairs_time.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_mirror.py -x -q --timeout 300 --timeout-method thread -k "general_phi or kmv_non" > gpurun_out/pairs_$TAG.log 2>&1 || { tail -20 gpurun_out/pairs_$TAG.log; exit 1; }
tail -1 gpurun_out/pairs_$TAG.log
timeout -k 10 300 python tools/kmv_mlp_time.py 2,5000,1,20,8,2 2>/dev/null || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pairs_tr_$TAG -o run --output-format csv -- python3 $R/tools/kmv_mlp_time.py 2,5000,1,20,8,2 > $R/gpurun_out/pairs_tr_$TAG.log 2>&1 || exit 3
grep kmvp $R/gpurun_out/pairs_tr_$TAG/run_kernel_stats.csv | cut -d, -f1-4
