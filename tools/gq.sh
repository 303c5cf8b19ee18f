#!/bin/bash
# MFMA pair-tile kernels: parity tests, recipe timing (new vs register-ring), kernel-trace stats.
# Usage: bash tools/gq.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_mirror.py -x -v --timeout 300 --timeout-method thread -k "general_phi or kmv_non" > gpurun_out/q_$TAG.log 2>&1 || { tail -30 gpurun_out/q_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/q_$TAG.log | tail -2
timeout -k 10 300 python tools/kmv_mlp_time.py 2,5000,1,20,8,2 2,2000,3,20,8,2 2>&1 | tee gpurun_out/q_time_$TAG.jsonl || exit 2
timeout -k 10 300 python tools/kmv_mlp_time.py 2,5000,1,20,8,3 2>&1 | tee -a gpurun_out/q_time_$TAG.jsonl || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/q_tr_$TAG -o run --output-format csv -- python3 $R/tools/kmv_mlp_time.py 2,5000,1,20,8,2 > $R/gpurun_out/q_tr_$TAG.log 2>&1 || exit 4
grep -E "kmvq|kmvp" $R/gpurun_out/q_tr_$TAG/run_kernel_stats.csv | cut -d, -f1-4
