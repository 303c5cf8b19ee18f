#!/bin/bash
# C5 A/B of one MLP-residual switch: parity tests of the fused MLP residual, then the C5 bench line with
# the default and with <VAR>=0, and a kernel trace of the default. Usage: bash tools/c5_ab.sh <tag> <VAR>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
VAR=${2:-PDEINV_MLP_WL1}
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "residual_mlp or mlp_fused" > gpurun_out/ab_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/ab_$TAG.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || exit 11
cat gpurun_out/c5_$TAG.json
env $VAR=0 timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > gpurun_out/c5_${TAG}_off.json 2> gpurun_out/c5_${TAG}_off.err || exit 12
cat gpurun_out/c5_${TAG}_off.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5prof_$TAG -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/c5prof_$TAG.log 2>&1 || exit 13
echo done
