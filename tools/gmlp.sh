#!/bin/bash
# MLP residual iteration loop on the box: fused-path parity tests, the C5 bench line, a kernel-trace
# profile of the same. Usage: bash tools/gmlp.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "residual_mlp" > gpurun_out/mlp_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/mlp_$TAG.log | tail -22
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || exit 11
cat gpurun_out/c5_$TAG.json
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5prof_$TAG -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/c5prof_$TAG.log 2>&1 || exit 12
echo done
