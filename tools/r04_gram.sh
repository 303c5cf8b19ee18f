#!/bin/bash
# C2 simulator variants (step-loop Gram on MFMA): moment parity under each library, then the C2 A/B.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}; shift
for v in "$@"; do
  PDEINV_LIBRARY=pde-inverse-problem_amd/_build/var/$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_kernels.py -k "moments or sde" > gpurun_out/gram_${TAG}_${v%.so}_test.log 2>&1 || { tail -30 gpurun_out/gram_${TAG}_${v%.so}_test.log; exit 1; }
  tail -1 gpurun_out/gram_${TAG}_${v%.so}_test.log
done
bash tools/ab_cfg.sh $TAG C2 "$@"
