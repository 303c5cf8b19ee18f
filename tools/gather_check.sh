#!/bin/bash
# gather parity tests + C5 trace (gather kernel timing)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gather" > gpurun_out/gather_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gather_t.log | tail -3
[ $rc -eq 0 ] || exit $rc
bash tools/c5_trace.sh gath
