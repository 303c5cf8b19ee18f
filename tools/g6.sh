cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "residual_mlp" > gpurun_out/t6.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/t6.log | tail -22
