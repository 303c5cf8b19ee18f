cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
exit $rc
