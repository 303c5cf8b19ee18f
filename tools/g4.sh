cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mirror.py -k "general_phi or kmv_non_parametric" > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/t4.log | head -30
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u tools/kmv_mlp_time.py > gpurun_out/kmv_mlp_time2.log 2>&1; echo "time rc=$?"; tail -3 gpurun_out/kmv_mlp_time2.log
fi
