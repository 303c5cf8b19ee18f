cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused_gmm.py tests/test_gpu_golden.py "tests/test_gpu_kernels.py" -k "gmm or golden or fused" > gpurun_out/t3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t3.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 200 python -u bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3a.log 2>&1 && \
  PDEINV_LIBRARY=$PWD/tools/_bin/libpdeinv_b.so timeout -k 10 200 python -u bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3b.log 2>&1; echo "bench rc=$?"
fi
