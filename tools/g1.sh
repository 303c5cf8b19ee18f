cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_meanfield.py tests/test_gpu_multirank.py "tests/test_gpu_kernels.py::test_residual_mlp_library_two_threads_two_streams" > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u bench.py --config C4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c4.log 2>&1; echo "bench rc=$?"
fi
tail -5 gpurun_out/t1.log
