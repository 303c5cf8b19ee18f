#!/bin/bash
# r05: new-feature parity (QuadGram moments, KMV rebase, device OU sampler, path queries), then the C2 launch A/B.
cd "$GRAFT_REPO_ROOT"
V=pde-inverse-problem_amd/_build/var
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_meanfield.py \
  -k "moments or sde or residual_quadratic or ou_exact or kou_exact" > gpurun_out/r05_check1_tests.txt 2>&1 || { tail -30 gpurun_out/r05_check1_tests.txt; exit 1; }
tail -2 gpurun_out/r05_check1_tests.txt
for r in 1 2 3; do
  for v in base quadw1 default quadw7; do
    if [ $v = default ]; then timeout -k 10 120 python tools/sim_time.py | sed "s/^/$v /" || exit 1
    else PDEINV_LIBRARY=$PWD/$V/$v.so timeout -k 10 120 python tools/sim_time.py | sed "s/^/$v /" || exit 1; fi
  done
done 2>&1 | tee gpurun_out/r05_quad_ab.txt
