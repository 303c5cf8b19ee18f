#!/bin/bash
# r05: QuadGram C2 moments — parity subset, then the simulator launch A/B (HEAD sde.hip vs quad at 5/6/7 waves).
cd "$GRAFT_REPO_ROOT"
V=pde-inverse-problem_amd/_build/var
# timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
#   -k "moments or sde or residual_quadratic" tests/test_gpu_meanfield.py > gpurun_out/r05_quad_tests.txt 2>&1 || { tail -30 gpurun_out/r05_quad_tests.txt; exit 1; }
# tail -3 gpurun_out/r05_quad_tests.txt
for r in 1 2 3; do
  for v in base quadw1 default quadw7; do
    if [ $v = default ]; then timeout -k 10 120 python tools/sim_time.py | sed "s/^/$v /" || exit 1
    else PDEINV_LIBRARY=$PWD/$V/$v.so timeout -k 10 120 python tools/sim_time.py | sed "s/^/$v /" || exit 1; fi
  done
done 2>&1 | tee gpurun_out/r05_quad_ab.txt
