#!/bin/bash
# r05: C2 simulator trajectory stores, non-temporal (default) vs plain (PDEINV_SIM_PLAIN_STORES=1), alternating.
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for v in default plainst; do
    if [ $v = default ]; then timeout -k 10 120 python tools/sim_tau.py | head -1 | sed "s/^/$v /" || exit 1
    else PDEINV_LIBRARY=$PWD/pde-inverse-problem_amd/_build/var/$v.so timeout -k 10 120 python tools/sim_tau.py | head -1 | sed "s/^/$v /" || exit 1; fi
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05_store_ab.txt
