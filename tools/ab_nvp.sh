#!/bin/bash
# A/B of RealNVP gradient builds (PDEINV_LIBRARY) on one box: nvp_bench d = 2, 4, alternating.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/ab_nvp_${1:-x}.txt; : > $OUT
shift
for rep in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then L=pde-inverse-problem_amd/_build/libpdeinv.so; else L=pde-inverse-problem_amd/_build/var/$lib; fi
    r=$(PDEINV_LIBRARY=$L timeout -k 10 120 python tools/nvp_bench.py --steps 30 2>/dev/null) || { echo "$lib failed" >> $OUT; exit 3; }
    echo "$lib $(echo "$r" | python -c 'import sys,json;print(" ".join("%s %.3f ms"%(j["workload"][15:20],j["ms_per_step"]) for j in map(json.loads,sys.stdin)))')" | tee -a $OUT
  done
done
