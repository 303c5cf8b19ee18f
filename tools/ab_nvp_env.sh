#!/bin/bash
# A/B of RealNVP gradient variants selected by environment (e.g. PDEINV_NVP_PACK=0) on one box.
# Usage: bash tools/ab_nvp_env.sh <tag> "ENV=.. ENV2=.." "ENV=.." ...   (first = baseline "")
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/ab_nvp_${1:-x}.txt; : > $OUT
shift
for rep in 1 2; do
  for v in "$@"; do
    r=$(env $v timeout -k 10 120 python tools/nvp_bench.py --steps 30 2>/dev/null) || { echo "[$v] failed" >> $OUT; exit 3; }
    echo "[$v] $(echo "$r" | python -c 'import sys,json;print(" ".join("%s %.3f ms %.3f"%(j["workload"][15:20],j["ms_per_step"],j["valu_frac"]) for j in map(json.loads,sys.stdin)))')" | tee -a $OUT
  done
done
