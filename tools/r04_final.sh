#!/bin/bash
# Round-4 final records on one box: full GPU suite + smoke, the default bench command traced under
# rocprofv3 (same run) and plain, the C3 / C4 / C5 bench lines, RealNVP and the pair kernels.
# Every step under its own limit; a fatal status (timeout / abort / segfault) ends the script.
# Usage: bash tools/r04_final.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1 ;; esac; }
bash tools/gtest_all.sh $TAG; rc=$?; echo "tests rc=$rc"; fatal $rc tests
bash tools/r04_check.sh $TAG skip-tests; rc=$?; echo "check rc=$rc"; fatal $rc check
for c in C3 C4 C5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 > gpurun_out/final_${TAG}_$c.json 2> gpurun_out/final_${TAG}_$c.err
  rc=$?; echo "bench $c rc=$rc"; fatal $rc bench_$c
  python3 -c "import json; d=json.load(open('gpurun_out/final_${TAG}_$c.json')); print('$c', d['value'], d['unit'], d['ms_per_step'], d['roofline']['frac'])" || true
done
timeout -k 10 200 python3 tools/nvp_bench.py --steps 30 --warmup 5 --dims 2,4 > gpurun_out/final_${TAG}_nvp.jsonl 2>&1; rc=$?; echo "nvp rc=$rc"; fatal $rc nvp
cat gpurun_out/final_${TAG}_nvp.jsonl
timeout -k 10 300 python3 tools/kmv_mlp_time.py 2,5000,1,20,8,2 > gpurun_out/final_${TAG}_pairs.jsonl 2>&1; rc=$?; echo "pairs rc=$rc"; fatal $rc pairs
cat gpurun_out/final_${TAG}_pairs.jsonl
