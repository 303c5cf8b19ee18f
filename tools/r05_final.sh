#!/bin/bash
# Round-5 records on one box: full GPU suite + smoke; the default bench command traced under rocprofv3 (same run)
# and plain; the C3 / C4 / C5 lines and their rocprof kernel statistics; RealNVP and the pair recipe; the C5
# per-residual traffic (FETCH_SIZE / WRITE_SIZE passes). Every step under its own limit; a fatal status ends it.
# Usage: bash tools/r05_final.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1 ;; esac; }
bash tools/gtest_all.sh $TAG; rc=$?; echo "tests rc=$rc"; fatal $rc tests
bash tools/r04_check.sh $TAG skip-tests; rc=$?; echo "check rc=$rc"; fatal $rc check
for c in C3 C4 C5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 > gpurun_out/final_${TAG}_$c.json 2> gpurun_out/final_${TAG}_$c.err
  rc=$?; echo "bench $c rc=$rc"; fatal $rc bench_$c
  python3 -c "import json; d=json.load(open('gpurun_out/final_${TAG}_$c.json')); print('$c', d['value'], d['unit'], d['ms_per_step'], d['roofline']['frac'])" || true
done
bash tools/r04_prof_cfgs.sh $TAG; rc=$?; echo "prof cfgs rc=$rc"; fatal $rc prof
timeout -k 10 200 python3 tools/nvp_bench.py --steps 30 --warmup 5 --dims 2,4 > gpurun_out/final_${TAG}_nvp.jsonl 2>&1; rc=$?; echo "nvp rc=$rc"; fatal $rc nvp
timeout -k 10 300 python3 tools/kmv_mlp_time.py 2,5000,1,20,8,2 > gpurun_out/final_${TAG}_pairs.jsonl 2>&1; rc=$?; echo "pairs rc=$rc"; fatal $rc pairs
cd /tmp && export TMPDIR=/tmp
A5="--config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery"
RX="sde_simulate|mlpf|mlp_loss|gather_random|fillBuffer"
mkdir -p $R/gpurun_out/prof_${TAG}_c5pmc
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d $R/gpurun_out/prof_${TAG}_c5pmc/fetch -o run \
  --output-format csv -- python3 $R/bench.py $A5 > $R/gpurun_out/prof_${TAG}_c5pmc/fetch.log 2>&1; rc=$?; echo "c5 fetch rc=$rc"; fatal $rc fetch
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d $R/gpurun_out/prof_${TAG}_c5pmc/write -o run \
  --output-format csv -- python3 $R/bench.py $A5 > $R/gpurun_out/prof_${TAG}_c5pmc/write.log 2>&1; rc=$?; echo "c5 write rc=$rc"; fatal $rc write
cd $R
python3 tools/c5_traffic.py gpurun_out/prof_${TAG}_c5pmc 3 | tee gpurun_out/final_${TAG}_c5_traffic.txt
