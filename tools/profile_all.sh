#!/bin/bash
# Bench lines + rocprofv3 kernel-trace summaries for C2..C5 (one GPU). Output under gpurun_out/prof_all.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_all
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in C2 C3 C4 C5; do
  timeout -k 10 300 python3 $R/bench.py --config $C --steps 10 --warmup 3 > $OUT/bench_$C.json 2> $OUT/bench_$C.err || exit 11
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$C -o run --output-format csv -- python3 $R/bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > $OUT/prof_$C.log 2>&1 || exit 12
  echo "$C done"
done
