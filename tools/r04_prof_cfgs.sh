#!/bin/bash
# rocprofv3 --kernel-trace --stats of bench.py --config C3 / C4 / C5 (final code), one run each.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
cd /tmp && export TMPDIR=/tmp
for c in C3 C4 C5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_$c -o run --output-format csv \
    -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_${TAG}_$c.json 2> $R/gpurun_out/prof_${TAG}_$c.err || exit 1
  echo "$c done"
done
