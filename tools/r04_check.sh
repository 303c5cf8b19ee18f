#!/bin/bash
# Round-4 check on one box: full GPU suite + smoke, then the exact default bench command under
# rocprofv3 --kernel-trace --stats (same run: the printed line and the per-dispatch trace it came from),
# then the same command without the profiler. Usage: bash tools/r04_check.sh <tag> [skip-tests]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
if [ "${2:-}" != "skip-tests" ]; then
  bash tools/gtest_all.sh $TAG || exit $?
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv \
  -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err || exit 31
cd $R
python3 tools/trace_timed.py gpurun_out/prof_$TAG gpurun_out/bench_prof_$TAG.json > gpurun_out/trace_timed_$TAG.json || exit 32
cat gpurun_out/trace_timed_$TAG.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_plain_$TAG.json 2> gpurun_out/bench_plain_$TAG.err || exit 33
python3 -c "import json; d=json.load(open('gpurun_out/bench_plain_$TAG.json')); r=d['roofline']; print('plain', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_ms_min'], r['kernel_ms_median'], r['kernel_ms_max'], d['drift_err'])"
