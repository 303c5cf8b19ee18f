#!/bin/bash
# Kernel trace of the C5 bench (timing only, no parity tests), optionally a second trace with <VAR>=0 on
# the same box. Usage: bash tools/c5_trace.sh <tag> [VAR]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R=$PWD; TAG=${1:-x}; VAR=$2
cd /tmp && export TMPDIR=/tmp
show() {
python3 -c "
import csv
rows=list(csv.DictReader(open('$R/gpurun_out/c5prof_$1/run_kernel_stats.csv')))
print('$1 total MLP+sim ms per call-set:', round(sum(float(r['TotalDurationNs']) for r in rows)/1e6/3, 2))
for r in rows[:6]: print(r['Name'][:90], r['Calls'], r['AverageNs'])
"
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5prof_$TAG -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/c5prof_$TAG.log 2>&1 || exit 13
show $TAG
if [ -n "$VAR" ]; then
  export $VAR=0
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5prof_${TAG}_off -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/c5prof_${TAG}_off.log 2>&1 || exit 14
  show ${TAG}_off
fi
