#!/bin/bash
# Round 6: C4 fused simulate + KMV stamp sums — parity tests, then the C4 bench under both schedules.
# Usage: bash tools/r06_c4.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1 ;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_meanfield.py -x -q --timeout 200 --timeout-method thread \
  -k "mf_kmv or mf_next or kmv_moments or pairwise_golden" > gpurun_out/r06_${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_${TAG}_tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
for sch in simkmv sim simkmv sim; do
  timeout -k 10 200 python3 bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-recovery --c4-schedule $sch \
    > gpurun_out/r06_${TAG}_c4_$sch.json 2> gpurun_out/r06_${TAG}_c4_$sch.err
  rc=$?; echo "bench $sch rc=$rc"; fatal $rc bench
  python3 -c "import json; d=json.load(open('gpurun_out/r06_${TAG}_c4_$sch.json')); print('$sch', d['ms_per_step'], d['roofline']['kernel_ms'] if 'kernel_ms' in d['roofline'] else d['roofline'].get('achieved'), d.get('residual',{}).get('ms'))" || true
done
