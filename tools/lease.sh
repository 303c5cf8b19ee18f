#!/bin/bash
# One driver for the GPU-box measurements (run through gpurun from the repo root). Every GPU step runs under its
# own time limit; a fatal status (time limit, abort, segfault) ends the script and nothing further touches the GPU.
#
#   bash tools/lease.sh tests <tag> [pytest -k expr]    full GPU suite (or a -k subset) + smoke
#   bash tools/lease.sh bench <tag> <C2|C3|C4|C5>... [-- extra bench.py args]
#                                                        bench lines, one JSON file per config
#   bash tools/lease.sh check <tag>                      the default bench command under rocprofv3 --kernel-trace
#                                                        --stats (same run: the printed line and its trace; the
#                                                        timed dispatches picked out by tools/trace_timed.py), then
#                                                        the same command without the profiler
#   bash tools/lease.sh prof <tag> <C2|C3|C4|C5>...      rocprofv3 --kernel-trace --stats per config
#   bash tools/lease.sh pmc <tag> <config> <regex> "<counters>" ["<counters>" ...]
#                                                        one --pmc pass per counter group over bench.py --config
#   bash tools/lease.sh final <tag>                      tests + check + C3/C4/C5 lines + their profiles + RealNVP
#                                                        + the pair recipe + the C5 traffic passes
#   bash tools/lease.sh extra <tag>                      the last three alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
R=$PWD
MODE=${1:?mode}
TAG=${2:?tag}
shift 2
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1 ;; esac; }

run_tests() {
  local K=${1:-}
  if [ -n "$K" ]; then
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "$K" \
      > gpurun_out/gtest_$TAG.log 2>&1
  else
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
      > gpurun_out/gtest_$TAG.log 2>&1
  fi
  local rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/gtest_$TAG.log | tail -8
  fatal $rc tests
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; fatal $rc smoke
  [ $rc -eq 0 ] || exit 9
}

run_bench() {
  local extra=() cfgs=()
  while [ $# -gt 0 ]; do
    if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi
    cfgs+=("$1"); shift
  done
  for c in "${cfgs[@]}"; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 "${extra[@]}" \
      > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
    local rc=$?; echo "bench $c rc=$rc"; fatal $rc bench_$c
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$c.json')); \
print('$c', d['value'], d['unit'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d['roofline'].get('frac'))" || true
  done
}

run_check() {
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG \
    -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 \
    > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err)
  local rc=$?; echo "profiled bench rc=$rc"; fatal $rc check_prof; [ $rc -eq 0 ] || exit 31
  python3 tools/trace_timed.py gpurun_out/prof_$TAG gpurun_out/bench_prof_$TAG.json > gpurun_out/trace_timed_$TAG.json \
    || exit 32
  cat gpurun_out/trace_timed_$TAG.json
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_plain_$TAG.json \
    2> gpurun_out/bench_plain_$TAG.err
  rc=$?; echo "plain bench rc=$rc"; fatal $rc check_plain; [ $rc -eq 0 ] || exit 33
  python3 -c "import json; d=json.load(open('gpurun_out/bench_plain_$TAG.json')); r=d['roofline']; \
print('plain', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_ms_min'], r['kernel_ms_median'], \
r['kernel_ms_max'], d.get('drift_err'))"
}

run_prof() {
  for c in "$@"; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d $R/gpurun_out/prof_${TAG}_$c -o run --output-format csv -- python3 $R/bench.py --config $c --steps 10 \
      --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_${TAG}_$c.json 2> $R/gpurun_out/prof_${TAG}_$c.err)
    local rc=$?; echo "prof $c rc=$rc"; fatal $rc prof_$c; [ $rc -eq 0 ] || exit 41
  done
}

run_pmc() {
  local cfg=$1 rx=$2; shift 2
  local i=0
  for P in "$@"; do
    i=$((i + 1))
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$rx" \
      -d $R/gpurun_out/pmc_${TAG}/p$i -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 3 \
      --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/pmc_${TAG}_p$i.log 2>&1)
    local rc=$?; echo "pmc pass $i rc=$rc ($P)"; fatal $rc pmc_$i
  done
  python3 tools/pmc_table.py gpurun_out/pmc_${TAG} || true
}

case $MODE in
  tests) run_tests "${1:-}" ;;
  bench) run_bench "$@" ;;
  check) run_check ;;
  prof) run_prof "$@" ;;
  pmc) run_pmc "$@" ;;
  final|extra)
    if [ $MODE = final ]; then
      run_tests
      run_check
      run_bench C3 C4 C5
      run_prof C3 C4 C5
    fi
    timeout -k 10 200 python3 tools/nvp_bench.py --steps 30 --warmup 5 --dims 2,4 > gpurun_out/final_${TAG}_nvp.jsonl 2>&1
    rc=$?; echo "nvp rc=$rc"; fatal $rc nvp
    timeout -k 10 300 python3 tools/kmv_mlp_time.py 2,5000,1,20,8,2 > gpurun_out/final_${TAG}_pairs.jsonl 2>&1
    rc=$?; echo "pairs rc=$rc"; fatal $rc pairs
    RX="sde_simulate|mlpf|mlp_loss|gather_random|fillBuffer"
    for c in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "$RX" \
        -d $R/gpurun_out/prof_${TAG}_c5pmc/$(echo $c | tr A-Z a-z | cut -d_ -f1) -o run --output-format csv \
        -- python3 $R/bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery \
        > $R/gpurun_out/prof_${TAG}_c5pmc_$c.log 2>&1)
      rc=$?; echo "c5 $c rc=$rc"; fatal $rc c5_$c
    done
    python3 tools/c5_traffic.py gpurun_out/prof_${TAG}_c5pmc 3 | tee gpurun_out/final_${TAG}_c5_traffic.txt
    ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
