#!/bin/bash
# Round-3 measurement pass for BASELINE configs C2..C5 on one GPU (MI355X_MICROARCH.md HBM/rocprofv3 recipe):
#   bench line; rocprofv3 --kernel-trace --stats; FETCH_SIZE and WRITE_SIZE in SEPARATE --pmc passes
#   restricted to the config's dominant kernels. Output: gpurun_out/prof_r03/<C>/...
# Usage: bash tools/profile_r03.sh "C2 C3 C4 C5"
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_r03
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CONFIGS=${1:-"C2 C3 C4 C5"}
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-recovery"
for C in $CONFIGS; do
  case $C in
    C2|C3) RX="sde_simulate";;
    C4) RX="sde_simulate|kmv_moments_weights|mf_sums";;
    C5) RX="sde_simulate|mlpf|mlp_loss|gather_random|rgemm|wgrad";;
  esac
  mkdir -p $OUT/$C
  timeout -k 10 300 python3 $R/bench.py --config $C --steps 10 --warmup 3 --no-recovery > $OUT/$C/bench.json 2> $OUT/$C/bench.err || exit 11
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$C/trace -o run --output-format csv -- python3 $R/bench.py --config $C $ARGS > $OUT/$C/trace.log 2>&1 || exit 12
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d $OUT/$C/fetch -o run --output-format csv -- python3 $R/bench.py --config $C $ARGS > $OUT/$C/fetch.log 2>&1 || exit 13
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d $OUT/$C/write -o run --output-format csv -- python3 $R/bench.py --config $C $ARGS > $OUT/$C/write.log 2>&1 || exit 14
  echo "$C done"
done
