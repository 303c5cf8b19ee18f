#!/bin/bash
# Round-3 MLP-residual loop: parity tests, the C5 bench line, the SQ LDS/issue counter pass over the
# MLP kernels, and (optionally) the C3 bench line + its SQ pass. Usage: bash tools/r03_mlp.sh <tag> [c3]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "residual_mlp" > gpurun_out/mlp_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/mlp_$TAG.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || exit 11
cat gpurun_out/c5_$TAG.json
ARGS="--config C5 --steps 2 --warmup 1 --particles 1048576 --no-cpu-baseline --no-recovery"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5prof_$TAG -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/c5prof_$TAG.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SALU --kernel-include-regex mlpf -d $R/gpurun_out/mlp_pmc2_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/mlp_pmc2_$TAG.log 2>&1 || exit 13
if [ "$2" = "c3" ]; then
  cd $R
  timeout -k 10 300 python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline --no-recovery > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err || exit 14
  cat gpurun_out/c3_$TAG.json
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex sde_simulate -d $R/gpurun_out/c3_pmc_$TAG -o run --output-format csv -- python3 $R/bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/c3_pmc_$TAG.log 2>&1 || exit 15
fi
echo done
