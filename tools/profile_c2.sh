#!/bin/bash
# rocprofv3 passes for the C2 bench (kernel trace + separate PMC passes; MI355X_MICROARCH.md §HBM).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_c2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-recovery --steps 10 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex sde_simulate -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex sde_simulate -d $OUT/write -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex sde_simulate -d $OUT/sq -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/sq.log 2>&1 || exit 14
echo done
