#!/bin/bash
# r05 counter passes (separate rocprofv3 --pmc runs, MI355X_MICROARCH.md §rocprofv3 slots):
#   C3: two SQ passes — the VALU instruction classes of the fused simulate + GMM residual launch and its VALU
#       issue cycles (SQ_ACTIVE_INST_VALU, quad-cycles) against the kernel's cycles (GRBM_GUI_ACTIVE / 8);
#   C2: FETCH_SIZE and WRITE_SIZE of the headline simulator launch on the current build (roofline.traffic).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/pmc_r05
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A3="--config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery"
A2="--config C2 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT64 \
  SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex sde_simulate \
  -d $OUT/c3_sq1 -o run --output-format csv -- python3 $R/bench.py $A3 > $OUT/c3_sq1.log 2>&1 || exit 11
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex sde_simulate \
  -d $OUT/c3_sq2 -o run --output-format csv -- python3 $R/bench.py $A3 > $OUT/c3_sq2.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex sde_simulate -d $OUT/c2_fetch -o run \
  --output-format csv -- python3 $R/bench.py $A2 > $OUT/c2_fetch.log 2>&1 || exit 13
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex sde_simulate -d $OUT/c2_write -o run \
  --output-format csv -- python3 $R/bench.py $A2 > $OUT/c2_write.log 2>&1 || exit 14
echo pmc done
