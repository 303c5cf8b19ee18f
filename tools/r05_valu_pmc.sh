#!/bin/bash
# r05: SQ calibration of tools/valu_rate.hip (issue cycles per VALU instruction as SQ_ACTIVE_INST_VALU counts them,
# one dispatch per opcode), the unit tools/c3_valu_model.py prices the C3 step loop in.
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/pmc_r05
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc_r05/valu_rate -o run --output-format csv -- $R/tools/_bin/valu_rate 3 \
  > $R/gpurun_out/pmc_r05/valu_rate_pmc.log 2>&1
