#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/pmc_r05
cd /tmp && export TMPDIR=/tmp
for W in 1 2 4 6 8; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc_r05/valu_rate_w$W -o run --output-format csv -- $R/tools/_bin/valu_rate $W \
  > $R/gpurun_out/pmc_r05/valu_rate_w$W.log 2>&1 || exit 1
done
