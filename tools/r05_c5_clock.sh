#!/bin/bash
# r05: the clock and the matrix-pipe occupancy of the C5 residual's kernels (one SQ + GRBM pass): effective clock =
# GRBM_GUI_ACTIVE / 8 / duration, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / 8).
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/pmc_r05
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "mlpf|mlp_loss" -d $R/gpurun_out/pmc_r05/c5_clock -o run --output-format csv \
  -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/pmc_r05/c5_clock.log 2>&1
