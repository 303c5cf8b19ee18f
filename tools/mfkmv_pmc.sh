#!/bin/bash
# SQ counter passes over the C4 fused simulate + KMV stamp sums (sde_mf_kmv_kernel) beside the simulate + next sums
# (sde_simulate_kernel), through tools/mfkmv_time.py's child (MFKMV_ONLY picks the runs). Run via gpurun from the
# repo root: bash tools/mfkmv_pmc.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
R=$PWD
TAG=${1:?tag}
P=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
   "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
   "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_WAVE_CYCLES SQ_WAVES")
i=0
for C in "${P[@]}"; do
  i=$((i + 1))
  (cd /tmp && export TMPDIR=/tmp MFKMV_ONLY=fused_no_traj,sim_next_no_traj && timeout -s KILL 120 rocprofv3 --pmc $C \
    --kernel-include-regex "sde_mf_kmv|sde_simulate" -d $R/gpurun_out/pmc_$TAG/p$i -o run --output-format csv \
    -- python3 $R/tools/mfkmv_time.py --child > $R/gpurun_out/pmc_${TAG}_p$i.log 2>&1)
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc ;; esac
done
python3 tools/pmc_table.py gpurun_out/pmc_$TAG
