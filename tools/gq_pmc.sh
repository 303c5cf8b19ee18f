#!/bin/bash
# SQ counter passes over the MFMA pair-tile kernels (reference default net 20 x 8, d = 2).
# Usage: bash tools/gq_pmc.sh <tag> [case]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
CASE=${2:-2,2000,1,20,8,2}
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/kmv_mlp_time.py $CASE"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-include-regex kmvq_ -d $R/gpurun_out/q_pmc1_$TAG -o run --output-format csv -- $P > $R/gpurun_out/q_pmc1_$TAG.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC --kernel-include-regex kmvq_ -d $R/gpurun_out/q_pmc2_$TAG -o run --output-format csv -- $P > $R/gpurun_out/q_pmc2_$TAG.log 2>&1 || exit 13
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --kernel-include-regex kmvq_ -d $R/gpurun_out/q_pmc3_$TAG -o run --output-format csv -- $P > $R/gpurun_out/q_pmc3_$TAG.log 2>&1 || exit 14
cd $R && python3 tools/pmc_table.py gpurun_out/q_pmc1_$TAG gpurun_out/q_pmc2_$TAG gpurun_out/q_pmc3_$TAG | tee gpurun_out/q_pmc_$TAG.txt
