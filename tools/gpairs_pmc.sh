#!/bin/bash
# Kernel stats + PMC passes over the general-Phi KMV pair kernels (reference default net 20 x 8, d = 2).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
CASE=${2:-2,2000,1,20,8,2}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pairs_tr_$TAG -o run --output-format csv -- python3 $R/tools/kmv_mlp_time.py $CASE > $R/gpurun_out/pairs_tr_$TAG.log 2>&1 || exit 11
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-include-regex kmvp_ -d $R/gpurun_out/pairs_pmc1_$TAG -o run --output-format csv -- python3 $R/tools/kmv_mlp_time.py $CASE > $R/gpurun_out/pairs_pmc1_$TAG.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --kernel-include-regex kmvp_ -d $R/gpurun_out/pairs_pmc2_$TAG -o run --output-format csv -- python3 $R/tools/kmv_mlp_time.py $CASE > $R/gpurun_out/pairs_pmc2_$TAG.log 2>&1 || exit 13
echo done
