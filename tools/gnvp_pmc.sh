#!/bin/bash
# PMC pass over the RealNVP gradient kernel (instruction mix, busy / wave cycles, LDS conflicts).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-include-regex realnvp_grad -d $R/gpurun_out/nvppmc1_$TAG -o run --output-format csv -- python3 $R/tools/nvp_bench.py --steps 2 --warmup 1 --dims 4 > $R/gpurun_out/nvppmc1_$TAG.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --kernel-include-regex realnvp_grad -d $R/gpurun_out/nvppmc2_$TAG -o run --output-format csv -- python3 $R/tools/nvp_bench.py --steps 2 --warmup 1 --dims 4 > $R/gpurun_out/nvppmc2_$TAG.log 2>&1 || exit 13
echo done
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE --kernel-include-regex realnvp_grad -d $R/gpurun_out/nvppmc3_$TAG -o run --output-format csv -- python3 $R/tools/nvp_bench.py --steps 2 --warmup 1 --dims 4 > $R/gpurun_out/nvppmc3_$TAG.log 2>&1 || exit 14
echo done3
