#!/bin/bash
# PMC passes over the C5 MLP-residual kernels: SQ issue/wait counters (two passes) and L2 hit/miss.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
ARGS="--config C5 --steps 2 --warmup 1 --particles 1048576 --no-cpu-baseline --no-recovery"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "rgemm|wgrad2" -d $R/gpurun_out/mlp_pmc1_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/mlp_pmc1_$TAG.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SALU --kernel-include-regex "rgemm|wgrad2" -d $R/gpurun_out/mlp_pmc2_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/mlp_pmc2_$TAG.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-include-regex "rgemm|wgrad2" -d $R/gpurun_out/mlp_pmc3_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/mlp_pmc3_$TAG.log 2>&1 || exit 14
echo done
