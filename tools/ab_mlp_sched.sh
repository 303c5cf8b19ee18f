#!/bin/bash
# A/B of the rgemm / wgrad2 schedule variants (PDEINV_MLP_SCHED) on the C5 residual: kernel trace per variant.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
cd /tmp && export TMPDIR=/tmp
for V in ${2:-0 1 2 3}; do
  PDEINV_MLP_SCHED=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_${TAG}_v$V -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/ab_${TAG}_v$V.log 2>&1 || exit 12
  python3 $R/tools/kstat_big.py $R/gpurun_out/ab_${TAG}_v$V "mlpf|mlp_loss" | sed "s/^/v$V /"
done
