#!/bin/bash
# r05: the first-order two-stream chain (mlp_fused.hip run_chunk_fo2): MLP residual parity, then C5 with it off / on
# (PDEINV_MLP_FO2=0/1, alternating), then a kernel trace of the default build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fo2_prof
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_mirror.py tests/test_gpu_meanfield.py -k "residual_mlp or kmv or vs_pairwise_restatement" \
  > gpurun_out/r05_fo2_tests.txt 2>&1 || { tail -30 gpurun_out/r05_fo2_tests.txt; exit 1; }
tail -2 gpurun_out/r05_fo2_tests.txt
for r in 1 2 3; do
  for fo in 0 1; do
    PDEINV_MLP_FO2=$fo timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline \
      --no-recovery > gpurun_out/r05_c5_fo2_$fo.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r05_c5_fo2_$fo.json')); r=d['roofline']; print('fo2=$fo', round(d['ms_per_step'],2), 'residual', round(r['kernel_ms'],2), 'frac', round(r['frac'],4))"
  done
done 2>&1 | tee gpurun_out/r05_c5_fo2_ab.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fo2_prof -o run --output-format csv -- python3 bench.py --config C5 \
  --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > gpurun_out/r05_fo2_prof.log 2>&1
