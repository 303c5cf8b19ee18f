#!/bin/bash
# r05: MLP residual parity (incl. first-order boundary chunks), then C5 with / without the first-order chain (A/B).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_mirror.py -k "residual_mlp or ou_exact or vs_pairwise_restatement" > gpurun_out/r05_c5_tests.txt 2>&1 || { tail -30 gpurun_out/r05_c5_tests.txt; exit 1; }
tail -2 gpurun_out/r05_c5_tests.txt
for r in 1 2; do
  for fo in 0 1; do
    PDEINV_MLP_FIRST_ORDER=$fo timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline \
      --no-recovery > gpurun_out/r05_c5_fo$fo.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r05_c5_fo$fo.json')); r=d['roofline']; print('first_order=$fo', round(d['ms_per_step'],2), 'residual', round(r['kernel_ms'],2), 'frac', round(r['frac'],4))"
  done
done 2>&1 | tee gpurun_out/r05_c5_fo_ab.txt
timeout -k 10 120 rocprofv3 -L > gpurun_out/r05_counters_list.txt 2>&1 || true
