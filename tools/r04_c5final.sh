#!/bin/bash
# C5 with the 2^22-row chunk default: the multi-rank GPU tests (world-2 C5 caps the chunk at its rows), then
# the C5 bench line twice.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py > gpurun_out/c5f_multirank.log 2>&1 || { tail -30 gpurun_out/c5f_multirank.log; exit 1; }
tail -1 gpurun_out/c5f_multirank.log
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --config C5 --steps 20 --warmup 3 > gpurun_out/c5f_$rep.json 2> gpurun_out/c5f_$rep.err || { tail -20 gpurun_out/c5f_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c5f_$rep.json')); r=d['roofline']; print('C5', d['ms_per_step'], d['value'], r['kernel_ms'], r['kernel_ms_min'], r['kernel_ms_median'], r['kernel_ms_max'], r['frac'], r['achieved'], r['traffic'])"
done
