#!/bin/bash
# Output-layer kernel loop: MLP / general-Phi parity tests, C5 A/B (env variants, alternating), kernel trace.
# Usage: bash tools/r03_out.sh <tag> "ENV=.." "ENV=.." ...
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}; shift
R=$PWD
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mirror.py -k "residual_mlp or kmv_mlp or general_phi or kfp_mlp" > gpurun_out/out_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/out_$TAG.log | tail -5
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > gpurun_out/c5ab_$TAG.json 2> gpurun_out/c5ab_$TAG.err || exit 11
    echo "[$v] $(python -c 'import json,sys;r=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print("%.2f ms step, residual %.2f ms, frac %.4f"%(r["ms_per_step"],r["roofline"]["kernel_ms"],r["roofline"]["frac"]))' gpurun_out/c5ab_$TAG.json)" | tee -a gpurun_out/c5ab_$TAG.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5prof_$TAG -o run --output-format csv -- python3 $R/bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery > $R/gpurun_out/c5prof_$TAG.log 2>&1 || exit 12
echo done
