#!/bin/bash
# RealNVP iteration loop on the box: parity tests, throughput (tools/nvp_bench.py), kernel trace.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp.py -k "realnvp or nvp" > gpurun_out/nvp_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/nvp_$TAG.log | tail -22
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/nvp_bench.py --steps 20 > gpurun_out/nvp_bench_$TAG.jsonl 2> gpurun_out/nvp_bench_$TAG.err || exit 11
cat gpurun_out/nvp_bench_$TAG.jsonl
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/nvpprof_$TAG -o run --output-format csv -- python3 $R/tools/nvp_bench.py --steps 5 --warmup 1 > $R/gpurun_out/nvpprof_$TAG.log 2>&1 || exit 12
echo done
