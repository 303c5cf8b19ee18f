#!/bin/bash
# Round-end check on one box: full GPU suite + smoke (tools/gtest_all.sh), then the default bench line.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
bash tools/gtest_all.sh $TAG || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.err || exit 21
cat gpurun_out/bench_default_$TAG.json
