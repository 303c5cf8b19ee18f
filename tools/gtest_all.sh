#!/bin/bash
# Full GPU test suite + smoke on the box. Usage: bash tools/gtest_all.sh <tag> [pytest -k expr]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "$K" > gpurun_out/gtest_$TAG.log 2>&1
else
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gtest_$TAG.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/gtest_$TAG.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 9
