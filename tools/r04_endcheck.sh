#!/bin/bash
# End-of-round check on the final code: full GPU suite + smoke, the default bench line, then the F1W4 A/B
# (tools/r04_f1w4.sh: parity under PDEINV_MLP_F1W4=1 and C5 alternating).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gtest_all.sh r04z || exit $?
timeout -k 10 300 python3 bench.py > gpurun_out/bench_r04z.json 2> gpurun_out/bench_r04z.err || exit 21
cat gpurun_out/bench_r04z.json
bash tools/r04_f1w4.sh
