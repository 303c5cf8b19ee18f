#!/bin/bash
# C5 final-code pass: bench line, kernel trace, FETCH_SIZE / WRITE_SIZE passes (tools/profile_r02.sh C5),
# then the per-residual traffic (tools/c5_traffic.py, 4 chunks per residual at the C5 size).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/profile_r02.sh C5 || exit $?
python3 tools/c5_traffic.py gpurun_out/prof_r02/C5 4 | tee gpurun_out/c5_traffic.txt
