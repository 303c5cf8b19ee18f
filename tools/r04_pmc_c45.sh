#!/bin/bash
# r04 final code: FETCH_SIZE / WRITE_SIZE passes for C4 and C5 (tools/profile_r02.sh), C5 per-residual traffic
# (tools/c5_traffic.py; 3 chunks per residual at the 2^22 default: 0T rows + initial + terminal sets).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/profile_r02.sh "C4 C5" || exit $?
python3 tools/c5_traffic.py gpurun_out/prof_r02/C5 3 | tee gpurun_out/c5_traffic_r04.txt
