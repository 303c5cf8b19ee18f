#!/bin/bash
# wgrad2 / wgrad_o with buffer-descriptor B loads (in-tree library): the full GPU suite, then the C5 A/B against
# the previous mlp_fused (var library given as $1).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/wgbuf_test.log 2>&1 || { tail -30 gpurun_out/wgbuf_test.log; exit 1; }
tail -1 gpurun_out/wgbuf_test.log
bash tools/ab_cfg.sh wgbuf C5 ${1:-mfold.so}
