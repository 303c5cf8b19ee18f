#!/bin/bash
# world-2 C5 bench on one GPU (the multirank test's launch), output to gpurun_out/
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PDEINV_DIST_BACKEND=gloo timeout -k 10 170 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29717 bench.py --gpus 2 --config C5 --steps 2 --warmup 1 --particles 65536 --no-cpu-baseline --no-recovery > gpurun_out/c5w2.out 2> gpurun_out/c5w2.err
rc=$?; echo "rc=$rc"; date; tail -3 gpurun_out/c5w2.out; tail -20 gpurun_out/c5w2.err
