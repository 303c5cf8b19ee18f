#!/bin/bash
# C4 A/B: serial (separate sums / sums fused into the KMV pass) vs the two-stream pipeline; kernel trace.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-recovery --c4-serial --c4-separate-sums > gpurun_out/c4sep_$TAG.json 2>gpurun_out/c4sep_$TAG.err || exit 11
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-recovery --c4-serial > gpurun_out/c4fus_$TAG.json 2>gpurun_out/c4fus_$TAG.err || exit 12
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-recovery > gpurun_out/c4pipe_$TAG.json 2>gpurun_out/c4pipe_$TAG.err || exit 13
python3 -c "
import json
for f in ('c4sep', 'c4fus', 'c4pipe'):
    j = json.load(open('gpurun_out/%s_$TAG.json' % f))
    print(f, 'ms/step %.3f' % j['ms_per_step'], 'sim %.3f' % j['roofline']['kernel_ms'], 'sums %.3f' % j['mean_path']['ms'], 'res %.3f' % j['residual']['ms'], j['value'])
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4prof_$TAG -o run --output-format csv -- python3 $R/bench.py --config C4 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > $R/gpurun_out/c4prof_$TAG.log 2>&1 || exit 14
python3 $R/tools/kstat_big.py $R/gpurun_out/c4prof_$TAG "sde|kmv|mf_|slab"
