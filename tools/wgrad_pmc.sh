#!/bin/bash
# C5 bench line + two SQ counter passes over the layer-2 weight-gradient kernels (wgrad_l1 / wgrad2).
# Usage: bash tools/wgrad_pmc.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
R=$PWD
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || exit 11
python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5_$TAG.json').read().strip().splitlines()[-1]); print('C5 kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
ARGS="--config C5 --steps 2 --warmup 1 --particles 1048576 --no-cpu-baseline --no-recovery"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD --kernel-include-regex wgrad -d $R/gpurun_out/wpmc1_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/wpmc1_$TAG.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_ACTIVE_INST_MISC --kernel-include-regex wgrad -d $R/gpurun_out/wpmc2_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/wpmc2_$TAG.log 2>&1 || exit 14
cd $R && python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
for p in ("wpmc1", "wpmc2"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/{p}_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:70]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(p, k, ", ".join(f"{c}={x:.4g}" for c, x in sorted(v.items())))
PY
