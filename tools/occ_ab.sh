#!/bin/bash
# A/B of simulator build variants on the C2 bench line: bash tools/occ_ab.sh <variant>... (libraries in
# pde-inverse-problem_amd/_build/var/<variant>.so, "base" = the in-tree library), two alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
V=pde-inverse-problem_amd/_build/var
for rnd in 0 1; do
for L in base "$@"; do
  if [ $L = base ]; then unset PDEINV_LIBRARY; else export PDEINV_LIBRARY=$V/$L.so; fi
  timeout -k 10 120 python3 bench.py --config C2 --steps 20 --warmup 5 --no-cpu-baseline --no-recovery > gpurun_out/ab_$L.json 2>gpurun_out/ab_$L.err
  rc=$?; [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -3 gpurun_out/ab_$L.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$L.json')); r=d['roofline']; print('$rnd $L', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],4), round(r.get('frac_of_box_write_ceiling',0),3))"
done
done
