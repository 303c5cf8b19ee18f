#!/bin/bash
# A/B the C2 bench line: in-tree build vs pde-inverse-problem_amd/_build/variants/<v>/libpdeinv.so, alternating.
cd "$GRAFT_REPO_ROOT"
V=${1:-prio}
for v in base $V base $V base $V; do
  if [ "$v" = base ]; then timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-recovery > gpurun_out/c2ab.json 2>/dev/null || exit 1
  else PDEINV_LIBRARY=$PWD/pde-inverse-problem_amd/_build/variants/$v/libpdeinv.so timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-recovery > gpurun_out/c2ab.json 2>/dev/null || exit 1; fi
  python -c "import json; d=json.load(open('gpurun_out/c2ab.json')); print('$v', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4))"
done
