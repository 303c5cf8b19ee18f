cd "$GRAFT_REPO_ROOT"
for v in base w4 base w4; do
  if [ "$v" = base ]; then timeout -k 10 200 python bench.py --config C3 --steps 20 --warmup 3 --no-cpu-baseline --no-recovery > gpurun_out/c3ab.json 2>/dev/null || exit 1
  else PDEINV_LIBRARY=$PWD/pde-inverse-problem_amd/_build/variants/$v/libpdeinv.so timeout -k 10 200 python bench.py --config C3 --steps 20 --warmup 3 --no-cpu-baseline --no-recovery > gpurun_out/c3ab.json 2>/dev/null || exit 1; fi
  python -c "import json; d=json.load(open('gpurun_out/c3ab.json')); print('$v', round(d['ms_per_step'],3), round(d['standalone_residual']['ms'],3), round(d['simulate_only_ms'],3))"
done
