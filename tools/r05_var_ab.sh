#!/bin/bash
# r05: C5 A/B of variant libraries (tools/build_var.sh) against the default build, one box: parity subset per library,
# bench lines and a kernel trace each (tools/r05_c5_trace.sh). Usage: bash tools/r05_var_ab.sh <tag> <variant>...
cd "$GRAFT_REPO_ROOT"; TAG=$1; shift
bash tools/r05_c5_trace.sh ${TAG}_def || exit 1
for v in "$@"; do
  bash tools/r05_c5_trace.sh ${TAG}_$v PDEINV_LIBRARY=$GRAFT_REPO_ROOT/pde-inverse-problem_amd/_build/var/$v.so || exit 1
done
bash tools/r05_c5_trace.sh ${TAG}_defb || exit 1
python3 - "$TAG" "$@" <<'PY'
import csv, glob, sys
tag = sys.argv[1]; tags = [tag + '_def'] + [tag + '_' + v for v in sys.argv[2:]] + [tag + '_defb']
res = {}
for t in tags:
    f = glob.glob('gpurun_out/prof_%s/**/run_kernel_stats.csv' % t, recursive=True)[0]
    res[t] = {x['Name'][19:70]: float(x['AverageNs']) / 1e6 for x in csv.DictReader(open(f))}
print('kernel'.ljust(52), '  '.join(t[len(tag) + 1:].rjust(7) for t in tags))
for n in sorted(res[tags[0]], key=lambda k: -res[tags[0]][k])[:16]:
    print(n.ljust(52), '  '.join('%7.3f' % res[t].get(n, 0) for t in tags))
PY
