#!/bin/bash
# A/B the simulator variants of tools/sim_variants.py on one box: the in-tree build vs
# pde-inverse-problem_amd/_build/variants/*/libpdeinv.so.
R=${GRAFT_REPO_ROOT:-$PWD}
for v in "" $(ls -d $R/pde-inverse-problem_amd/_build/variants/*/ 2>/dev/null); do
  if [ -z "$v" ]; then echo "== in-tree"; timeout -k 10 200 python3 $R/tools/sim_variants.py || exit 1
  else echo "== $(basename $v)"; PDEINV_LIBRARY=$v/libpdeinv.so timeout -k 10 200 python3 $R/tools/sim_variants.py || exit 1; fi
done
