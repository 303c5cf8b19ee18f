#!/bin/bash
# r05 mid-round GPU pass: full GPU suite, training iteration records, C3 line (VALU issue block), the C4 strong-
# scaling N = 1 point on the rebased KMV pass, and the C2 PairGram / QuadGram A/B on this box.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05_mid_gtest.txt 2>&1 \
  || { tail -40 $O/r05_mid_gtest.txt; exit 1; }
tail -2 $O/r05_mid_gtest.txt
timeout -k 10 300 python tools/train_bench.py --iters 200 --warmup 20 --out $O/r05_train_bench.jsonl > /dev/null 2> $O/r05_train_bench.err || exit 2
timeout -k 10 200 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-recovery > $O/r05_bench_c3.json 2>/dev/null || exit 3
timeout -k 10 300 python bench.py --config C4 --scaling strong --steps 5 --warmup 2 --no-cpu-baseline --no-recovery > $O/r05_c4_strong_n1.json 2>/dev/null || exit 4
for r in 1 2 3; do
  for v in default quad6; do
    if [ $v = default ]; then timeout -k 10 120 python tools/sim_time.py | sed "s/^/$v /" || exit 5
    else PDEINV_LIBRARY=$PWD/pde-inverse-problem_amd/_build/var/$v.so timeout -k 10 120 python tools/sim_time.py | sed "s/^/$v /" || exit 5; fi
  done
done > $O/r05_quad_ab_box2.txt 2>&1
cat $O/r05_quad_ab_box2.txt
