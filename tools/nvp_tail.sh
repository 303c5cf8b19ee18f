cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for s in 294912 320000 393216; do
  timeout -k 10 100 python3 tools/nvp_bench.py --steps 30 --warmup 5 --dims 4 --samples $s | tee -a gpurun_out/nvp_tail.jsonl || exit 1
done
