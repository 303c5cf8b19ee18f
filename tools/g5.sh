cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_pairs -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kmv_mlp_time.py 2,5000,1,20,8,2 > $GRAFT_REPO_ROOT/gpurun_out/prof_pairs.log 2>&1
echo "rc=$?"; head -8 $GRAFT_REPO_ROOT/gpurun_out/prof_pairs/run_kernel_stats.csv | cut -c1-220
