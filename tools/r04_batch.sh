#!/bin/bash
# Round-4 measurement batch on one box. Every step runs under its own time limit; an ordinary failure
# (a test or a script returning 1..3) is recorded and the batch goes on, but a time limit, abort or
# segfault (124 / 137 / 134 / 139) ends the batch there. Usage: bash tools/r04_batch.sh <tag> [steps]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-x}
STEPS=${2:-tests,check,pairs,pairs_pmc,c4,train,isa}
R=$PWD
LOG=gpurun_out/batch_$TAG.txt
: > $LOG
step() {  # step <name> <command...>
  local name=$1; shift
  case ",$STEPS," in *",$name,"*) ;; *) return 0 ;; esac
  local t0=$SECONDS
  "$@"
  local rc=$?
  echo "step $name rc=$rc $((SECONDS - t0)) s" | tee -a $LOG
  case $rc in 124|134|137|139) echo "fatal rc in step $name: stopping" | tee -a $LOG; exit $rc ;; esac
  return 0
}
if [ "${GTEST_K:-}" = all ]; then
  step tests bash tools/gtest_all.sh $TAG
else
  step tests bash tools/gtest_all.sh $TAG "${GTEST_K:-multirank or accuracy or general_phi or kmv_non or partial_s or residual_mlp}"
fi
step check bash tools/r04_check.sh $TAG skip-tests
pairs_time() {
  timeout -k 10 300 python3 tools/kmv_mlp_time.py 2,5000,1,20,8,2 2,2000,3,20,8,2 2,5000,1,20,8,3 > gpurun_out/q_time_$TAG.jsonl 2>&1 || return $?
  cat gpurun_out/q_time_$TAG.jsonl
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/q_tr_$TAG -o run \
     --output-format csv -- python3 $R/tools/kmv_mlp_time.py 2,5000,1,20,8,2 > $R/gpurun_out/q_tr_$TAG.log 2>&1) || return $?
  grep -E "kmvq|kmvp" gpurun_out/q_tr_$TAG/run_kernel_stats.csv | cut -d, -f1-4
}
step pairs pairs_time
step pairs_pmc bash tools/gq_pmc.sh $TAG
step c4 bash tools/r04_c4.sh $TAG
step train timeout -k 10 400 python3 tools/train_bench.py --out gpurun_out/train_$TAG.jsonl
isa() {
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/isa_rate.hip -o /tmp/isa_rate_$TAG 2> /dev/null || return 2
  timeout -k 10 60 /tmp/isa_rate_$TAG | tee gpurun_out/isa_rate_$TAG.txt
}
step isa isa
step nvp_pmc bash tools/gnvp_pmc.sh $TAG
nvp_time() { timeout -k 10 200 python3 tools/nvp_bench.py --steps 30 --warmup 5 --dims 2,4 | tee gpurun_out/nvp_$TAG.jsonl; }
step nvp nvp_time
nvp_trace() {
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/nvp_tr_$TAG -o run \
     --output-format csv -- python3 $R/tools/nvp_bench.py --steps 20 --warmup 5 --dims 4 > $R/gpurun_out/nvp_tr_$TAG.log 2>&1) || return $?
  cut -d, -f1-4 gpurun_out/nvp_tr_$TAG/run_kernel_stats.csv | cut -c1-150
}
step nvp_trace nvp_trace
step nvp_ab bash tools/ab_nvp.sh $TAG ${NVP_VARS:-}
cat $LOG
