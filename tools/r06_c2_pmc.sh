#!/bin/bash
# Round 6, VERDICT r05 item 5: why the C2 simulator stores at ~5.3-5.5 TB/s against a ~6.9 TB/s fill of the same
# buffer. (1) the store-pattern probe (tools/store_pattern.hip: the simulator's store shape with no arithmetic, and
# flat fills); (2) counter passes over the default C2 bench command, which runs the simulator launches and then
# write_ceiling()'s torch fill of the same trajectory buffer: the L2's memory-side write requests (TCC_EA0_WRREQ,
# 64-byte ones, their stall cycles), the L1 -> L2 write requests, and the SQ's store-issue and wait cycles.
# Every pass under its own limit; a fatal status ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/r06_c2pmc
mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1 ;; esac; }
timeout -k 10 120 $R/tools/_bin/store_pattern > $OUT/store_pattern.txt 2>&1; rc=$?; echo "store_pattern rc=$rc"; fatal $rc probe
cat $OUT/store_pattern.txt
cd /tmp && export TMPDIR=/tmp
A2="--config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-recovery"
RX="sde_simulate|FillFunctor|fill"
i=0
for P in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_WRITE_sum GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
         "TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
         "TCC_BUSY_sum TCC_REQ_sum TCC_TAG_STALL_sum TCC_STREAMING_REQ_sum GRBM_GUI_ACTIVE" \
         "TA_BUSY_avr TA_FLAT_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d $OUT/p$i -o run --output-format csv \
    -- python3 $R/bench.py $A2 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc ($P)"; fatal $rc pass$i
done
python3 $R/tools/pmc_table.py $OUT 2>/dev/null | head -60 || true
