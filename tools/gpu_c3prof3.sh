#!/bin/bash
# C3 kernel trace + address-path counters (separate passes)
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step kt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c3kt" -o kt -- python3 "$R/bench.py" --workload c3 --steps 10 --warmup 2 --no-cpu ${BARGS:-} > "$R/gpurun_out/c3kt.log" 2>&1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  step pmc$i timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/c3pmc$i" -o p -- python3 "$R/bench.py" --workload c3 --steps 3 --warmup 1 --no-cpu ${BARGS:-} > "$R/gpurun_out/c3pmc$i.log" 2>&1
done
exit 0
