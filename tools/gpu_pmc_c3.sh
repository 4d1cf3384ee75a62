#!/bin/bash
# PMC passes over the C3 (diamond) leg alone; each pass its own run
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
i=0
WL=${WL:-c3}
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TC_STALL_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" ${EXTRA_SETS:-}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/pmc_${TAG:-$WL}$i" -o p -- python3 "$R/bench.py" --workload $WL --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_${TAG:-$WL}$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  case $rc in 0) ;; *) tail -5 "$R/gpurun_out/pmc_${TAG:-$WL}$i.log"; exit $rc;; esac
done
exit 0
