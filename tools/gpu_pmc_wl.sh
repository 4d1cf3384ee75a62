#!/bin/bash
# PMC passes over one bench workload (WL), each counter set its own run,
# kernel-trace only (no sys / runtime trace)
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
i=0
WL=${WL:-inter}
for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_SETS:-}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/pmc_$WL$i" -o p -- python3 "$R/bench.py" --workload $WL --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_$WL$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  case $rc in 0) ;; *) tail -5 "$R/gpurun_out/pmc_$WL$i.log"; exit $rc;; esac
done
exit 0
