#!/bin/bash
# PMC passes over a short bench run (counters in separate passes; no sys/runtime trace)
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_SETS:-}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/pmc$i" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  case $rc in 0) ;; *) tail -5 "$R/gpurun_out/pmc$i.log"; exit $rc;; esac
done
exit 0
