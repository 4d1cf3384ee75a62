#!/bin/bash
# round 4 (y): counters of the C4 decision kernels (where the 4..16-point
# kernels' non-issue cycles go), one pass per counter set, fan-out off
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  [ $i -eq 3 ] && for k in "rdo_kernel<16, 16" "rdo_kernel<8, 8" "rdo_kernel<4, 4"; do echo "== $k (passes 1-2)"; python3 tools/pmc_kernel.py "$k" gpurun_out/r4y_pmc1 gpurun_out/r4y_pmc2; done
  step pmc$i env LAVISH_FAN_STREAMS=1 timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/r4y_pmc$i -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4y_pmc$i.log 2>&1
done
for k in "rdo_kernel<16, 16" "rdo_kernel<8, 8" "rdo_kernel<4, 4" "rdo_kernel<32, 32" "rdo_kernel<64, 64"; do
  echo "== $k"; python3 tools/pmc_kernel.py "$k" gpurun_out/r4y_pmc1 gpurun_out/r4y_pmc2 gpurun_out/r4y_pmc3
done
exit 0
