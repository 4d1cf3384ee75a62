#!/bin/bash
# Evidence pass: HBM write ceiling microbench + C4 VALU / memory counters
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/microbench/hbm_write_bw.hip -o /tmp/hbm_write_bw || exit 1
timeout -k 10 120 /tmp/hbm_write_bw > gpurun_out/hbm_write_bw.txt 2>&1; rc=$?; echo "hbm_write_bw rc=$rc"; [ $rc -ne 0 ] && exit $rc
tail -3 gpurun_out/hbm_write_bw.txt
WL=c4 bash tools/gpu_pmc_wl.sh
