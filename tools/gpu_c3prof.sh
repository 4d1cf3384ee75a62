#!/bin/bash
# C3 leg: kernel-trace stats + the SQ / TA-TCP-TD / TCC counter passes
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
TAG=${TAG:-c3}
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o k -- python3 "$R/bench.py" --workload c3 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/prof_$TAG.log"; exit $rc; }
WL=c3 bash "$R/tools/gpu_pmc_c3.sh"
