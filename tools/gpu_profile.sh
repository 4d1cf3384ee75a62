#!/bin/bash
# Profiling pass for profiles/: kernel-trace stats of the default bench step,
# then FETCH_SIZE and WRITE_SIZE in separate PMC passes (no sys/runtime trace).
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o kt -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -1 "$R/gpurun_out/prof.log"
[ $rc -ne 0 ] && exit $rc
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$R/gpurun_out/pmc_$c" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc_$c.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE" "$R/gpurun_out/pmc_traffic.json"
exit 0
