#!/bin/bash
# Full GPU pass for profiles/: parity tests, smoke, default bench (+ CPU
# baseline), kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes (separate
# runs), then the C4 bench (+ CPU baseline) and its kernel trace.  Stops at the
# first failure.
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
step bench timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-400
step bench_c4 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --cpu-seconds 8 > gpurun_out/bench_c4.log 2>&1
step bench_inter timeout -k 10 300 python -u bench.py --workload inter --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/bench_inter.log 2>&1
cd /tmp && export TMPDIR=/tmp
step rocprof_inter timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_inter" -o kt -- python3 "$R/bench.py" --workload inter --steps 50 --warmup 5 --no-cpu > "$R/gpurun_out/prof_inter.log" 2>&1
step rocprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o kt -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof.log" 2>&1
step rocprof_c4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c4" -o kt -- python3 "$R/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof_c4.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$R/gpurun_out/pmc_$c" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_$c.log" 2>&1
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE" "$R/gpurun_out/pmc_traffic.json"
exit 0
