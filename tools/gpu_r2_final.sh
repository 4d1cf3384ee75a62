#!/bin/bash
# Round-2 evidence pass: the whole -m gpu suite, smoke, the default bench line
# (+ CPU baseline), the component workloads (c4, inter, pixel, warp, compound,
# tpl, rate), kernel-trace stats of the default / c4 / warp runs, and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
step bench timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
for wl in c4 c3sub inter pixel warp compound tpl rate; do
  step bench_$wl timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --cpu-seconds 8 > gpurun_out/bench_$wl.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
step rocprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o kt -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof.log" 2>&1
step rocprof_c4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c4" -o kt -- python3 "$R/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof_c4.log" 2>&1
step rocprof_warp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_warp" -o kt -- python3 "$R/bench.py" --workload warp --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof_warp.log" 2>&1
step rocprof_compound timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_compound" -o kt -- python3 "$R/bench.py" --workload compound --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof_compound.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$R/gpurun_out/pmc_$c" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-c4 > "$R/gpurun_out/pmc_$c.log" 2>&1
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE" "$R/gpurun_out/pmc_traffic.json"
exit 0
