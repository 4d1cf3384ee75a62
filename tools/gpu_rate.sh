#!/bin/bash
# coefficient-rate bench line + kernel-trace stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload rate --steps 10 --warmup 3 > gpurun_out/bench_rate.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_rate.log; exit $rc; }
grep '^{' gpurun_out/bench_rate.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_rate" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload rate --steps 5 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_rate.log" 2>&1; echo "prof rc=$?"
