#!/bin/bash
# TPL leg: parity tests, bench line + kernel-trace stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tpl.py tests/test_gpu_qfacade.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tpl.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_tpl.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload tpl --steps 20 --warmup 5 > gpurun_out/bench_tpl.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_tpl.log; exit $rc; }
grep '^{' gpurun_out/bench_tpl.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_tpl" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload tpl --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_tpl.log" 2>&1; echo "prof rc=$?"
