#!/bin/bash
# quick iteration: selected GPU tests (TESTS), then bench workloads (WLS)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
if [ -n "$TESTS" ]; then
  step pytest timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
  tail -2 gpurun_out/pytest_q.log
fi
for wl in ${WLS:-}; do
  step bench_$wl timeout -k 10 300 python -u bench.py --workload ${wl%%:*} --steps 20 --warmup 5 --no-cpu ${BARGS:-} > gpurun_out/bench_${wl%%:*}.log 2>&1
  grep '^{' gpurun_out/bench_${wl%%:*}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', d['ms_per_step'], d.get('legs_ms'), d.get('legs_overlapped_ms'), d['roofline'].get('frac'))"
done
exit 0
