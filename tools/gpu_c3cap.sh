#!/bin/bash
# C3 grid-cap sweep for the overlapped default step (LAVISH_C3_WGS), after the
# motion-search GPU tests
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 300 python -u -m pytest tests/test_gpu_mcomp_fixtures.py tests/test_gpu_fullsize.py tests/test_gpu_tplmv.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
tail -1 gpurun_out/pytest_q.log
for cap in ${CAPS:-0 256 512 768 1024}; do
  step bench_$cap env LAVISH_C3_WGS=$cap timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/bench_cap$cap.log 2>&1
  grep '^{' gpurun_out/bench_cap$cap.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cap $cap', d['ms_per_step'], d.get('legs_ms'), d.get('legs_overlapped_ms'))"
done
exit 0
