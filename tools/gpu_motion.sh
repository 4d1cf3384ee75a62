#!/bin/bash
# Motion-search GPU pass: fixture parity, motion tests, C3 / C3+subpel bench legs.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_gpu_mcomp_fixtures.py tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "mcomp or diamond or subpel or bigdia or full_pixel or c3" \
  > gpurun_out/pytest_motion.log 2>&1
tail -3 gpurun_out/pytest_motion.log
step c3 timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_c3.log 2>&1
grep -v amdgpu.ids gpurun_out/bench_c3.log | tail -1 | cut -c1-600
step c3sub timeout -k 10 300 python -u bench.py --workload c3sub --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_c3sub.log 2>&1
grep -v amdgpu.ids gpurun_out/bench_c3sub.log | tail -1 | cut -c1-600
exit 0
