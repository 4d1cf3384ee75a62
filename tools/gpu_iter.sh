#!/bin/bash
# iteration pass: selected GPU tests, then bench workloads (BENCH_WLS)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for wl in ${BENCH_WLS:-rdo}; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_$wl.log | tail -2 | cut -c1-1500
  [ $rc -ne 0 ] && exit $rc
done
exit 0
