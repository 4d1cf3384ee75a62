#!/bin/bash
# C4 occupancy A/B: the rdo GPU tests on variant A, then the c4 step on A
# (2 waves for 512+ coefficients incl. 64-point, 4 for 16x16), B (64-point
# sizes left at 1 wave) and C (no request: the previous build)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 400 python -u -m pytest tests/test_gpu_rdo.py tests/test_gpu_fullsize.py -k "rdo or c4" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c4occ.log 2>&1
tail -1 gpurun_out/pytest_c4occ.log
for v in C A C A; do
  if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/liblavish_c4$v.so; fi
  step bench_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_c4$v.log 2>&1
  grep '^{' gpurun_out/bench_c4$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'])"
done
exit 0
