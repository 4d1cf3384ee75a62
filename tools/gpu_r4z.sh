#!/bin/bash
# round 4 (z): C4 per-size kernels least work first (LAVISH_RDO_ORDER=1, the
# latency-bound large sizes start beside the small ones) vs most work first
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest env LAVISH_RDO_ORDER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_rdo.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4z_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4z_pytest.log | tail -1
for rep in 1 2 3; do
  for o in 0 1; do
    step c4_o$o env LAVISH_RDO_ORDER=$o timeout -k 10 150 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4z_c4_o${o}_$rep.log 2>&1
    grep '^{' gpurun_out/r4z_c4_o${o}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 order $o', d['ms_per_step'])"
  done
done
step pytest_c3 timeout -k 10 400 python -u -m pytest tests/test_gpu_mcomp.py tests/test_gpu_mcomp_fixtures.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4z_pytest_c3.log 2>&1
grep -E "passed|failed" gpurun_out/r4z_pytest_c3.log | tail -1
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then L=tools/dbg/lib_c3prev.so; else L=aom-av1-lavish_amd/liblavish_hip.so; fi
    step c3_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4z_c3_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4z_c3_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v', d['ms_per_step'])"
    step rdo_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/r4z_rdo_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4z_rdo_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo $v', d['ms_per_step'], d['legs_ms'])"
  done
done
exit 0
