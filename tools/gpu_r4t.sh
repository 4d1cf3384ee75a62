#!/bin/bash
# round 4 (t): C3 walk with per-step site offsets (B: lib_c3site) vs the
# per-site tile_off (A): search tests with B, c3 and default-bench A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so tools/dbg/*.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest env LAVISH_HIP_LIB=tools/dbg/lib_c3site.so timeout -k 10 400 python -u -m pytest tests/test_gpu_mcomp.py tests/test_gpu_mcomp_fixtures.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4t_pytest.log | tail -1
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_c3site.so; fi
    step c3_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4t_c3_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4t_c3_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v', d['ms_per_step'])"
    step rdo_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/r4t_rdo_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4t_rdo_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo $v', d['ms_per_step'], d['legs_ms'])"
  done
done
exit 0
