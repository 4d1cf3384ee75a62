#!/bin/bash
# round 4 (p): TPL speculative walk with global-memory ranking SADs (no prefilled
# windows) vs the same walk without speculation (lib_tplnospec): tests,
# phase clock, bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so tools/dbg/*.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 400 python -u -m pytest tests/test_gpu_tplmv.py tests/test_gpu_tpl.py tests/test_gpu_mcomp.py tests/test_gpu_mcomp_fixtures.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4p_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4p_pytest.log | tail -1
echo running tplprof; env LAVISH_HIP_LIB=tools/dbg/lib_tplprof.so timeout -k 10 120 python -u tools/tpl_prof.py 5 > gpurun_out/r4p_tplprof.log 2>&1; rc=$?; echo tplprof rc=$rc; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
tail -1 gpurun_out/r4p_tplprof.log
for rep in 1 2; do
  for v in A N; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_tplnospec.so; fi
    step tpl_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload tpl --steps 10 --warmup 3 --no-cpu > gpurun_out/r4p_tpl_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4p_tpl_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tpl $v', d['ms_per_step'], d.get('legs_ms'))"
  done
done
exit 0
