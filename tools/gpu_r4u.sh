#!/bin/bash
# round 4 (u): TPL plain walk with pipelined polls and the known centres'
# ranking loads issued before the above-right wait (A) vs without (O:
# lib_c3site, the committed walk + the C3 site offsets); search suites
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so tools/dbg/*.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 500 python -u -m pytest tests/test_gpu_tplmv.py tests/test_gpu_tpl.py tests/test_gpu_mcomp.py tests/test_gpu_mcomp_fixtures.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4u_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4u_pytest.log | tail -1
for rep in 1 2; do
  for v in A O; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_c3site.so; fi
    step tpl_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload tpl --steps 10 --warmup 3 --no-cpu > gpurun_out/r4u_tpl_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4u_tpl_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tpl $v', d['ms_per_step'], d.get('legs_ms'))"
  done
done
exit 0
