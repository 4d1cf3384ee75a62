#!/bin/bash
# round 4 (w): C3 grid cap sweep beside C2 (default step); TPL with the known
# centres' ranking loads issued before the above-right wait (P: lib_tplpre)
# vs the committed walk (A)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so tools/dbg/*.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest env LAVISH_HIP_LIB=tools/dbg/lib_tplpre.so timeout -k 10 400 python -u -m pytest tests/test_gpu_tplmv.py tests/test_gpu_tpl.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4w_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4w_pytest.log | tail -1
for rep in 1 2; do
  for v in A P; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_tplpre.so; fi
    step tpl_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload tpl --steps 10 --warmup 3 --no-cpu > gpurun_out/r4w_tpl_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4w_tpl_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tpl $v', d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for g in 0 256 384 512 640 768; do
    step rdo_g$g timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 --c3-wg-cap $g > gpurun_out/r4w_rdo_g${g}_$rep.log 2>&1
    grep '^{' gpurun_out/r4w_rdo_g${g}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo g $g', d['ms_per_step'], d.get('legs_overlapped_ms'))"
  done
done
exit 0
