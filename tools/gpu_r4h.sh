#!/bin/bash
# round 4 (h): C3 with one-wave workgroups (default) vs four-wave
# (LAVISH_C3_WPG=4) vs a 5-waves/SIMD build (tools/dbg/lib_c3w5.so); the
# headline; the C5 wavefront's host enqueue time
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_gpu_mcomp.py tests/test_gpu_mcomp_fixtures.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4h_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4h_pytest.log | tail -1
for rep in 1 2; do
  for v in w1 w4 w5; do
    L=aom-av1-lavish_amd/liblavish_hip.so; E=""
    [ $v = w4 ] && E="LAVISH_C3_WPG=4"
    [ $v = w5 ] && L=tools/dbg/lib_c3w5.so
    step c3_$v env $E LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4h_c3_$v.log 2>&1
    grep '^{' gpurun_out/r4h_c3_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v', d['ms_per_step'])"
  done
done
for v in w1 w4; do
  E=""; [ $v = w4 ] && E="LAVISH_C3_WPG=4"
  step rdo_$v env $E timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/r4h_rdo_$v.log 2>&1
  grep '^{' gpurun_out/r4h_rdo_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo $v', d['ms_per_step'], d['legs_ms'], d.get('legs_overlapped_ms'))"
done
for cfg in "4 " "4 --c5-no-graphs"; do
  set -- $cfg
  step c5w timeout -k 10 170 python -u bench.py --workload c5 --c5-form wavefront --c5-chunks $1 $2 --steps 5 --warmup 2 --no-cpu > gpurun_out/r4h_c5w$1$2.log 2>&1
  grep '^{' gpurun_out/r4h_c5w$1$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 wavefront chunks $1 $2', d['ms_per_step'], 'host enqueue', d['host_enqueue_ms_per_step'])"
done
exit 0
