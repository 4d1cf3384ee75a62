#!/bin/bash
# round-3 C4 / rate / TPL changes: their GPU tests, then each bench beside
# the previous build (tools/dbg/liblavish_c4C.so: rdo without the occupancy
# request and the SWAR nz contexts, TPL search without the window-served
# cost list and job prefetch)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 500 python -u -m pytest tests/test_gpu_rdo.py tests/test_gpu_costcoeffs.py tests/test_gpu_tplmv.py tests/test_gpu_tpl.py tests/test_gpu_fullsize.py tests/test_gpu_trellis.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3c.log 2>&1
tail -1 gpurun_out/pytest_r3c.log
for wl in c4 rate tpl; do
  for v in C A C A; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/liblavish_c4C.so; fi
    step bench_${wl}_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_${wl}_$v.log 2>&1
    grep '^{' gpurun_out/bench_${wl}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $v', d['ms_per_step'], d.get('legs_ms', ''))"
  done
done
exit 0
