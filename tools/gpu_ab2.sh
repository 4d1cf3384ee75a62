#!/bin/bash
# A/B on one box: (1) C2's store policy in the default overlapped step -- the
# in-tree build (sc1 write-through stores) vs tools/dbg/liblavish_c2nt.so
# (nontemporal stores); (2) the C3 leg vs tools/dbg/liblavish_c3old.so
# (loads of out-of-range sites / finished jobs not masked).  The txq and
# motion GPU tests run first on the in-tree build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 400 python -u -m pytest tests/test_gpu_txq.py tests/test_gpu_fixtures.py tests/test_gpu_mcomp_fixtures.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab2.log 2>&1
tail -1 gpurun_out/pytest_ab2.log
for v in nt sc1 nt sc1 nt sc1; do
  if [ $v = sc1 ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/liblavish_c2nt.so; fi
  step rdo_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/bench_rdo_$v.log 2>&1
  grep '^{' gpurun_out/bench_rdo_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo $v', d['ms_per_step'], d['legs_ms']['c2_txq_frame'], d['legs_ms']['c3_diamond'], d['legs_overlapped_ms'])"
done
exit 0
