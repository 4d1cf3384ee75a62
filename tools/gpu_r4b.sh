#!/bin/bash
# round 4 (b): slotted reconstruction job lists (no atomics / memset), the
# TPL timeout handling, C5 at 4K -- GPU suite, c4 A/B against the round-3
# build, the c4 kernel trace (serialized: one fan stream), c5 wavefront at
# world 1
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1
tail -1 gpurun_out/r4b_pytest.log
for v in B A B A; do
  if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_base.so; fi
  step bench_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4b_c4_$v.log 2>&1
  grep '^{' gpurun_out/r4b_c4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $v', d['ms_per_step'], d['roofline'].get('frac'))"
done
step trace env LAVISH_FAN_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b_c4kt -o kt -- python3 -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4b_c4kt.log 2>&1
for ch in 4 1; do
  step c5w$ch timeout -k 10 300 python -u bench.py --workload c5 --c5-form wavefront --c5-chunks $ch --steps 5 --warmup 2 --no-cpu > gpurun_out/r4b_c5w$ch.log 2>&1
  grep '^{' gpurun_out/r4b_c5w$ch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 wavefront chunks $ch', d['ms_per_step'])"
done
exit 0
