#!/bin/bash
# C3 A/B on one box: the in-tree build vs tools/dbg/liblavish_c3old.so
# (the eight-jobs DIAMOND kernel before masking the loads of out-of-range
# sites and finished jobs), alternating
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
for v in old new old new old new; do
  if [ $v = new ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/liblavish_c3old.so; fi
  step bench_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c3 --steps 30 --warmup 5 --no-cpu > gpurun_out/bench_c3_$v.log 2>&1
  grep '^{' gpurun_out/bench_c3_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['legs_ms']['c3_diamond'])"
done
exit 0
