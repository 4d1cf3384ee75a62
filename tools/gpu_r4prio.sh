#!/bin/bash
# round 4: the default step with C2 on a high-priority stream (--c2-priority 1)
# beside C3 vs normal priority
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
for rep in 1 2 3; do
  for p in 0 1; do
    step rdo_p$p timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 --c2-priority $p > gpurun_out/r4prio_p${p}_$rep.log 2>&1
    grep '^{' gpurun_out/r4prio_p${p}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo prio $p', d['ms_per_step'], d.get('legs_overlapped_ms'))"
  done
done
exit 0
