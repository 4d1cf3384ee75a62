#!/bin/bash
# round 4 (v): default step with C2 held to fewer workgroups per CU by an LDS
# pad (LAVISH_C2_LDS_PAD) and C3's grid capped (LAVISH_C3_WGS) beside it
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
for pad in 0 16384 45056; do
  for g in 0 512 1024; do
    step rdo_p${pad}_g$g env LAVISH_C2_LDS_PAD=$pad LAVISH_C3_WGS=$g timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/r4v_rdo_p${pad}_g${g}.log 2>&1
    grep '^{' gpurun_out/r4v_rdo_p${pad}_g${g}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo pad $pad g $g', d['ms_per_step'], d.get('legs_overlapped_ms'), d['legs_ms']['c2_txq_frame'])"
  done
done
exit 0
