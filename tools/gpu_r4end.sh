#!/bin/bash
# round 4 end: whole GPU suite, smoke and the default bench on the final library
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step suite timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4end_suite.log 2>&1
tail -2 gpurun_out/r4end_suite.log
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4end_smoke.log 2>&1
tail -1 gpurun_out/r4end_smoke.log
step bench timeout -k 10 300 python -u bench.py > gpurun_out/r4end_bench.log 2>&1
grep '^{' gpurun_out/r4end_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d.get('legs_ms'), d['roofline'].get('frac'), d.get('cpu_baseline',{}).get('value'), d['c4']['ms_per_frame'])"
exit 0
