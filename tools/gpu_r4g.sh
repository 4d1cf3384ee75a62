#!/bin/bash
# round 4 (g): the whole GPU suite; C5 wavefront over 4 streams (graphs,
# event dependencies); TPL with / without the wavefront waits (timing-only
# build: what the row handoffs cost); C4 counters (VALU + HBM passes ->
# profiles/c4_valu.json); the default bench with its kernel trace
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r4g_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4g_pytest.log | tail -1
for ch in 4 1; do
  step c5w$ch timeout -k 10 170 python -u bench.py --workload c5 --c5-form wavefront --c5-chunks $ch --steps 5 --warmup 2 --no-cpu > gpurun_out/r4g_c5w$ch.log 2>&1
  grep '^{' gpurun_out/r4g_c5w$ch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 wavefront streams chunks $ch', d['ms_per_step'])"
done
for rep in 1 2; do
  for v in A t1; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_tpl1.so; fi
    step tpl_$v env LAVISH_HIP_LIB=$L timeout -k 10 170 python -u bench.py --workload tpl --steps 10 --warmup 3 --no-cpu > gpurun_out/r4g_tpl_$v.log 2>&1
    grep '^{' gpurun_out/r4g_tpl_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tpl $v', d['ms_per_step'], d.get('legs_ms'))"
  done
done
i=0
for set in "SQ_INSTS_VALU GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  step c4pmc$i timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/r4g_c4pmc$i -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4g_c4pmc$i.log 2>&1
done
step bench timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4g_bench.log 2>&1
grep '^{' gpurun_out/r4g_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo', d['ms_per_step'], d['roofline']['frac'], d['c4']['ms_per_frame'], d['c4']['roofline'])"
step trace timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g_kt -o kt -- python3 -u bench.py --steps 20 --warmup 5 --serial --no-cpu --no-c4 > gpurun_out/r4g_kt.log 2>&1
exit 0
