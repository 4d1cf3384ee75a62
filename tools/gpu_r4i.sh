#!/bin/bash
# round 4 (i): the C2 32-point class on a second stream (LAVISH_TXQ_FRAME_MODE=2
# A/B); slot-per-workgroup inverse lists (tests + c4); TPL counters
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_gpu_inv.py tests/test_gpu_rdo.py tests/test_gpu_fullsize.py tests/test_gpu_txq.py tests/test_gpu_fixtures.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4i_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4i_pytest.log | tail -1
step pytest2 env LAVISH_TXQ_FRAME_MODE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_txq.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4i_pytest2.log 2>&1
grep -E "passed|failed" gpurun_out/r4i_pytest2.log | tail -1
for rep in 1 2; do
  for m in 1 2; do
    step rdo_m$m env LAVISH_TXQ_FRAME_MODE=$m timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/r4i_rdo_m$m.log 2>&1
    grep '^{' gpurun_out/r4i_rdo_m$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo mode $m', d['ms_per_step'], d['legs_ms'], d.get('legs_overlapped_ms'))"
    step c2_m$m env LAVISH_TXQ_FRAME_MODE=$m timeout -k 10 150 python -u bench.py --workload c2 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4i_c2_m$m.log 2>&1
    grep '^{' gpurun_out/r4i_c2_m$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 mode $m', d['ms_per_step'])"
  done
done
step c4 timeout -k 10 150 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4i_c4.log 2>&1
grep '^{' gpurun_out/r4i_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['ms_per_step'])"
step c4trace env LAVISH_FAN_STREAMS=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i_c4kt -o kt -- python3 -u bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > gpurun_out/r4i_c4kt.log 2>&1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  step tplpmc$i timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/r4i_tplpmc$i -o p -- python3 bench.py --workload tpl --steps 3 --warmup 1 --no-cpu > gpurun_out/r4i_tplpmc$i.log 2>&1
done
exit 0
