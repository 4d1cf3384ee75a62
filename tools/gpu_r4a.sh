#!/bin/bash
# round 4 (a): the C4 reconstruction from the chosen coded blocks only --
# GPU suite, then the c4 step A/B against the round-3 build
# (tools/dbg/lib_base.so), its kernel trace; then the C3 counter passes
# (diamond_lj_kernel: TA / SQ wait / VALU / L2) the verdict asked for
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1
tail -1 gpurun_out/r4a_pytest.log
for v in B A B A; do
  if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_base.so; fi
  step bench_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4a_c4_$v.log 2>&1
  grep '^{' gpurun_out/r4a_c4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $v', d['ms_per_step'])"
done
step trace timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4a_c4kt -o kt -- python3 -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4a_c4kt.log 2>&1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" \
           "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  step c3pmc$i timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/r4a_c3pmc$i -o p -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4a_c3pmc$i.log 2>&1
done
exit 0
