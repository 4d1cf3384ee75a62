#!/bin/bash
# round 4 (c): the C3 search with every candidate load of a step in flight
# (range-checked buffer loads) -- search tests, then rdo / c3 A/B against
# the round-3 build, C3 counters
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_gpu_mcomp.py tests/test_gpu_mcomp_fixtures.py tests/test_gpu_fullsize.py tests/test_gpu_tplmv.py tests/test_gpu_tpl.py tests/test_gpu_subpel.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4c_pytest.log | tail -1
for wl in c3 rdo; do
  for v in B A B A; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_base.so; fi
    step bench_${wl}_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/r4c_${wl}_$v.log 2>&1
    grep '^{' gpurun_out/r4c_${wl}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $v', d['ms_per_step'], d.get('legs_ms'), d.get('legs_overlapped_ms'))"
  done
done
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" \
           "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  step c3pmc$i timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/r4c_c3pmc$i -o p -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4c_c3pmc$i.log 2>&1
done
exit 0
