#!/bin/bash
# round 4 (n): slotted inverse reading 8 slot counts per workgroup at a
# 4096-workgroup cap (A) vs one count per workgroup at 16 384 (P); suites
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_gpu_inv.py tests/test_gpu_rdo.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4n_pytest.log | tail -1
for rep in 1 2; do
  for v in A P; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_invprev.so; fi
    step c4_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4n_c4_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4n_c4_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $v', d['ms_per_step'])"
  done
done
step c4trace env LAVISH_FAN_STREAMS=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n_c4kt -o kt -- python3 -u bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > gpurun_out/r4n_c4kt.log 2>&1
exit 0
