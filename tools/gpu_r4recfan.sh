#!/bin/bash
# round 4: C4 reconstruction with the sizes' inverse launches over the fan-out
# streams (A: the library) vs one after another on the caller's stream (B:
# tools/dbg/lib_recserial.so, the previous commit); rdo / full-size suites
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so tools/dbg/*.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 500 python -u -m pytest tests/test_gpu_rdo.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py tests/test_gpu_inv.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4recfan_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4recfan_pytest.log | tail -1
for rep in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_recserial.so; fi
    step c4_$v$rep env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4recfan_c4_$v$rep.log 2>&1
    grep '^{' gpurun_out/r4recfan_c4_$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $v', d['ms_per_step'])"
  done
done
step valu timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU --output-format csv -d gpurun_out/r4valu_v -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4valu_v.log 2>&1
step fetch timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4valu_f -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4valu_f.log 2>&1
step write timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4valu_w -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4valu_w.log 2>&1
step summary python3 tools/valu_summary.py gpurun_out/r4valu_v 4 gpurun_out/c4_valu.json gpurun_out/r4valu_f gpurun_out/r4valu_w
cat gpurun_out/c4_valu.json | head -5
exit 0
