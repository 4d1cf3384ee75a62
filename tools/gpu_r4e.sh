#!/bin/bash
# round 4 (e): C5 at 4K (received edges checked, captured-graph chunks), the
# third-pass tplmv pin; then timing-only experiments -- C3 with the mv-cost
# loads on one address (e1) / 128-byte-aligned candidate rows (e2); C4 with
# the rdo decision kernels' occupancy (a: 16x16 3 waves, 64x64 1 wave; b: +
# 32x32 1 wave; c: 64x64 1 wave) -- each beside the current build; c5
# wavefront timings
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_shard.py tests/test_gpu_tplmv.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r4e_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4e_pytest.log | tail -1
for rep in 1 2; do
  for v in A e1 e2; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_c3$v.so; fi
    step c3_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4e_c3_$v.log 2>&1
    grep '^{' gpurun_out/r4e_c3_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v', d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for v in A a b c; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_rdo$v.so; fi
    step c4_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4e_c4_$v.log 2>&1
    grep '^{' gpurun_out/r4e_c4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $v', d['ms_per_step'])"
  done
done
for v in A a b; do
  if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_rdo$v.so; fi
  step trace_$v env LAVISH_HIP_LIB=$L LAVISH_FAN_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4e_c4kt_$v -o kt -- python3 -u bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > gpurun_out/r4e_c4kt_$v.log 2>&1
done
for cfg in "4 " "1 " "4 --c5-no-graphs"; do
  set -- $cfg
  step c5w timeout -k 10 300 python -u bench.py --workload c5 --c5-form wavefront --c5-chunks $1 $2 --steps 5 --warmup 2 --no-cpu > gpurun_out/r4e_c5w$1$2.log 2>&1
  grep '^{' gpurun_out/r4e_c5w$1$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 wavefront chunks $1 $2', d['ms_per_step'])"
done
exit 0
