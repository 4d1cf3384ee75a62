#!/bin/bash
# round 4 (d): timing-only experiments -- C3 with the mv-cost loads on one
# address (e1) / with 128-byte-aligned candidate rows (e2); C4 with the rdo
# decision kernels' occupancy requests (a: 16x16 3 waves, 64x64 1 wave;
# b: + 32x32 1 wave; c: 64x64 1 wave) -- each beside the current build
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
for rep in 1 2; do
  for v in A e1 e2; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_c3$v.so; fi
    step c3_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4d_c3_$v.log 2>&1
    grep '^{' gpurun_out/r4d_c3_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v', d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for v in A a b c; do
    if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_rdo$v.so; fi
    step c4_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4d_c4_$v.log 2>&1
    grep '^{' gpurun_out/r4d_c4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $v', d['ms_per_step'])"
  done
done
export TMPDIR=/tmp
for v in A a b; do
  if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_rdo$v.so; fi
  step trace_$v env LAVISH_HIP_LIB=$L LAVISH_FAN_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d_c4kt_$v -o kt -- python3 -u bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > gpurun_out/r4d_c4kt_$v.log 2>&1
done
exit 0
