#!/bin/bash
# round 4 (f): decimated entropy-cost tables in the C3 search (A/B through
# LAVISH_C3_MVDEC), the headline step, and the C5 wavefront with each chunk a
# replayed HIP graph (captured after one uncaptured run)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 700 python -u -m pytest tests/test_gpu_inv.py tests/test_gpu_fixtures.py tests/test_gpu_rdo.py tests/test_gpu_mcomp.py tests/test_gpu_mcomp_fixtures.py tests/test_gpu_fullsize.py tests/test_gpu_tplmv.py tests/test_gpu_tpl.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4f_pytest.log | tail -1
for rep in 1 2; do
  for v in 0 1; do
    step c3_dec$v env LAVISH_C3_MVDEC=$v timeout -k 10 150 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4f_c3_dec$v.log 2>&1
    grep '^{' gpurun_out/r4f_c3_dec$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 dec$v', d['ms_per_step'])"
  done
done
for v in 0 1; do
  step rdo_dec$v env LAVISH_C3_MVDEC=$v timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > gpurun_out/r4f_rdo_dec$v.log 2>&1
  grep '^{' gpurun_out/r4f_rdo_dec$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rdo dec$v', d['ms_per_step'], d['legs_ms'], d.get('legs_overlapped_ms'))"
done
for cfg in "4 " "1 " "4 --c5-no-graphs"; do
  set -- $cfg
  step c5w timeout -k 10 170 python -u bench.py --workload c5 --c5-form wavefront --c5-chunks $1 $2 --steps 5 --warmup 2 --no-cpu > gpurun_out/r4f_c5w$1$2.log 2>&1
  grep '^{' gpurun_out/r4f_c5w$1$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 wavefront chunks $1 $2', d['ms_per_step'])"
done
step c5band timeout -k 10 170 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu > gpurun_out/r4f_c5band.log 2>&1
grep '^{' gpurun_out/r4f_c5band.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 band', d['ms_per_step'])"
for v in B A; do
  if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_base.so; fi
  step c4_$v env LAVISH_HIP_LIB=$L timeout -k 10 150 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4f_c4_$v.log 2>&1
  grep '^{' gpurun_out/r4f_c4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $v', d['ms_per_step'])"
done
step c4trace env LAVISH_FAN_STREAMS=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f_c4kt -o kt -- python3 -u bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > gpurun_out/r4f_c4kt.log 2>&1
exit 0
