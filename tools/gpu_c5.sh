#!/bin/bash
# C5 sharding checks on one GPU: the rect / 2-rank tests, then the c5 bench
# (world 1) in both forms
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_fullsize.py -k "c5 or shard" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1
grep -E 'PASS|FAIL|passed|failed' gpurun_out/pytest_c5.log | tail -8
for form in band wavefront; do
  step bench_$form timeout -k 10 200 python -u bench.py --workload c5 --c5-form $form --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c5_$form.log 2>&1
  grep '^{' gpurun_out/bench_c5_$form.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$form', d['ms_per_step'], d['config']['parallelism'])"
done
exit 0
