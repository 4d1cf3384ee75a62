#!/bin/bash
# Inverse-transform A/B: the whole GPU suite and smoke on the new build, then
# the c4 step (and its per-kernel trace) on the base (B) and new (A) builds
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
for v in B A B A; do
  if [ $v = A ]; then L=aom-av1-lavish_amd/liblavish_hip.so; else L=tools/dbg/lib_base.so; fi
  step bench_$v env LAVISH_HIP_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_inv$v.log 2>&1
  grep '^{' gpurun_out/bench_inv$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'])"
done
export TMPDIR=/tmp
step trace timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inv -o inv -- python3 -u bench.py --workload c4 --steps 20 --warmup 5 --no-cpu > gpurun_out/trace_inv.log 2>&1
f=$(ls gpurun_out/prof_inv/*/inv_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && grep -i inv_tile "$f" | cut -c1-200
exit 0
