#!/bin/bash
# C3 iteration: motion parity subset, bench c3 / c3sub, one instruction-mix PMC pass
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-it}
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "mcomp or diamond or subpel or bigdia or full_pixel or c3" > gpurun_out/pytest_$TAG.log 2>&1
tail -2 gpurun_out/pytest_$TAG.log
for wl in c3 c3sub; do
  step $wl timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_${wl}_$TAG.log 2>&1
  grep '^{' gpurun_out/bench_${wl}_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['legs_ms'], d['c3'])"
done
cd /tmp && export TMPDIR=/tmp
step pmc timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_mix_$TAG" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c3 --steps 3 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/pmc_mix_$TAG.log" 2>&1
exit 0
