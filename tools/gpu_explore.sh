#!/bin/bash
# exploration pass: per-size C2 timings, C4/C5 bench lines, rocprof of C4
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 180 python -u tools/exp_c2_sizes.py > gpurun_out/c2_sizes.log 2>&1
rc=$?; echo "c2 sizes rc=$rc"; grep -v amdgpu.ids gpurun_out/c2_sizes.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 > gpurun_out/c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; grep -v amdgpu.ids gpurun_out/c4.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; grep -v amdgpu.ids gpurun_out/c5.log | tail -2; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c4" -o kt -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_c4.log" 2>&1
echo "rocprof c4 rc=$?"
exit 0
