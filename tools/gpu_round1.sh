#!/bin/bash
# GPU pass: parity tests, smoke, bench, kernel-trace profile.
# Stops at the first crash/timeout (rc 124/134/137/139); a plain test failure
# (rc 1) does not stop the later steps.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }

timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
fatal $rc && exit $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
fatal $rc && exit $rc

timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
fatal $rc && exit $rc

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o kt -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
exit 0
