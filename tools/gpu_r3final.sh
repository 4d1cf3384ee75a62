#!/bin/bash
# Round-3 closing evidence, part 1: the whole -m gpu suite, smoke, the
# default bench line (CPU baseline included), a serial kernel trace (C2
# frame span + C3 duration) and the HBM counter passes of the default step
# (FETCH_SIZE and WRITE_SIZE in separate runs -> profiles/pmc_traffic.json)
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp
step pmc_fetch timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmcf" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-c4 --serial > "$R/gpurun_out/pmcf.log" 2>&1
step pmc_write timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmcw" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-c4 --serial > "$R/gpurun_out/pmcw.log" 2>&1
cd "$R"
step pmc_summary python3 tools/pmc_summary.py gpurun_out/pmcf gpurun_out/pmcw gpurun_out/pmc_traffic.json
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
step bench timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
grep '^{' gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('legs_ms'), d.get('legs_overlapped_ms'), d['roofline'].get('frac'), d['roofline'].get('traffic'))"
cd /tmp
step rocprof_serial timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_serial" -o kt -- python3 "$R/bench.py" --serial --steps 10 --warmup 2 --no-cpu --no-c4 > "$R/gpurun_out/prof_serial.log" 2>&1
exit 0
