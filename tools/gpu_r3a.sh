#!/bin/bash
# Round-3 first pass: the -m gpu suite, smoke, the default bench line, a
# serial kernel trace (C2 frame span + C3 diamond duration), the C4 VALU /
# HBM counter passes (profiles/c4_valu.json), then the trellis A/B
# (class-branching helpers, tools/dbg/build_trellis_cb.sh).  Stops at the
# first failing GPU step except the last (an experiment).
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
step bench timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
step rocprof_serial timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_serial" -o kt -- python3 "$R/bench.py" --serial --steps 10 --warmup 2 --no-cpu --no-c4 > "$R/gpurun_out/prof_serial.log" 2>&1
step pmc_c4_valu timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_c4v" -o p -- python3 "$R/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_c4v.log" 2>&1
step pmc_c4_fetch timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_c4f" -o p -- python3 "$R/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_c4f.log" 2>&1
step pmc_c4_write timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_c4w" -o p -- python3 "$R/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_c4w.log" 2>&1
cd "$R"
python3 tools/valu_summary.py gpurun_out/pmc_c4v 4 gpurun_out/c4_valu.json gpurun_out/pmc_c4f gpurun_out/pmc_c4w
LAVISH_HIP_LIB=tools/dbg/liblavish_cb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_trellis.py tests/test_gpu_pins.py tests/test_gpu_costcoeffs.py -k "optimize_b or cost" -q --timeout 120 --timeout-method thread > gpurun_out/trellis_cb.log 2>&1
echo "trellis_cb rc=$?"
tail -3 gpurun_out/trellis_cb.log
exit 0
