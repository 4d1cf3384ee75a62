#!/bin/bash
# round 4: refresh profiles/c4_valu.json (per-step VALU count + PMC HBM bytes
# of the c4 workload), one counter set per rocprofv3 pass
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step valu timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU --output-format csv -d gpurun_out/r4valu_v -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4valu_v.log 2>&1
step fetch timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4valu_f -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4valu_f.log 2>&1
step write timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4valu_w -o p -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4valu_w.log 2>&1
step summary python3 tools/valu_summary.py gpurun_out/r4valu_v 4 gpurun_out/c4_valu.json gpurun_out/r4valu_f gpurun_out/r4valu_w
cat gpurun_out/c4_valu.json | head -5
exit 0
