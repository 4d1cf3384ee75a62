#!/bin/bash
# Round-3 closing evidence, part 2: C4 VALU counters (profiles/c4_valu.json,
# the default line's c4 roofline) and kernel trace, then the component
# bench lines (tpl, rate, c3sub, c5)
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
cd /tmp && export TMPDIR=/tmp
step pmc_c4_valu timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_c4v" -o p -- python3 "$R/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_c4v.log" 2>&1
step pmc_c4_fetch timeout -k 10 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_c4f" -o p -- python3 "$R/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_c4f.log" 2>&1
step pmc_c4_write timeout -k 10 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_c4w" -o p -- python3 "$R/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_c4w.log" 2>&1
step c4_kt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c4kt" -o kt -- python3 "$R/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/c4kt.log" 2>&1
cd "$R"
step valu python3 tools/valu_summary.py gpurun_out/pmc_c4v 4 gpurun_out/c4_valu.json gpurun_out/pmc_c4f gpurun_out/pmc_c4w
cp gpurun_out/c4_valu.json profiles/c4_valu.json
for wl in c4 tpl rate c3sub c5; do
  step bench_$wl timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --cpu-seconds 6 > gpurun_out/bench_$wl.log 2>&1
  grep '^{' gpurun_out/bench_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', d['ms_per_step'], d['value'], d['roofline'].get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
done
exit 0
