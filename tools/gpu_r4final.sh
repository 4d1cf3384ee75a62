#!/bin/bash
# round 4 (final): the committed state -- suite, smoke, default bench + traces,
# c4 / tpl / c3 / c5 benches
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
md5sum aom-av1-lavish_amd/liblavish_hip.so
step() { local name=$1; shift; echo "running $name"; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0; }
step suite timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4final_suite.log 2>&1
tail -2 gpurun_out/r4final_suite.log
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4final_smoke.log 2>&1
tail -1 gpurun_out/r4final_smoke.log
step bench timeout -k 10 300 python -u bench.py > gpurun_out/r4final_bench.log 2>&1
grep '^{' gpurun_out/r4final_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d.get('legs_ms'), d['roofline'].get('frac'), d.get('cpu_baseline',{}).get('value'))"
step benchserial timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final_serialkt -o kt -- python3 -u bench.py --serial --no-cpu --steps 20 --warmup 5 > gpurun_out/r4final_serialkt.log 2>&1
grep '^{' gpurun_out/r4final_serialkt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('serial', d['ms_per_step'], d.get('legs_ms'))"
step benchovl timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final_ovlkt -o kt -- python3 -u bench.py --no-cpu --no-c4 --steps 20 --warmup 5 > gpurun_out/r4final_ovlkt.log 2>&1
step c4trace env LAVISH_FAN_STREAMS=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final_c4kt -o kt -- python3 -u bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > gpurun_out/r4final_c4kt.log 2>&1
for w in c4 tpl c3; do
  step b_$w timeout -k 10 200 python -u bench.py --workload $w > gpurun_out/r4final_$w.log 2>&1
  grep '^{' gpurun_out/r4final_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['ms_per_step'], d['value'], d['roofline'].get('frac'), d.get('cpu_baseline',{}).get('value'))"
done
step c5 timeout -k 10 200 python -u bench.py --workload c5 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4final_c5.log 2>&1
grep '^{' gpurun_out/r4final_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['ms_per_step'])"
exit 0
