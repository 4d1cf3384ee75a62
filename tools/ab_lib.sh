#!/bin/bash
# tools/ab_lib.sh TAG ALT_LIB ROUNDS BENCH_ARGS... -- A/B of two builds of the
# library on one box: `bench.py BENCH_ARGS` alternately with the tree's
# liblavish_hip.so and with ALT_LIB (LAVISH_HIP_LIB), ROUNDS times each;
# prints each run's ms_per_step.  Stops at the first failing run.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; ALT=$2; N=$3; shift 3
for i in $(seq 1 "$N"); do
  for v in cur alt; do
    if [ $v = alt ]; then export LAVISH_HIP_LIB=$ALT; else unset LAVISH_HIP_LIB; fi
    timeout -k 10 300 python3 -u bench.py "$@" > gpurun_out/${TAG}_${v}_$i.log 2>&1 || exit $?
    echo "$v $i $(grep '^{' gpurun_out/${TAG}_${v}_$i.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], (d.get("legs_ms") or {}).get("c2_txq_frame"), (d.get("roofline") or {}).get("frac"))')"
  done
done
