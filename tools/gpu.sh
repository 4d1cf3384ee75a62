#!/bin/bash
# tools/gpu.sh TAG STAGE [STAGE ...] -- the stages of one gpurun call.
#
# Every stage runs under its own time limit and writes under
# gpurun_out/TAG_*; the first stage that fails (fault, abort, time limit)
# ends the call -- nothing else touches the GPU after it.  Arguments of a
# stage are comma-separated (commas become spaces).
#
#   suite                 the whole GPU suite (pytest -m gpu)
#   test=EXPR             pytest -m gpu -k EXPR   (EXPR commas -> spaces)
#   file=PATH             pytest -m gpu PATH
#   smoke                 __graft_entry__.smoke()
#   bench=ARGS            python bench.py ARGS; prints the line's summary
#   kt=NAME=ARGS          rocprofv3 --kernel-trace --stats of bench.py ARGS
#   pmc=NAME=CTRS=ARGS    one rocprofv3 --pmc pass (CTRS comma-separated)
#   traffic=NAME=ARGS     FETCH_SIZE and WRITE_SIZE passes of bench.py ARGS
#                         + tools/pmc_summary.py -> gpurun_out/TAG_NAME_traffic.json
#   py=SCRIPT=ARGS        python SCRIPT ARGS (a tool that uses the GPU)
#
# e.g. gpurun -- bash tools/gpu.sh r5a suite smoke bench= kt=serial=--serial,--no-cpu
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
shift
md5sum aom-av1-lavish_amd/liblavish_hip.so
sp() { echo "${1//,/ }"; }
run() {  # run NAME LIMIT CMD...: stops the call on a failure
  local name=$1 lim=$2
  shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
summ() {  # the JSON line of a bench log, summarised
  grep '^{' "$1" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
r = d.get('roofline') or {}
print('  ms/step', d.get('ms_per_step'), 'value', d.get('value'), 'frac', r.get('frac'),
      'legs', d.get('legs_ms'), 'ovl', d.get('legs_overlapped_ms'),
      'cpu', (d.get('cpu_baseline') or {}).get('value'),
      'c4', (d.get('c4') or {}).get('ms_per_frame'))
for k in ('c5', 'c5_emulation', 'c3'):
    if k in d: print('  ', k, json.dumps(d[k])[:600])
"
}
n=0
for st in "$@"; do
  n=$((n + 1))
  kind=${st%%=*}
  rest=${st#*=}
  [ "$rest" = "$st" ] && rest=""
  case $kind in
    suite)
      run suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_suite.log 2>&1
      tail -2 gpurun_out/${TAG}_suite.log ;;
    test)
      run test$n 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -k "$(sp "$rest")" > gpurun_out/${TAG}_test$n.log 2>&1
      tail -3 gpurun_out/${TAG}_test$n.log ;;
    file)
      run file$n 600 python -u -m pytest $(sp "$rest") -m gpu -x -v --timeout 300 \
        --timeout-method thread > gpurun_out/${TAG}_file$n.log 2>&1
      tail -3 gpurun_out/${TAG}_file$n.log ;;
    smoke)
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > gpurun_out/${TAG}_smoke.log 2>&1
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    bench)
      run bench$n 400 python -u bench.py $(sp "$rest") > gpurun_out/${TAG}_bench$n.log 2>&1
      echo "  bench $(sp "$rest")"; summ gpurun_out/${TAG}_bench$n.log ;;
    kt)
      name=${rest%%=*}; args=${rest#*=}
      run kt_$name 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/${TAG}_kt_$name -o kt -- python3 -u bench.py $(sp "$args") \
        > gpurun_out/${TAG}_kt_$name.log 2>&1
      summ gpurun_out/${TAG}_kt_$name.log ;;
    pmc)
      name=${rest%%=*}; r2=${rest#*=}; ctrs=${r2%%=*}; args=${r2#*=}
      run pmc_$name 200 rocprofv3 --kernel-trace --pmc $(sp "$ctrs") --output-format csv \
        -d gpurun_out/${TAG}_pmc_$name -o p -- python3 -u bench.py $(sp "$args") \
        > gpurun_out/${TAG}_pmc_$name.log 2>&1 ;;
    traffic)
      name=${rest%%=*}; args=${rest#*=}
      for c in FETCH_SIZE WRITE_SIZE; do
        run ${c}_$name 200 rocprofv3 --kernel-trace --pmc $c --output-format csv \
          -d gpurun_out/${TAG}_${c}_$name -o p -- python3 -u bench.py $(sp "$args") \
          > gpurun_out/${TAG}_${c}_$name.log 2>&1
      done
      python3 tools/pmc_summary.py gpurun_out/${TAG}_FETCH_SIZE_$name \
        gpurun_out/${TAG}_WRITE_SIZE_$name gpurun_out/${TAG}_${name}_traffic.json ;;
    py)
      name=${rest%%=*}; args=${rest#*=}
      run py$n 400 python3 -u "$name" $(sp "$args") > gpurun_out/${TAG}_py$n.log 2>&1
      tail -5 gpurun_out/${TAG}_py$n.log ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
exit 0
