#!/bin/bash
# C3 leg kernel trace (tiles build + search), default grid
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c3kt" -o kt -- python3 "$R/bench.py" --workload c3 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/c3kt.log" 2>&1
echo "kt rc=$?"
python3 - <<'PY'
import csv, os
R = os.environ["GRAFT_REPO_ROOT"]
for r in csv.DictReader(open(R + "/gpurun_out/c3kt/kt_kernel_stats.csv")):
    print(r["Name"][:50], r["Calls"], r["AverageNs"], r["MinNs"])
PY
