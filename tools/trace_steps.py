#!/usr/bin/env python3
"""Timeline of repeated C4 steps from a rocprofv3 --kernel-trace CSV: the
kernels (in start order) are split into steps after each occurrence of the
step's last kernel (default recon_sb_kernel), and per kernel name the median
start offset / end offset from the step's start and duration are printed,
plus the median step span and the median gap between steps (us).
usage: trace_steps.py KERNEL_TRACE_CSV [last_kernel_substring] [skip_steps]"""
import csv
import statistics
import sys


def short(name):
    name = name.replace("void ", "").replace("lavish::(anonymous namespace)::", "")
    return name.replace("lavish::", "").split("(")[0]


def main(path, last="recon_sb", skip=5):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
          for r in rows]
    steps, cur = [], []
    for k in ks:
        cur.append(k)
        if last in k[0]:
            steps.append(cur)
            cur = []
    steps = steps[skip:] if len(steps) > skip + 1 else steps
    per = {}
    spans, gaps = [], []
    for i, st in enumerate(steps):
        t0 = min(s for _, s, _ in st)
        spans.append((max(e for _, _, e in st) - t0) / 1e3)
        if i + 1 < len(steps):
            gaps.append((steps[i + 1][0][1] - max(e for _, _, e in st)) / 1e3)
        for n, s, e in st:
            per.setdefault(n, []).append(((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
    print("steps %d, split after %s" % (len(steps), last))
    print("median step span %.1f us, median gap to next step %.1f us"
          % (statistics.median(spans), statistics.median(gaps) if gaps else 0.0))
    for n, v in sorted(per.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
        print("  %-55s x%-3d start %7.1f end %7.1f dur %7.1f" % (
            n[:55], len(v) // max(1, len(steps)), statistics.median(x[0] for x in v),
            statistics.median(x[1] for x in v), statistics.median(x[2] for x in v)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "recon_sb",
         int(sys.argv[3]) if len(sys.argv) > 3 else 5)
