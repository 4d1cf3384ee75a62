#!/usr/bin/env python3
"""Group a rocprofv3 kernel trace into lavish_txq_frame launches and report
the average frame span (first start -> last end), to compare with bench.py's
event-timed roofline.avg_launch_ms.  A frame is the 2 txq_multi_kernel
dispatches of one step (round 3: one launch per VGPR class) or, in older
traces, the 14 txq_plane_kernel dispatches over 3 streams."""
import csv, sys

def main(path):
    allr = list(csv.DictReader(open(path)))
    rows = [r for r in allr if "txq_multi_kernel" in r["Kernel_Name"]]
    per_frame = 2
    if not rows:
        rows = [r for r in allr if "txq_plane_kernel" in r["Kernel_Name"]]
        per_frame = 14
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    spans = []
    for i in range(0, len(rows) - per_frame + 1, per_frame):
        grp = rows[i:i + per_frame]
        spans.append((max(int(r["End_Timestamp"]) for r in grp) - min(int(r["Start_Timestamp"]) for r in grp)) / 1e6)
    # skip warmup frames (first 2)
    tail = spans[2:] if len(spans) > 4 else spans
    print("frames=%d avg_span_ms=%.4f min=%.4f max=%.4f" % (len(tail), sum(tail) / len(tail), min(tail), max(tail)))

if __name__ == "__main__":
    main(sys.argv[1])
