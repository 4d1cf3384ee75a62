#!/usr/bin/env python3
"""Per-step VALU instruction count of a bench workload from one rocprofv3
--pmc pass (SQ_INSTS_VALU [+ GRBM_GUI_ACTIVE]) of `bench.py --workload WL
--steps S --warmup W --no-cpu`: per kernel, the average SQ_INSTS_VALU per
dispatch and the dispatches per step (all dispatches / (S + W)); the step's
total is what bench.py's VALU roofline divides by the live step time.  The
HBM bytes per step (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md) are added
when those passes are given.

usage: valu_summary.py VALU_DIR STEPS_TOTAL OUT_JSON [FETCH_DIR WRITE_DIR]"""
import collections
import csv
import glob
import json
import os
import sys


def counters(d, name):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name and "rocclr" not in r["Kernel_Name"]:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main(vdir, steps_total, out, fdir=None, wdir=None):
    steps_total = int(steps_total)
    v = counters(vdir, "SQ_INSTS_VALU")
    kernels, tot = {}, 0.0
    for k, vals in sorted(v.items()):
        per_step = len(vals) / steps_total
        avg = sum(vals[1:]) / len(vals[1:]) if len(vals) > 1 else vals[0]
        kernels[k] = {"dispatches_per_step": per_step, "valu_instr_per_dispatch": round(avg)}
        tot += avg * per_step
    res = {"source": "rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU, %d steps incl. warmup; "
                     "per-dispatch averages exclude each kernel's first dispatch" % steps_total,
           "valu_instr_per_step": round(tot), "kernels": kernels}
    if fdir and wdir:
        f, w = counters(fdir, "FETCH_SIZE"), counters(wdir, "WRITE_SIZE")
        hbm = 0.0
        for k in set(f) | set(w):
            for src, mul in ((f.get(k, []), 2.0), (w.get(k, []), 1.0)):
                if src:
                    avg = sum(src[1:]) / len(src[1:]) if len(src) > 1 else src[0]
                    hbm += mul * avg * 1024.0 * len(src) / steps_total
        res["hbm_bytes_per_step"] = round(hbm)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"valu_instr_per_step": res["valu_instr_per_step"],
                      "hbm_bytes_per_step": res.get("hbm_bytes_per_step")}))


if __name__ == "__main__":
    main(*sys.argv[1:])
