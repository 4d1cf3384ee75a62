#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs of
bench.py) into per-dispatch HBM bytes per kernel and per step, following
/opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]": both counters are in
KB; FETCH_SIZE is doubled on gfx950 (it reports half the bytes of wide
streaming reads).  Writes profiles/pmc_traffic.json.

usage: pmc_summary.py FETCH_DIR WRITE_DIR OUT_JSON"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    # drop the first (warm-up) dispatch of each kernel
    return {k: (sum(v[1:]) / len(v[1:]) if len(v) > 1 else v[0]) for k, v in acc.items()}


def main(fdir, wdir, out):
    f = per_kernel(fdir, "FETCH_SIZE")
    w = per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        if "rocclr" in k:
            continue
        fb = 2.0 * f.get(k, 0.0)
        wb = w.get(k, 0.0)
        kernels[k] = {"fetch_bytes_x2": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb)}
    txq = [v for k, v in kernels.items() if "txq_plane_kernel" in k or "txq_multi_kernel" in k]
    dia = [v for k, v in kernels.items()
           if "diamond_kernel" in k or "diamond_lj_kernel" in k or "ref_tiles_kernel" in k]
    res = {
        "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE in separate passes of "
                  "bench.py; per-dispatch average excluding the first dispatch; FETCH_SIZE x2 "
                  "(gfx950 correction, MI355X_MICROARCH.md HBM section); KB -> bytes",
        "kernels": kernels,
        "frame_hbm_bytes_per_launch": round(sum(v["hbm_bytes"] for v in txq)) if txq else None,
        "diamond_hbm_bytes_per_launch": round(sum(v["hbm_bytes"] for v in dia)) if dia else None,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("frame_hbm_bytes_per_launch", "diamond_hbm_bytes_per_launch")}))


if __name__ == "__main__":
    main(*sys.argv[1:4])
