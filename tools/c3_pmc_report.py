#!/usr/bin/env python3
"""C3 counter report: the SQ / TA-TCP-TD / TCC passes of tools/gpu_pmc_c3.sh
plus the kernel-trace stats for one tag, reduced to per-dispatch values and
derived ratios for diamond_kernel (the last dispatch of each pass).

usage: c3_pmc_report.py TAG [TAG ...]  ->  JSON on stdout"""
import collections
import csv
import glob
import json
import sys


def counters(d, needle="diamond_kernel"):
    out = {}
    for path in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            if needle in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        out.update({k: v[-1] for k, v in acc.items()})
    return out


def stats(d, needle="diamond_kernel"):
    for path in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if needle in r["Name"]:
                return {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
    return {}


def report(tag, root="gpurun_out"):
    c = {}
    for i in (1, 2, 3):
        c.update(counters("%s/pmc_%s%d" % (root, tag, i)))
    s = stats("%s/prof_%s" % (root, tag))
    waves = c.get("SQ_WAVES", 1.0)
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    derived = {
        "wave_quad_cycles_per_wave": wc / waves,
        "frac_wait_any": c.get("SQ_WAIT_ANY", 0) / wc if wc else None,
        "frac_wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
        "frac_active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
        "salu_per_wave": c.get("SQ_INSTS_SALU", 0) / waves,
        "vmem_rd_per_wave": c.get("SQ_INSTS_VMEM_RD", 0) / waves,
        "clock_GHz": (c["GRBM_GUI_ACTIVE"] / 8 / (s["avg_ms"] * 1e-3) / 1e9)
        if "GRBM_GUI_ACTIVE" in c and s else None,
        "tcp_hit_rate": 1 - c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"]
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in c else None,
        "tcc_hit_rate": c["TCC_HIT_sum"] / c["TCC_REQ_sum"] if "TCC_REQ_sum" in c else None,
    }
    if "GRBM_GUI_ACTIVE" in c:
        busy = c["GRBM_GUI_ACTIVE"] / 8 * 256  # CU-cycles (8 XCDs x 32 CUs)
        derived["ta_busy_frac"] = c.get("TA_TA_BUSY_sum", 0) / busy
    return {"tag": tag, "kernel_stats": s, "counters": c, "derived": derived}


if __name__ == "__main__":
    print(json.dumps([report(t) for t in sys.argv[1:]], indent=1))
