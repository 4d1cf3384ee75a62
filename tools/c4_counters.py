#!/usr/bin/env python3
"""Per-kernel counters of the C4 step, isolated (`bench.py --workload c4
--fan-width 1`: every kernel on the caller's stream, one at a time), from one
rocprofv3 --kernel-trace --stats run and rocprofv3 --pmc passes of the same
command; plus the whole-step VALU / HBM summary bench.py's c4.roofline reads
(profiles/c4_valu.json).

usage: c4_counters.py ROUND KT_DIR PMC_DIR [PMC_DIR ...] --traffic TRAFFIC_JSON
                      --steps-total N --out KERNELS_JSON --valu-out VALU_JSON

Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* /
SQ_BUSY_CYCLES count quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs;
a wave issues one VALU instruction per 2 cycles on its SIMD (64 lanes over a
SIMD-32), so the VALU-issue peak is 1024 SIMDs x 32 lanes x clock.  The
kernel's clock is GRBM_GUI_ACTIVE / 8 over its traced duration.

Derived per kernel:
  valu_issue_frac   = SQ_INSTS_VALU x 64 / duration / 78.6 Tops (the roofline
                      peak bench.py prices C4 against: 256 CUs x 4 SIMDs x 32
                      lanes x 2.4 GHz)
  valu_busy_per_SIMD = SQ_INSTS_VALU x 2 / (cycles x 1024): the fraction of
                      SIMD cycles issuing VALU (2 cycles each) at the kernel's clock
  resident_waves_per_SIMD = SQ_WAVE_CYCLES x 4 / (cycles x 1024)
  wait_any / wait_inst_any / active_inst_any fractions of SQ_WAVE_CYCLES
The kernel signature (VGPR / SGPR / LDS / scratch / spills from the library's
code-object metadata, tools/kernel_resources.py) is recorded beside the
counts; bench.py drops the counted fields when the library's kernels no
longer carry that signature (the counts would describe other code)."""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
PEAK_TOPS = 78.6     # bench.py VALU_PEAK_TOPS
SIMDS = 1024


def short(name):
    """'void lavish::(anonymous namespace)::rdo_kernel<16, 16, 1, 0, false>(...)'
    -> 'rdo_kernel<16, 16, 1, 0, false>'."""
    n = name.replace("void ", "").replace("lavish::(anonymous namespace)::", "")
    return n.split("(")[0]


def durations(kt_dir):
    path = glob.glob(os.path.join(kt_dir, "**", "*kernel_stats.csv"), recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(path)):
        if "rocclr" in r["Name"]:
            continue
        out[short(r["Name"])] = {"us": float(r["AverageNs"]) / 1e3, "calls": int(r["Calls"])}
    return out


def pmc(dirs):
    """{kernel: {counter: per-dispatch average over dispatches after the first}}."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(dict)
            names = {}
            for r in csv.DictReader(open(f)):
                if "rocclr" in r["Kernel_Name"]:
                    continue
                k = short(r["Kernel_Name"])
                per[(k, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
                names[k] = 1
            for k in names:
                ids = sorted((i for kk, i in per if kk == k), key=int)
                for i in (ids[1:] or ids):
                    for c, v in per[(k, i)].items():
                        acc[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in acc.items()}


def dispatch_counts(dirs, steps_total):
    n = collections.Counter()
    for d in dirs[:1]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            for r in csv.DictReader(open(f)):
                if "rocclr" in r["Kernel_Name"]:
                    continue
                key = (short(r["Kernel_Name"]), r["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    n[key[0]] += 1
    return {k: v / steps_total for k, v in n.items()}


def signatures(lib):
    """{short kernel name: resource signature} from the library's code objects."""
    import kernel_resources as KR
    res = KR.kernel_resources(lib)
    names = sorted(res)
    return {short(d or n): res[n] for n, d in zip(names, KR.demangled(names))}


def derive(us, c):
    out = {"kernel_us": round(us, 1)}
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
    if "SQ_INSTS_VALU" in c and us:
        out["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * 64 / (us * 1e-6) / 1e12 / PEAK_TOPS, 4)
    if cyc:
        out["clock_GHz"] = round(cyc / (us * 1e3), 3)
        if "SQ_WAVE_CYCLES" in c:
            out["resident_waves_per_SIMD"] = round(c["SQ_WAVE_CYCLES"] * 4 / (cyc * SIMDS), 2)
        if "SQ_INSTS_VALU" in c:
            out["valu_busy_per_SIMD"] = round(c["SQ_INSTS_VALU"] * 2 / (cyc * SIMDS), 3)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for k, name in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                        ("SQ_ACTIVE_INST_ANY", "active_inst_any_frac")):
            if k in c:
                out[name] = round(c[k] / wc, 3)
    v = c.get("SQ_INSTS_VALU")
    if v:
        for k, name in (("SQ_INSTS_SALU", "salu_per_valu"), ("SQ_INSTS_LDS", "lds_per_valu"),
                        ("SQ_INSTS_VMEM_RD", "vmem_rd_per_valu")):
            if k in c:
                out[name] = round(c[k] / v, 4)
    if c.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in c:
        out["lds_bank_conflict_cycles_per_lds_instr"] = round(
            c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3)
    if c.get("SQ_WAVES"):
        out["waves"] = int(c["SQ_WAVES"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round", type=int)
    ap.add_argument("kt")
    ap.add_argument("pmc", nargs="+")
    ap.add_argument("--traffic", required=True)
    ap.add_argument("--steps-total", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--valu-out", required=True)
    ap.add_argument("--lib", default=os.path.join(ROOT, "aom-av1-lavish_amd", "liblavish_hip.so"))
    a = ap.parse_args()
    dur = durations(a.kt)
    cnt = pmc(a.pmc)
    per_step = dispatch_counts(a.pmc, a.steps_total)
    traffic = json.load(open(a.traffic))["kernels"]
    sig = signatures(a.lib)
    kernels = {}
    for k in sorted(cnt, key=lambda k: -dur.get(k, {"us": 0})["us"]):
        d = derive(dur.get(k, {"us": 0})["us"], cnt[k])
        d["dispatches_per_step"] = round(per_step.get(k, 0), 3)
        t = next((v for kk, v in traffic.items() if short(kk) == k), None)
        if t:
            d["hbm_bytes"] = t["hbm_bytes"]
        d["signature"] = sig.get(k)
        d["counters"] = cnt[k]
        kernels[k] = d
    worst = min((k for k in kernels if "valu_issue_frac" in kernels[k]),
                key=lambda k: kernels[k]["valu_issue_frac"])
    res = {"round": a.round,
           "method": "rocprofv3 --kernel-trace --stats and --pmc passes (separate runs) of "
                     "`bench.py --workload c4 --fan-width 1 --no-cpu` (every C4 kernel on the "
                     "caller's stream, one at a time); per-dispatch averages exclude each "
                     "kernel's first dispatch; tools/c4_counters.py (units in its docstring)",
           "kernel_trace": os.path.relpath(a.kt, ROOT), "pmc": [os.path.relpath(p, ROOT) for p in a.pmc],
           "serial_sum_us": round(sum(v["kernel_us"] * v["dispatches_per_step"]
                                      for v in kernels.values()), 1),
           "lowest_valu_issue": worst, "kernels": kernels}
    json.dump(res, open(a.out, "w"), indent=1)
    # the whole-step summary bench.py's c4.roofline reads
    valu = sum(v["counters"].get("SQ_INSTS_VALU", 0) * v["dispatches_per_step"]
               for v in kernels.values())
    hbm = sum(v.get("hbm_bytes", 0) * v["dispatches_per_step"] for v in kernels.values())
    vj = {"round": a.round,
          "source": "tools/c4_counters.py over %s: SQ_INSTS_VALU per dispatch x dispatches "
                    "per step; HBM = FETCH_SIZE x2 + WRITE_SIZE (%s)"
                    % (", ".join(res["pmc"]), os.path.relpath(a.traffic, ROOT)),
          "valu_instr_per_step": round(valu), "hbm_bytes_per_step": round(hbm),
          "kernels": {k: {"dispatches_per_step": v["dispatches_per_step"],
                          "valu_instr_per_dispatch": round(v["counters"].get("SQ_INSTS_VALU", 0)),
                          "signature": v["signature"]} for k, v in kernels.items()}}
    json.dump(vj, open(a.valu_out, "w"), indent=1)
    print(json.dumps({"valu_instr_per_step": vj["valu_instr_per_step"],
                      "hbm_bytes_per_step": vj["hbm_bytes_per_step"], "worst": worst,
                      "kernels": {k: {kk: v.get(kk) for kk in ("kernel_us", "valu_issue_frac",
                                                               "resident_waves_per_SIMD",
                                                               "valu_busy_per_SIMD",
                                                               "wait_any_frac")}
                                  for k, v in kernels.items()}}, indent=1))


if __name__ == "__main__":
    main()
