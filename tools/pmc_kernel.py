#!/usr/bin/env python3
"""Per-dispatch counter values of one kernel from rocprofv3 --pmc passes
(DIR/*/..._counter_collection.csv), averaged over its dispatches after the
first.  usage: pmc_kernel.py SUBSTRING DIR [DIR ...] [--json OUT]"""
import collections
import csv
import glob
import json
import os
import sys


def collect(sub, dirs):
    acc = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(dict)
            for r in csv.DictReader(open(f)):
                if sub in r["Kernel_Name"]:
                    per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            ids = sorted(per, key=int)[1:] or sorted(per, key=int)
            for i in ids:
                for k, v in per[i].items():
                    acc[k].append(v)
    return {k: sum(v) / len(v) for k, v in sorted(acc.items())}


if __name__ == "__main__":
    args = sys.argv[1:]
    out = None
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        args = args[:i] + args[i + 2:]
    res = collect(args[0], args[1:])
    for k, v in res.items():
        print("%-32s %.0f" % (k, v))
    if out:
        json.dump({"kernel": args[0], "dirs": args[1:], "per_dispatch": res}, open(out, "w"),
                  indent=1)
