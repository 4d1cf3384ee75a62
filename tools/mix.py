"""Per-wave instruction mix of the diamond kernel from a rocprofv3 --pmc run."""
import collections
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    if (sys.argv[2] if len(sys.argv) > 2 else "diamond") in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = acc["SQ_WAVES"][-1]
print({k: round(v[-1] / w, 1) for k, v in sorted(acc.items())})
