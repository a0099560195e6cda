"""Average rocprofv3 --pmc counters per kernel: python tools/pmc_summary.py DIR [filter]"""
import collections
import csv
import glob
import sys

flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    print("   ", "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(d.items())))
