"""Print a rocprofv3 kernel_stats.csv compactly: python tools/kstats.py DIR [filter]"""
import csv
import glob
import sys

path = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in csv.DictReader(open(path)):
    if flt in r["Name"]:
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} "
              f"min_us={float(r['MinNs'])/1e3:9.2f}")
