"""One steady-state step of a `rocprofv3 --kernel-trace --output-format csv` run, kernel
by kernel: `python tools/step_trace.py <dir with *_kernel_trace.csv> [anchor]`.
The step runs from the second-to-last launch of the anchor kernel (K1 by default) to
the last one; prints each launch's grid and duration, the non-K1 kernel sum and the
span between the two K1s."""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "compensate_list"
    path = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    s, e = idx[-2], idx[-1]
    tot = 0.0
    for r in rows[s:e]:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if anchor not in r["Kernel_Name"]:
            tot += us
        print(f"{r['Kernel_Name'][:56]:56s} grid={r['Grid_Size_X']:>10s} {us:9.2f} us")
    span = (int(rows[e]["Start_Timestamp"]) - int(rows[s]["End_Timestamp"])) / 1e3
    print(f"non-anchor kernel sum {tot:.1f} us, span between anchors {span:.1f} us")


if __name__ == "__main__":
    main()
