"""Condense a rocprofv3 run (kernel-trace stats + PMC passes) into profiles/<round>/.

  python tools/profile_summary.py gpurun_out/prof_TAG gpurun_out/pmc_TAG profiles/round1 [bench.json]

Writes kernel_stats.md (the --stats summary), step_timeline.txt (one bench step) and
pmc.json: per-kernel FETCH_SIZE / WRITE_SIZE in KB as rocprofv3 reports them, and
HBM bytes per launch = 2 x FETCH_SIZE x 1024 (gfx950 counts half the bytes of wide
streaming reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE x 1024.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def main():
    prof, pmc, out = sys.argv[1:4]
    bench = sys.argv[4] if len(sys.argv) > 4 else None
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(f"{prof}/**/*kernel_stats.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(stats)), key=lambda r: -float(r["TotalDurationNs"]))
    with open(f"{out}/kernel_stats.md", "w") as f:
        f.write("| kernel | calls | avg us | min us | max us | total ms | % |\n|---|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                    f"{float(r['MinNs'])/1e3:.2f} | {float(r['MaxNs'])/1e3:.2f} | "
                    f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |\n")
    shutil.copy(stats, f"{out}/kernel_stats.csv")
    trace = glob.glob(f"{prof}/**/*kernel_trace.csv", recursive=True)[0]
    tr = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(tr) if "k_compensate_list" in r["Kernel_Name"]]
    with open(f"{out}/step_timeline.txt", "w") as f:
        i0, i1 = idx[-2], idx[-1]
        prev = None
        for r in tr[i0:i1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            f.write(f"{r['Kernel_Name'][:70]:70s} {(e - s) / 1e3:10.2f} us  gap {((s - prev) / 1e3 if prev else 0):7.2f} us\n")
            prev = e
        f.write(f"step span {(int(tr[i1]['Start_Timestamp']) - int(tr[i0]['Start_Timestamp'])) / 1e6:.3f} ms\n")
    res = {}
    if pmc and os.path.isdir(pmc):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for fn in glob.glob(f"{pmc}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(fn)):
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            if not k.startswith("void dgc::") and not k.startswith("dgc::"):
                continue
            f_kb = max(cs.get("FETCH_SIZE", [0])) if cs.get("FETCH_SIZE") else None
            w_kb = max(cs.get("WRITE_SIZE", [0])) if cs.get("WRITE_SIZE") else None
            res[k[:100]] = {"FETCH_SIZE_KB_max_per_launch": f_kb, "WRITE_SIZE_KB_max_per_launch": w_kb,
                            "hbm_bytes_per_launch_corrected": (2 * f_kb * 1024 if f_kb is not None else 0) +
                            (w_kb * 1024 if w_kb is not None else 0)}
        with open(f"{out}/pmc.json", "w") as f:
            json.dump(res, f, indent=1)
    if bench:
        shutil.copy(bench, f"{out}/bench.json")
    print(f"wrote {out}")


if __name__ == "__main__":
    main()
