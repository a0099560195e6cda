"""Condense one bench command's rocprofv3 runs into profiles/<round>/.

  python tools/profile_summary.py WORKLOAD PROF_DIR PMC_DIR OUT_DIR [bench.json] [command]

PROF_DIR: `rocprofv3 --kernel-trace --stats` of the command; PMC_DIR: its separate
`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes (FETCH_SIZE and WRITE_SIZE do not fit
one pass on gfx950). Writes, for WORKLOAD:

  kernel_stats_<W>.md / .csv   the --stats summary
  kstats_<W>.json              {kernel: calls, avg/min/max/total ms} (bench.py reads K1's avg)
  step_timeline_<W>.txt        the kernels of the last full step, with gaps
  pmc_<W>.json                 per kernel, the AVERAGE per launch of FETCH_SIZE and WRITE_SIZE
                               (KB as rocprofv3 reports them). HBM bytes per launch =
                               2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 ONLY for the kernels
                               whose reads are 16-B-per-lane coalesced streams (STREAMING:
                               the guide calibrates the x2 for exactly that access shape,
                               MI355X_MICROARCH.md §HBM "FETCH_SIZE reports exactly 1/2 ...";
                               "other access widths are uncalibrated"); every other kernel
                               gets hbm_bytes_per_launch = null and the uncalibrated range
                               [FETCH + WRITE, 2 x FETCH + WRITE] instead.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


# kernels whose global reads are 16-B-per-lane coalesced streams (float4 / dwordx4
# tiles over contiguous vec / grad / mmt): K1, the full select pass, the lowering
# counts, the probe and K7's multi-tensor apply
STREAMING = ("k_compensate_list", "k_compensate4", "k_select_pass", "k_lower_counts", "k_probe", "k_sgd",
             "k_fill_zero")


def main():
    wl, prof, pmc, out = sys.argv[1:5]
    bench = sys.argv[5] if len(sys.argv) > 5 else None
    command = sys.argv[6] if len(sys.argv) > 6 else None
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(f"{prof}/**/*kernel_stats.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(stats)), key=lambda r: -float(r["TotalDurationNs"]))
    with open(f"{out}/kernel_stats_{wl}.md", "w") as f:
        if command:
            f.write(f"`{command}`\n\n")
        f.write("| kernel | calls | avg us | min us | max us | total ms | % |\n|---|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                    f"{float(r['MinNs'])/1e3:.2f} | {float(r['MaxNs'])/1e3:.2f} | "
                    f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |\n")
    shutil.copy(stats, f"{out}/kernel_stats_{wl}.csv")
    ks = {r["Name"][:120]: {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                            "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6,
                            "total_ms": float(r["TotalDurationNs"]) / 1e6} for r in rows}
    trace = glob.glob(f"{prof}/**/*kernel_trace.csv", recursive=True)
    warm = json.loads(open(bench).read().strip().splitlines()[-1]).get("warmup", 0) if bench else 0
    if trace:
        tr = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
        # the --stats average includes the warmup launches (first touch of the buffers:
        # up to 4x slower); the bench times the launches after them
        for name, v in ks.items():
            durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr
                    if r["Kernel_Name"][:120] == name]
            if len(durs) > warm:
                v["timed_avg_ms"] = sum(durs[warm:]) / len(durs[warm:])
                v["timed_launches"] = len(durs) - warm
    with open(f"{out}/kstats_{wl}.json", "w") as f:
        json.dump(ks, f, indent=1)
    if trace:
        idx = [i for i, r in enumerate(tr) if "k_compensate_list" in r["Kernel_Name"]]
        if len(idx) >= 2:
            with open(f"{out}/step_timeline_{wl}.txt", "w") as f:
                i0, i1 = idx[-2], idx[-1]
                prev = None
                for r in tr[i0:i1]:
                    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                    f.write(f"{r['Kernel_Name'][:70]:70s} {(e - s) / 1e3:10.2f} us  "
                            f"gap {((s - prev) / 1e3 if prev else 0):7.2f} us\n")
                    prev = e
                f.write(f"step span {(int(tr[i1]['Start_Timestamp']) - int(tr[i0]['Start_Timestamp'])) / 1e6:.3f} ms\n")
    if pmc and os.path.isdir(pmc):
        # per kernel and counter, the values in dispatch order; the first `warm` launches
        # of each kernel are dropped as kstats drops them (the warmup steps: first touch
        # of the buffers, full passes before the lists exist), so the bytes per launch and
        # the timed duration per launch describe the same launches
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for fn in glob.glob(f"{pmc}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(fn)):
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
                agg[r["Kernel_Name"]][r["Counter_Name"]].append((key, float(r["Counter_Value"])))
        res = {}
        for k, cs in agg.items():
            if "dgc::" not in k:
                continue
            timed = {c: [v for _, v in sorted(vals)][warm:] or [v for _, v in sorted(vals)] for c, vals in cs.items()}
            avg = {c: sum(v) / len(v) for c, v in timed.items()}
            f_kb, w_kb = avg.get("FETCH_SIZE"), avg.get("WRITE_SIZE")
            fb = f_kb * 1024 if f_kb is not None else 0
            wb = w_kb * 1024 if w_kb is not None else 0
            stream = any(s in k for s in STREAMING)
            hb = (2 * fb + wb) if stream else None
            t_ms = ks.get(k[:120], {}).get("timed_avg_ms")
            res[k[:120]] = {"launches": max(len(v) for v in cs.values()),
                            "timed_launches": max(len(v) for v in timed.values()), "FETCH_SIZE_KB_avg": f_kb,
                            "WRITE_SIZE_KB_avg": w_kb, "calibrated": stream,
                            "hbm_bytes_per_launch": hb,
                            "hbm_bytes_per_launch_range": None if stream else [fb + wb, 2 * fb + wb],
                            # the implied rate over the same (timed) launches; above the 8 TB/s
                            # peak it says the bytes or the time are not the same launches'
                            "implied_GBs": (round((hb if hb is not None else fb + wb) / (t_ms * 1e6), 1)
                                            if t_ms else None)}
        with open(f"{out}/pmc_{wl}.json", "w") as f:
            json.dump({"command": command, "kernels": res}, f, indent=1)
    if bench:
        # the bench ran before these profiles existed on the box: point its roofline at
        # the K1 duration and PMC traffic of THIS profile of the same command
        d = json.loads(open(bench).read().strip().splitlines()[-1])
        k1 = [v for name, v in ks.items() if "k_compensate_list" in name]
        rf = d.get("roofline", {})
        rel = os.path.relpath(out, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        if k1:
            v1 = max(k1, key=lambda v: v["calls"])
            rf["rocprof_avg_launch_ms"] = v1.get("timed_avg_ms", v1["avg_ms"])
            rf["rocprof_source"] = f"{rel}/kstats_{wl}.json"
        if pmc and os.path.isdir(pmc):
            t = [v["hbm_bytes_per_launch"] for name, v in res.items()
                 if "k_compensate_list" in name and v["hbm_bytes_per_launch"] is not None]
            if t:
                rf["traffic"] = max(t)
                rf["traffic_source"] = f"{rel}/pmc_{wl}.json"
        with open(f"{out}/bench_{wl}.json", "w") as f:
            f.write(json.dumps(d) + "\n")
    print(f"wrote {out} for {wl}")


if __name__ == "__main__":
    main()
