"""DESIGN.md §5's table rows from profiles/<round>/bench_<W>.json (+ kstats / pmc beside them).

  python tools/design_table.py profiles/round6 resnet50 vgg16_bn flat-1B flat-7B-bf16 [resnet50_alternating ...]
"""
import json
import os
import sys


def row(d, W, pmc):
    r, h, pr = d["roofline"], d["step_hbm"], d.get("hbm_probe", {})
    sel = d.get("selection_steps", {})
    fps = sel.get("full_passes_per_step") or [0]
    rs = sel.get("resamples", {})
    nsteps = max(1, sel.get("steps", 1))
    k1 = [v for k, v in pmc.get("kernels", {}).items() if "k_compensate_list" in k]
    pmc_gb = f"{k1[0]['hbm_bytes_per_launch'] / 1e9:.2f}" if k1 and k1[0].get("hbm_bytes_per_launch") else "—"
    cb = d.get("cpu_baseline", {})
    return (f"| {W} | {d['ms_per_step']:.4f} | {d['value']:.3g} | {r['avg_launch_ms']:.3f} / "
            f"{(r.get('rocprof_avg_launch_ms') or 0):.3f} ms | {r['frac']:.3f} | {pr.get('GBs', 0) / 1e3:.2f} TB/s | "
            f"{pr.get('k1_frac_of_probe', 0):.3f} | {h['frac_of_8TBs']:.3f} | {pmc_gb} / "
            f"{r['algorithmic_bytes_per_launch'] / 1e9:.2f} GB | {sum(fps) / len(fps):.1f} | "
            f"{(rs.get('set', 0) + rs.get('exact', 0)) / nsteps:.1f} | "
            f"{cb.get('value', 0):.3g} ({cb.get('cores', '—')} thr) |")


def main():
    base = sys.argv[1]
    print("| Workload | ms/step | grad elem/s | K1 live / rocprof | K1 / 8 TB/s | probe | K1 / probe | step / 8 TB/s "
          "| K1 PMC / algorithmic | full passes / step | resamples / step | CPU port |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for W in sys.argv[2:]:
        f = os.path.join(base, f"bench_{W}.json")
        if not os.path.exists(f):
            print(f"| {W} | (missing) |")
            continue
        d = json.loads(open(f).read().strip().splitlines()[-1])
        p = os.path.join(base, f"pmc_{W}.json")
        pmc = json.load(open(p)) if os.path.exists(p) else {}
        print(row(d, W, pmc))


if __name__ == "__main__":
    main()
