"""One line per bench JSON: python tools/bench_table.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as e:
        print(f, "unreadable:", e)
        continue
    r, h = d["roofline"], d["step_hbm"]
    pr = d.get("hbm_probe", {})
    cb = d.get("cpu_baseline", {})
    print(f"{d['config']['workload'][:14]:14s} ms/step {d['ms_per_step']:.4f} value {d['value']:.3e} "
          f"K1 {r['avg_launch_ms']:.4f} ms frac {r['frac']:.3f} step_frac {h['frac_of_8TBs']:.3f} "
          f"probe {pr.get('GBs', 0):.0f} GB/s k1/probe {pr.get('k1_frac_of_probe', 0):.3f} "
          f"cpu {cb.get('value', 0):.3e} sel {json.dumps(d.get('selection'))[:160]}")
