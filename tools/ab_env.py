"""Same-box A/B of environment switches: bench.py lines under each setting, alternating.

  python tools/ab_env.py WORKLOAD REPS 'label=ENV=V,ENV2=V2' 'label2=' ...

Prints one JSON line per run and a summary (median ms/step per setting). Each run is a
separate process (the library reads its switches once per process).
"""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    wl, reps = sys.argv[1], int(sys.argv[2])
    settings = []
    for spec in sys.argv[3:]:
        label, _, envs = spec.partition("=")
        env = {}
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        settings.append((label, env))
    res = {label: [] for label, _ in settings}
    for r in range(reps):
        for label, env in settings:
            e = dict(os.environ)
            e.update(env)
            out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "5",
                                  "--workload", wl, "--no-cpu", "--no-extras"], env=e, capture_output=True, text=True,
                                 timeout=600)
            if out.returncode != 0:
                print(out.stderr[-3000:], file=sys.stderr)
                raise SystemExit(f"{label}: bench failed ({out.returncode})")
            d = json.loads(out.stdout.strip().splitlines()[-1])
            sel = d.get("selection_steps", {})
            row = {"rep": r, "setting": label, "ms_per_step": d["ms_per_step"], "k1_ms": d["phase_ms"]["compensate"],
                   "full_passes": sum(sel.get("full_passes_per_step", [])), "resamples": sel.get("resamples")}
            print(json.dumps(row), flush=True)
            res[label].append(d["ms_per_step"])
    print(json.dumps({"workload": wl, "median_ms": {k: round(statistics.median(v), 4) for k, v in res.items()},
                      "runs": {k: [round(x, 4) for x in v] for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
