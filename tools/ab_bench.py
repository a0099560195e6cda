"""Same-box A/B of whole bench steps: `python tools/ab_bench.py WORKLOAD A B [C ...] [reps]`
runs `bench.py --workload WORKLOAD --no-cpu` for A, B, ... in turn, alternating `reps`
times, and prints ms/step, K1 ms and the phase times per run (MI355X boxes differ by
~10 %, so only same-box comparisons mean anything). A / B: a library (this tree's
bench.py with DGC_HIP_LIB = it; it must export the symbols dgc/_lib.py binds — build it
from a nearby revision: `make -C <old csrc> OUT_DIR=<repo>/adam-compression_amd/lib/ab_old`)
or a directory holding a whole tree with its built library (`git worktree add .ab_head
HEAD` + make), whose own bench.py runs — for changes above the library."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    wl, libs = sys.argv[1], sys.argv[2:]
    reps = 2
    if libs and libs[-1].isdigit():   # trailing repetition count
        reps = int(libs.pop())
    for _ in range(reps):
        for lib in libs:
            if os.path.isdir(lib):
                env, root = dict(os.environ), os.path.abspath(lib)
                env.pop("DGC_HIP_LIB", None)
            else:
                env, root = dict(os.environ, DGC_HIP_LIB=os.path.abspath(lib), DGC_LIB_PARTIAL="1"), REPO
            out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--workload", wl, "--no-cpu", "--no-extras",
                                  "--steps", "20", "--warmup", "5"], env=env, check=True, capture_output=True,
                                 text=True).stdout
            d = json.loads(out.strip().splitlines()[-1])
            print(json.dumps({"lib": lib, "ms_per_step": round(d["ms_per_step"], 4),
                              "k1_ms": round(d["roofline"]["avg_launch_ms"], 4), "phase_ms": d["phase_ms"]}),
                  flush=True)


if __name__ == "__main__":
    main()
