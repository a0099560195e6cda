"""Per-step speculative-list state of a flat bench workload: the list threshold K1
used (spec[0] before the step), the final threshold, their ratio (the margin m x
growth that step), the window-list size and the branch.

  python tools/spec_trace.py [flat-1B|flat-7B-bf16] [steps]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "flat-1B"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    run = bench.FlatRun(bench.WORKLOADS[wl], 0, 1, torch.device("cuda:0"), "sparse")
    b = run.b
    for i in range(steps):
        used = float(b.spec[0].item())
        run.step(i)
        torch.cuda.synchronize()
        inf = b.last_info()
        t = inf["threshold"]
        print(json.dumps({"step": i, "list_t": used, "t": t, "list_over_t": used / t if t else None,
                          "window_keys": inf["window_keys"], "full_passes": inf["full_passes"],
                          "branch": inf["branch"], "candidates": inf["candidates"]}), flush=True)


if __name__ == "__main__":
    main()
