"""Per-tensor selection records of a model workload in the bench's steady state:
branch, candidates, full passes, recounts per compressed tensor for the last steps.

  python tools/model_infos.py [resnet50|vgg16_bn] [steps] [all]

Same ModelRun (gradients, seeds) as bench.py; prints one JSON line per step with the
tensors that did more than a list-served first-k selection.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    full = len(sys.argv) > 3 and sys.argv[3] == "all"   # every tensor, not only the notable ones
    dev = torch.device("cuda:0")
    run = bench.ModelRun(bench.WORKLOADS[wl], 0, 1, dev, "sparse", steps)   # a gradient set per step
    b = run.b
    for i in range(steps):
        run.step(i)
        torch.cuda.synchronize()
        rows = []
        for t, inf in enumerate(b.infos()):
            if not full and inf["branch"] in ("ok", "trunc") and inf["full_passes"] == 0 and inf["recounts"] == 0:
                continue
            rows.append(dict(t=t, n=b.numels[t], k=b.attrs[t][0], **{k: inf[k] for k in (
                "branch", "candidates", "full_passes", "recounts", "overflow_segments", "threshold0",
                "threshold", "list_threshold")}))
        print(json.dumps({"step": i, "tensors": len(b.names), "notable": rows}), flush=True)


if __name__ == "__main__":
    main()
