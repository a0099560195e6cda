"""Host vs GPU time of the drop-in optimizer step (bench.DropinRun): per-step host time
of the Python call (no sync) against the synchronised step time, for batch modes.
  python tools/dropin_prof.py [resnet50|vgg16_bn] [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[model]
    for label, mk in (("dgcbatch", lambda: bench.ModelRun(wl, 0, 1, dev, "inline")),
                      ("optimizer", lambda: bench.DropinRun(wl, 0, 1, dev, True, steps + 5))):
        run = mk()
        for i in range(5):
            run.step(i)
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for i in range(steps):
            h0 = time.perf_counter()
            run.step(5 + i)
            host.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        print(f"{label}: {dt * 1e3:.4f} ms/step, host {sum(host) / steps * 1e3:.4f} ms/step "
              f"(min {min(host) * 1e3:.4f})", flush=True)
        if label == "optimizer":   # host time by part of the step (no GPU sync in between)
            ph = [0.0] * 4
            for i in range(steps):
                t = [time.perf_counter()]
                for (_, p), g in zip(run.named, run.sets[i % len(run.sets)]):
                    p.grad = g
                t.append(time.perf_counter())
                for _, hook in run.hooks:
                    hook()
                t.append(time.perf_counter())
                run.opt.synchronize()
                t.append(time.perf_counter())
                run.opt.zero_grad()
                t.append(time.perf_counter())
                for j in range(4):
                    ph[j] += t[j + 1] - t[j]
            torch.cuda.synchronize()
            print("  host us/step: " + ", ".join(f"{k} {v / steps * 1e6:.1f}" for k, v in
                                                zip(("assign", "hooks", "synchronize", "zero_grad"), ph)), flush=True)
        del run


if __name__ == "__main__":
    main()
