"""Where k_count_emit spends its time: per-group phase stamps of the profiling build
(make -C adam-compression_amd/csrc k5prof) over a few flat-1B bench steps.

  python tools/ce_prof.py [workload] [steps]

Prints, for the last step, percentiles over the groups of each phase (us) and of the
phase ends relative to the earliest group start.
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DGC_HIP_LIB"] = os.path.join(REPO, "adam-compression_amd", "lib", "k5prof", "libdgc_hip.so")
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from dgc import _lib  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "flat-1B"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    L = _lib.lib()
    L.dgc_ce_prof.restype = ctypes.c_int
    L.dgc_ce_prof.argtypes = [ctypes.c_void_p]
    run = bench.FlatRun(bench.WORKLOADS[wl], 0, 1, torch.device("cuda:0"), "sparse")
    for i in range(steps):
        run.step(i)
    torch.cuda.synchronize()
    buf = np.zeros((2048, 6), np.uint64)
    _lib.check(L.dgc_ce_prof(buf.ctypes.data))
    ng = -(-run.N // (1024 * 1024))   # groups of 1M elements
    t = buf[:min(ng, 2048)].astype(np.float64) * 0.01   # us
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    names = ["count", "scan+lookback", "emit", "copy-out", "arrival"]
    for k, nm in enumerate(names):
        d = t[:, k + 1] - t[:, k]
        print(f"{nm:14s} p50 {np.percentile(d, 50):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f} us")
    for k in range(6):
        e = t[:, k] - t0
        print(f"stamp {k}: p0 {e.min():7.2f}  p50 {np.percentile(e, 50):7.2f}  max {e.max():7.2f} us from the first start")


if __name__ == "__main__":
    main()
