"""Where the model sets' K3 (k_rs_small_multi: one workgroup per tensor's sampled
threshold) spends its time, in the bench's steady state: the profiling build's
per-workgroup stamps (radix_select.hpp RS_STAMP) for the last step — start, keys loaded
and the pass-0 floor, the floor picked, each radix pass, the threshold written, the
selection state reset.

  make -C adam-compression_amd/csrc k5prof
  python tools/k3_prof.py [resnet50|vgg16_bn] [steps]
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DGC_HIP_LIB"] = os.path.join(REPO, "adam-compression_amd", "lib", "k5prof", "libdgc_hip.so")
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd"), os.path.join(REPO, "tools")]

import torch  # noqa: E402

import bench  # noqa: E402
from dgc import _lib  # noqa: E402

NAMES = ("load+floor", "floor pick", "p0 hist", "p0 pick", "p1 hist", "p1 pick", "p2 hist", "p2 pick",
         "out", "reset")


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    L = _lib.lib()
    L.dgc_rs_prof.restype = ctypes.c_int
    L.dgc_rs_prof.argtypes = [ctypes.c_void_p]
    run = bench.ModelRun(bench.WORKLOADS[wl], 0, 1, torch.device("cuda:0"), "sparse", steps)   # per-step gradients
    buf = ((ctypes.c_uint64 * 12) * 64)()
    for i in range(steps):
        run.step(i)
    torch.cuda.synchronize()
    _lib.check(L.dgc_rs_prof(ctypes.byref(buf)))
    rows = [list(r) for r in buf]
    t0 = min((r[0] for r in rows if r[0]), default=0)
    out = []
    for b, r in enumerate(rows):
        if not r[0]:
            continue
        d = {"wg": b, "start": round((r[0] - t0) * 0.01, 2)}
        prev = r[0]
        for j, nm in enumerate(NAMES):
            x = r[j + 1]
            if x:
                d[nm] = round((x - prev) * 0.01, 2)
                prev = x
        d["end"] = round((prev - t0) * 0.01, 2)
        out.append(d)
    out.sort(key=lambda d: -d["end"])
    for d in out[:12]:
        print(json.dumps(d))


if __name__ == "__main__":
    main()
