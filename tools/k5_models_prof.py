"""Where the model sets' k_nth_select time goes, per tensor (workgroup), in the bench's
steady state: the profiling build's per-workgroup stamps (kernel start, replay start,
global / LDS / single-wave phase ends, kernel end), for the resampled tensors.

  make -C adam-compression_amd/csrc k5prof
  python tools/k5_models_prof.py [resnet50|vgg16_bn] [steps]

Prints, for the last step, one line per resampled tensor: candidates and phase times
(us) from the kernel's earliest workgroup start.
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


class K5Prof(ctypes.Structure):
    _fields_ = [("t", ctypes.c_uint64 * 8), ("steps", ctypes.c_uint32 * 4), ("sub", ctypes.c_uint64 * 8),
                ("bt", (ctypes.c_uint64 * 8) * 64), ("bn", ctypes.c_int64 * 64)]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    L = _lib.lib()
    L.dgc_k5_prof.restype = ctypes.c_int
    L.dgc_k5_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    run = bench.ModelRun(bench.WORKLOADS[wl], 0, 1, torch.device("cuda:0"), "sparse", steps)   # per-step gradients
    b = run.b
    for i in range(steps):
        torch.cuda.synchronize()
        _lib.check(L.dgc_k5_prof(None, 1))
        run.step(i)
        torch.cuda.synchronize()
        p = K5Prof()
        _lib.check(L.dgc_k5_prof(ctypes.byref(p), 0))
        infos = b.infos()
        rows = []
        t0 = min((p.bt[t][7] for t in range(min(64, len(infos))) if p.bt[t][7]), default=0)
        end = max((p.bt[t][6] for t in range(min(64, len(infos))) if p.bt[t][6]), default=0)
        for t, inf in enumerate(infos[:64]):
            if inf["branch"] != "resample":
                continue
            s = [x for x in p.bt[t]]
            us = lambda a, z: round((s[z] - s[a]) * 0.01, 1) if s[a] and s[z] else None  # noqa: E731
            rows.append(dict(t=t, name=b.names[t], cand=inf["candidates"], n=p.bn[t],
                             start=round((s[7] - t0) * 0.01, 1) if s[7] else None,
                             glob=us(0, 1), load=us(1, 2), lds=us(2, 3), wave=us(3, 4), store=us(4, 5),
                             done=round((s[5] - t0) * 0.01, 1) if s[5] else None,
                             end=round((s[6] - t0) * 0.01, 1) if s[6] else None))
        print(json.dumps({"step": i, "kernel_us": round((end - t0) * 0.01, 1), "resampled": rows}), flush=True)


if __name__ == "__main__":
    main()
