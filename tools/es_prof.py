"""Where the model sets' merged emit + K5s launch (k_emit_wide_t<true>) spends its time,
in the bench's steady state: the profiling build's per-workgroup stamps (select.hip
ES_STAMP) for the last step — every emit workgroup's entry, scan done and end; every set
workgroup's entry, its tensor's gather seen complete, and end — against the launch's
first entry.

  make -C adam-compression_amd/csrc k5prof
  python tools/es_prof.py [resnet50|vgg16_bn] [steps]
"""
import ctypes
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DGC_HIP_LIB"] = os.path.join(REPO, "adam-compression_amd", "lib", "k5prof", "libdgc_hip.so")
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd"), os.path.join(REPO, "tools")]

import torch  # noqa: E402

import bench  # noqa: E402
from dgc import _lib  # noqa: E402

NB = 4096
SEG, GROUP_QUARTER, SET_COOP, SET_BIG, SET_GMIN = 1024, 256, 16384, 128, 4


def layout(b):
    """(emit workgroups per tensor, set workgroups per tensor) as select.hip's bt_blocks."""
    grp, sets = [], []
    for n, (k, S, ks, stride) in zip(b.numels, b.attrs):
        nseg = -(-n // SEG)
        grp.append(-(-nseg // GROUP_QUARTER))
        cap = min(64 * k - 1, n)
        if k < 1 or cap <= k:
            sets.append(0)
        elif cap <= SET_COOP:
            sets.append(1)
        else:
            sets.append(min(SET_BIG, max(SET_GMIN, -(-cap // SET_COOP))))
    return grp, sets


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * len(xs)))], 2) if xs else None


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    L = _lib.lib()
    L.dgc_es_prof.restype = ctypes.c_int
    L.dgc_es_prof.argtypes = [ctypes.c_void_p]
    run = bench.ModelRun(bench.WORKLOADS[wl], 0, 1, torch.device("cuda:0"), "sparse", steps)   # per-step gradients
    b = run.b
    buf = ((ctypes.c_uint64 * 3) * NB)()
    for i in range(steps):
        run.step(i)
    torch.cuda.synchronize()
    _lib.check(L.dgc_es_prof(ctypes.byref(buf)))
    infos = b.infos()
    grp, sets = layout(b)
    ngb = sum(grp)
    rows = [list(r) for r in buf]
    total = ngb + sum(sets)
    t0 = min(rows[i][0] for i in range(min(total, NB)))
    us = lambda x: round((x - t0) * 0.01, 2)   # noqa: E731
    emit_end = [us(rows[i][2]) for i in range(ngb)]
    out = {"workload": wl, "emit_workgroups": ngb, "set_workgroups": sum(sets),
           "emit_scan_done_us": {"p50": pct([us(rows[i][1]) for i in range(ngb) if rows[i][1] >= t0], .5),
                                 "max": pct([us(rows[i][1]) for i in range(ngb) if rows[i][1] >= t0], 1)},
           "emit_end_us": {"p50": pct(emit_end, .5), "max": pct(emit_end, 1)}}
    tens = []
    e0 = s0 = 0
    for t, (g, sc) in enumerate(zip(grp, sets)):
        inf = infos[t]
        if sc and inf["branch"] == "resample":
            gather_done = max(us(rows[e0 + j][2]) for j in range(g))
            sb = [ngb + s0 + j for j in range(sc)]
            used = [r for r in sb if rows[r][1] >= t0]   # workgroups that waited (took part)
            tens.append({"t": t, "cand": inf["candidates"], "tie": inf["tie_rule"], "emit_wgs": g,
                         "gather_done": gather_done, "set_wgs": len(used),
                         "set_entry": min((us(rows[r][0]) for r in used), default=None),
                         "wait_done": max((us(rows[r][1]) for r in used), default=None),
                         "set_end": max((us(rows[r][2]) for r in used), default=None)})
        e0 += g
        s0 += sc
    tens.sort(key=lambda r: -(r["set_end"] or 0))
    out["sets_by_end"] = tens[:12]
    out["launch_end_us"] = max(us(rows[i][2]) for i in range(min(total, NB)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
