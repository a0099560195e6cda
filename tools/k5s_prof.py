"""Where a model set's K5s time goes (k_resample_set), in the bench's steady state:
the profiling build's stamps of each set's first workgroup — past the residency
consensus, min/max merged, radix select, compaction counts merged, emit end — for
the last steps.

  make -C adam-compression_amd/csrc k5prof
  python tools/k5s_prof.py [resnet50|vgg16_bn] [steps]
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
from k5_models_prof import K5Prof as _Base  # noqa: E402


class K5Prof(ctypes.Structure):
    _fields_ = _Base._fields_ + [("set", (ctypes.c_uint64 * 8) * 64)]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    L = _lib.lib()
    L.dgc_k5_prof.restype = ctypes.c_int
    L.dgc_k5_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    run = bench.ModelRun(bench.WORKLOADS[wl], 0, 1, torch.device("cuda:0"), "sparse", steps)   # per-step gradients
    b = run.b
    # resample_set_body's stamps (the set's first workgroup): 0 past the residency
    # consensus, 1 min/max merged, 2 radix select done, 3 compaction counts merged, 4 emit end
    names = ("minmax", "radix", "compact", "emit")
    for i in range(steps):
        torch.cuda.synchronize()
        _lib.check(L.dgc_k5_prof(None, 1))
        run.step(i)
        torch.cuda.synchronize()
        p = K5Prof()
        _lib.check(L.dgc_k5_prof(ctypes.byref(p), 0))
        infos = b.infos()
        t0 = min((p.set[t][0] for t in range(min(64, len(infos))) if p.set[t][0]), default=0)
        rows = []
        for t, inf in enumerate(infos[:64]):
            s = list(p.set[t])
            if not s[0]:
                continue
            r = dict(t=t, cand=inf["candidates"], k=b.attrs[t][0], tie=inf["tie_rule"],
                     start=round((s[0] - t0) * 0.01, 2))
            for j, nm in enumerate(names):
                r[nm] = round((s[j + 1] - s[j]) * 0.01, 2) if s[j + 1] and s[j] else None
            r["end"] = round((s[4] - t0) * 0.01, 2) if s[4] else None
            rows.append(r)
        rows.sort(key=lambda r: -(r["end"] or 0))
        # k_nth_select after it (every workgroup stamps its start [7] and end [6]):
        # first / last workgroup start and last end, from the same origin
        T = min(64, len(infos))
        st7 = [p.bt[t][7] for t in range(T) if p.bt[t][7]]
        en6 = [p.bt[t][6] for t in range(T) if p.bt[t][6]]
        rel = lambda x: round((x - t0) * 0.01, 2) if t0 and x else None  # noqa: E731
        nth = dict(first_start=rel(min(st7, default=0)), last_start=rel(max(st7, default=0)),
                   last_end=rel(max(en6, default=0)), workgroups=len(st7))
        # the finishing workgroup (an idle one: slots 0-2 = branch read, arrival, finish)
        fin = [t for t in range(T) if p.bt[t][1]]
        if fin:
            f = fin[0]
            nth["finisher"] = dict(t=f, start=rel(p.bt[f][7]), read=rel(p.bt[f][0]), arrived=rel(p.bt[f][1]),
                                   finished=rel(p.bt[f][2]), end=rel(p.bt[f][6]))
        print(json.dumps({"step": i, "nth_select": nth, "slowest": rows[:6]}), flush=True)


if __name__ == "__main__":
    main()
