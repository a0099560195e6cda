"""Where a model set's count pass (k_count_pass, the step's last launch of it) and the
multi-threshold lowering (k_lower_counts) spend their time: the profiling build's
per-workgroup stamps (select.hip PASS_STAMP) for the last step — entry, past the
tensor gate, loads done, arrival (atomics issued), end.

  make -C adam-compression_amd/csrc k5prof
  python tools/pass_prof.py [resnet50|vgg16_bn] [steps]
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

NB = 16384


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * len(xs)))], 2) if xs else None


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    L = _lib.lib()
    L.dgc_pass_prof.restype = ctypes.c_int
    L.dgc_pass_prof.argtypes = [ctypes.c_void_p]
    run = bench.ModelRun(bench.WORKLOADS[wl], 0, 1, torch.device("cuda:0"), "sparse", steps)   # per-step gradients
    buf = (((ctypes.c_uint64 * 6) * NB) * 2)()
    for i in range(steps):
        run.step(i)
    torch.cuda.synchronize()
    _lib.check(L.dgc_pass_prof(ctypes.byref(buf)))
    for kind, name in ((0, "k_count_pass (last)"), (1, "k_lower_counts")):
        rows = [list(r) for r in buf[kind]]
        # this launch's workgroups: the most recent entry stamps (a launch writes every
        # workgroup's entry; later stamps of a gated-out workgroup are older than it)
        t_last = max(r[0] for r in rows)
        live = [r for r in rows if r[0] and t_last - r[0] < 200000]   # within 2 ms of the newest
        t0 = min(r[0] for r in live)
        work = [r for r in live if r[1] >= r[0] and r[1] - r[0] < 200000]
        ms = lambda a, b: (b - a) * 0.01   # noqa: E731  (100 MHz ticks -> us)
        out = {"kernel": name, "workgroups": len(live), "working": len(work),
               "entry_spread_us": round(ms(t0, max(r[0] for r in live)), 2),
               "gated_exit_last_us": round(ms(t0, max(r[0] for r in live if r not in work)), 2)
               if len(work) < len(live) else None}
        if work:
            out["work_start_us"] = {"p0": pct([ms(t0, r[1]) for r in work], 0), "p50": pct([ms(t0, r[1]) for r in work], .5),
                                    "max": pct([ms(t0, r[1]) for r in work], 1)}
            ld = [r for r in work if r[5] >= r[1] and r[5] - r[1] < 200000]
            out["first_loads_us"] = {"p50": pct([ms(r[1], r[5]) for r in ld], .5), "max": pct([ms(r[1], r[5]) for r in ld], 1)}
            out["loads_us"] = {"p50": pct([ms(r[1], r[2]) for r in work], .5), "p90": pct([ms(r[1], r[2]) for r in work], .9),
                               "max": pct([ms(r[1], r[2]) for r in work], 1)}
            out["atomics_us"] = {"p50": pct([ms(r[2], r[3]) for r in work], .5), "max": pct([ms(r[2], r[3]) for r in work], 1)}
            ends = [r for r in work if r[4] >= r[3] and r[4] - r[3] < 200000]
            out["arrive_to_end_us"] = {"p50": pct([ms(r[3], r[4]) for r in ends], .5),
                                       "max": pct([ms(r[3], r[4]) for r in ends], 1)}
            out["last_end_us"] = round(ms(t0, max(r[4] for r in ends)), 2) if ends else None
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
