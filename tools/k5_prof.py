"""K5 phase times: where the exact resample replay spends its time, by candidate count.

Needs the profiling build (`make -C adam-compression_amd/csrc k5prof`, which writes
adam-compression_amd/lib/k5prof/libdgc_hip.so with -DDGC_K5_PROF); this script points
DGC_HIP_LIB at it. Per case: one warm-up select, then one profiled select; prints the
global / LDS / single-wave phase times (wall clock, 10 ns ticks) and their step counts.

  python tools/k5_prof.py
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DGC_HIP_LIB"] = os.path.join(REPO, "adam-compression_amd", "lib", "k5prof", "libdgc_hip.so")
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd"), os.path.join(REPO, "tools")]

import torch  # noqa: E402

from dgc import _lib  # noqa: E402
from k5_bench import select_case  # noqa: E402


class K5Prof(ctypes.Structure):
    _fields_ = [("t", ctypes.c_uint64 * 8), ("steps", ctypes.c_uint32 * 4), ("sub", ctypes.c_uint64 * 8),
                ("bt", (ctypes.c_uint64 * 8) * 64), ("bn", ctypes.c_int64 * 64)]


def main():
    L = _lib.lib()
    L.dgc_k5_prof.restype = ctypes.c_int
    L.dgc_k5_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    cases = [(400_000, 400, 2_000), (262_144, 263, 8_200), (1_000_000, 1000, 6_000), (589_824, 590, 18_700),
             (2_000_000, 2000, 12_000), (4_000_000, 2360, 30_000), (2_359_296, 2360, 72_000),
             (10_000_000, 10_000, 100_000), (100_000_000, 102_761, 1_000_000)]
    if len(sys.argv) > 1:   # only the cases whose target candidate count is listed
        keep = {int(a) for a in sys.argv[1:]}
        cases = [c for c in cases if c[2] in keep]
    for n, k, target in cases:
        select_case(L, n, k, target, reps=1)
        best = None
        for _ in range(3):   # the minimum of each phase over 3 profiled runs
            torch.cuda.synchronize()
            _lib.check(L.dgc_k5_prof(None, 1))
            r = select_case(L, n, k, target, reps=1)
            torch.cuda.synchronize()
            p = K5Prof()
            _lib.check(L.dgc_k5_prof(ctypes.byref(p), 0))
            t = [x * 0.01 for x in p.t]   # us
            ph = dict(global_us=t[1] - t[0], load_us=t[2] - t[1], lds_us=t[3] - t[2], wave_us=t[4] - t[3],
                      store_us=t[5] - t[4], total_us=t[5] - t[0], g_pass1_us=p.sub[0] * 0.01,
                      g_pass2_us=p.sub[1] * 0.01, g_swap_us=p.sub[2] * 0.01, g_prepare_us=p.sub[3] * 0.01,
                      w_median_us=p.sub[4] * 0.01, w_pair_us=p.sub[5] * 0.01, w_swap_us=p.sub[6] * 0.01, g_pass2_loop_w0_us=p.sub[7] * 0.01)
            best = ph if best is None else {key: min(v, ph[key]) for key, v in best.items()}
        r.update({key: round(v, 1) for key, v in best.items()})
        r.update(steps_global=p.steps[0], steps_lds=p.steps[1], steps_wave=p.steps[2], g_mixed_tiles=p.steps[3])
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
