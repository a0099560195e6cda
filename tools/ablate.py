"""Phase ablations on one MI355X (timing only; parity lives in tests/).

  python tools/ablate.py [--numel 1e9]

Times, with HIP events on the current stream, 10 reps each:
  * dgc_compress_begin (K1 + sample + speculative lists) and dgc_compress_finish;
  * dgc_decompress_packed at W = 1, 2, 4, 8 (synthetic ascending payloads);
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adam-compression_amd"))

import torch  # noqa: E402

from dgc import _lib  # noqa: E402
from dgc.bucket import DGCBucket  # noqa: E402


def timeit(fn, reps=10):
    """Average ms of fn over reps (after one untimed call)."""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--numel", type=float, default=1e9)
    args = ap.parse_args()
    N = int(args.numel)
    dev = torch.device("cuda:0")
    L = _lib.lib()
    b = DGCBucket(N, device=dev)
    g = torch.randn(N, device=dev)
    out = torch.empty(N, device=dev)
    res = {}
    S = (N - 5 + b.stride - 1) // b.stride          # samples from start 5
    smp = torch.empty(S, device=dev)
    stream = _lib.stream_of(dev)

    def comp(samples):
        _lib.check(L.dgc_compensate(g.data_ptr(), b.mmt.data_ptr(), b.vec.data_ptr(), None, N, 0.9, 1, 1,
                                    smp.data_ptr() if samples else None, 5, b.stride, S if samples else 0,
                                    stream), "dgc_compensate")
    res["compensate_plain_ms"] = timeit(lambda: comp(False))     # K1 arithmetic only (3R2W)
    res["compensate_sample_ms"] = timeit(lambda: comp(True))     # + fused strided sample
    b.spec.fill_(float("inf"))
    res["k1_nolist_ms"] = timeit(lambda: b.compensate(g))       # listing K1, nothing listed
    b.compensate(g)
    b.select()
    t = b.last_info()["threshold"]
    spec = torch.tensor([0.8 * t, t], device=dev)
    b.spec.copy_(spec)
    res["k1_list_ms"] = timeit(lambda: b.compensate(g))         # lists at 0.8 x the threshold
    b.spec.copy_(spec)
    b.compensate(g)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    b.select()                                                   # served by the lists (one call:
    e1.record()                                                  # select masks vec, lists go stale)
    torch.cuda.synchronize()
    res["finish_ms"] = e0.elapsed_time(e1)
    res["selection"] = b.last_info()
    for fill in ("inline", "k1", "start"):                      # whole step, three decompress schedules
        bf = DGCBucket(N, device=dev, fill=fill)
        res[f"step_fill_{fill}_ms"] = timeit(lambda: bf.step(g, out), reps=5)
        del bf
    k = b.k
    stride, voff, ioff = b.rank_stride, b.voff, b.ioff
    for W in (1, 2, 4, 8):
        pay = torch.zeros(W * stride, dtype=torch.uint8, device=dev)
        for r in range(W):
            idx = torch.sort(torch.randperm(N, device=dev)[:k]).values
            vals = torch.randn(k, device=dev)
            row = pay[r * stride:(r + 1) * stride]
            row[:8].view(torch.int64).fill_(k)
            row[voff:voff + 4 * k].view(torch.float32).copy_(vals)
            row[ioff:ioff + 8 * k].view(torch.int64).copy_(idx)
        ws = torch.empty(L.dgc_decompress_workspace(N, W), dtype=torch.uint8, device=dev)

        def dec():
            _lib.check(L.dgc_decompress_packed(pay.data_ptr(), W, stride, k, 0, 0, out.data_ptr(), N, 1.0 / W,
                                               ws.data_ptr(), ws.numel(), _lib.stream_of(dev)))
        res[f"decompress_W{W}_ms"] = timeit(dec)

        def scat():
            _lib.check(L.dgc_scatter_packed(pay.data_ptr(), W, stride, k, 0, 0, out.data_ptr(), N, 1.0 / W,
                                            ws.data_ptr(), ws.numel(), _lib.stream_of(dev)))
        res[f"scatter_W{W}_ms"] = timeit(scat)
        del pay
    print(json.dumps(res))


if __name__ == "__main__":
    main()
