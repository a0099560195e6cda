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


def steady(N, dev, grads, out, steps=7, **kw):
    """Phase times (HIP events on the current stream) averaged over the last 3 of
    `steps` bucket steps on alternating gradients, as bench.py runs them."""
    b = DGCBucket(N, device=dev, **kw)
    names = ("compensate", "select", "allgather", "decompress")
    acc = dict.fromkeys(names + ("step",), 0.0)
    for s in range(steps):
        ev = {n: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for n in names}
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        b.step(grads[s % 2], out, ev)
        t1.record()
        torch.cuda.synchronize()
        if s >= steps - 3:
            for n in names:
                acc[n] += ev[n][0].elapsed_time(ev[n][1]) / 3
            acc["step"] += t0.elapsed_time(t1) / 3
    info = b.last_info()
    acc["full_passes"], acc["overflow_segments"] = info["full_passes"], info["overflow_segments"]
    del b
    return {k: round(v, 4) if isinstance(v, float) else v for k, v in acc.items()}


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
    b.spec[:2].copy_(spec)
    res["k1_list_ms"] = timeit(lambda: b.compensate(g))         # lists at 0.8 x the threshold
    b.spec[:2].copy_(spec)
    b.compensate(g)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    b.select()                                                   # served by the lists (one call:
    e1.record()                                                  # select masks vec, lists go stale)
    torch.cuda.synchronize()
    res["finish_ms"] = e0.elapsed_time(e1)
    res["selection"] = b.last_info()
    del b
    g2 = torch.randn(N, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    variants = {"default": {}, "fill_allgather": dict(fill="allgather"),
                "no_momentum_masking": dict(momentum_masking=False)}
    for name, kw in variants.items():                           # steady-state steps, like bench.py
        res[f"steady_{name}"] = steady(N, dev, (g, g2), out, **kw)
    b = DGCBucket(N, device=dev)
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
        ws = torch.empty(L.dgc_decompress_packed_workspace(N, W, k), dtype=torch.uint8, device=dev)

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
