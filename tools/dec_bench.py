"""Decompress-only timing at one world size (for rocprofv3 per-kernel breakdowns).

  python tools/dec_bench.py [--W 8] [--numel 1e9] [--reps 10]

Builds W synthetic packed payloads of k = N/1000 ascending random indices each (the
shape of the 1B-bucket allgather output), twice (this step's and the previous one's),
and times dgc_fill_zero, dgc_scatter_packed (sparse, onto a zeroed buffer),
dgc_decompress_packed (dense) and dgc_decompress_packed_over (the sparse re-zero of
the previous payload's entries + the scatter), `reps` times each; prints the average
ms of each (HIP events on the current stream).

Split exchange (dgc/exchange.py, --parts 2 4 ...): per part count, the sender's
dgc_payload_split of one rank's payload, and each phase's dgc_scatter_split on the
part-major gather buffer; the last phase is what stays exposed after the last
collective (the earlier phases run while the later parts are in flight).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adam-compression_amd"))

import torch  # noqa: E402

from dgc import _lib  # noqa: E402
from dgc.compression import _layout  # noqa: E402


def timeit(fn, reps):
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
    ap.add_argument("--W", type=int, default=8)
    ap.add_argument("--numel", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--parts", type=int, nargs="*", default=[2, 4])
    args = ap.parse_args()
    N, W = int(args.numel), args.W
    k = (N + 999) // 1000
    dev = torch.device("cuda:0")
    L = _lib.lib()
    stride, voff, ioff = _layout(k, torch.float32, torch.int64)
    gen = torch.Generator(device=dev).manual_seed(3)

    def payload():
        pay = torch.zeros(W * stride, dtype=torch.uint8, device=dev)
        for r in range(W):
            idx = torch.sort(torch.randperm(N, device=dev, generator=gen)[:k]).values
            row = pay[r * stride:(r + 1) * stride]
            row[:8].view(torch.int64).fill_(k)
            row[voff:voff + 4 * k].view(torch.float32).copy_(torch.randn(k, device=dev, generator=gen))
            row[ioff:ioff + 8 * k].view(torch.int64).copy_(idx)
            del idx
        return pay

    pay, prev = payload(), payload()
    out = torch.empty(N, device=dev)
    ws = torch.empty(L.dgc_decompress_packed_workspace(N, W, k), dtype=torch.uint8, device=dev)
    s = _lib.stream_of(dev)

    def fill():
        _lib.check(L.dgc_fill_zero(out.data_ptr(), N, s), "dgc_fill_zero")

    def scatter():
        _lib.check(L.dgc_scatter_packed(pay.data_ptr(), W, stride, k, 0, 0, out.data_ptr(), N, 1.0 / W,
                                        ws.data_ptr(), ws.numel(), s), "dgc_scatter_packed")

    def dense():
        _lib.check(L.dgc_decompress_packed(pay.data_ptr(), W, stride, k, 0, 0, out.data_ptr(), N, 1.0 / W,
                                           ws.data_ptr(), ws.numel(), s), "dgc_decompress_packed")

    def over():
        _lib.check(L.dgc_decompress_packed_over(pay.data_ptr(), prev.data_ptr(), W, stride, k, 0, 0, out.data_ptr(),
                                                N, 1.0 / W, ws.data_ptr(), ws.numel(), s),
                   "dgc_decompress_packed_over")

    res = {"W": W, "numel": N, "k": k,
           "fill_ms": timeit(fill, args.reps), "scatter_ms": timeit(scatter, args.reps),
           "dense_ms": timeit(dense, args.reps), "over_ms": timeit(over, args.reps)}
    for P in args.parts:
        if W * P > 64 or P < 2:
            continue
        res[f"split{P}"] = split_times(L, pay, stride, W, P, k, N, out, s, args.reps)
    print(json.dumps(res), flush=True)


def split_times(L, pay, stride, W, P, k, N, out, s, reps):
    import ctypes
    pc = ctypes.c_int64(0)
    pb = L.dgc_payload_split_layout(k, P, 0, 0, ctypes.byref(pc))
    dev = out.device
    split = torch.zeros(L.dgc_payload_split_bytes(k, P, 0, 0), dtype=torch.uint8, device=dev)
    g = torch.zeros(P * W * pb, dtype=torch.uint8, device=dev)

    def pack(r):
        _lib.check(L.dgc_payload_split(pay[r * stride:].data_ptr(), k, P, 0, 0, split.data_ptr(), s),
                   "dgc_payload_split")

    for r in range(W):
        pack(r)
        for p in range(P):
            g[(p * W + r) * pb:(p * W + r + 1) * pb].copy_(split[p * pb:(p + 1) * pb])
    ws = torch.empty(L.dgc_decompress_split_workspace(N, W, P, k), dtype=torch.uint8, device=dev)

    def phase(p):
        _lib.check(L.dgc_scatter_split(g.data_ptr(), W, P, p, k, 0, 0, out.data_ptr(), N, 1.0 / W, 0, ws.data_ptr(),
                                       ws.numel(), s), "dgc_scatter_split")

    phases = [0.0] * P
    for _ in range(reps):
        _lib.check(L.dgc_fill_zero(out.data_ptr(), N, s), "dgc_fill_zero")
        for p in range(P):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            phase(p)
            b.record()
            b.synchronize()
            phases[p] += a.elapsed_time(b) / reps
    return {"pack_ms": timeit(lambda: pack(0), reps), "phase_ms": phases, "exposed_ms": phases[-1]}


if __name__ == "__main__":
    main()
