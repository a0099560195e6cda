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
    res["k1_ms"] = timeit(lambda: b.compensate(g))
    res["finish_ms"] = timeit(b.select)        # threshold + selection + emit (lists from K1)
    res["selection"] = b.last_info()
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
        del pay
    print(json.dumps(res))


if __name__ == "__main__":
    main()
