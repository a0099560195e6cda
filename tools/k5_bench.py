"""K5 (exact resample replay) cost by candidate count, and the candidate counts the
model workloads' resamples see. Run under `rocprofv3 --kernel-trace --stats` to get
k_nth_select's duration per case (one dgc_select call per case, in the order printed).

  python tools/k5_bench.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]

from dgc import _lib  # noqa: E402


def select_case(L, n, k, target, reps=3):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(n + k)
    vec = torch.randn(n, generator=g, device=dev)
    t0 = torch.topk(vec.abs(), target).values.min().view(1).contiguous()
    p = _lib.SelectParams()
    p.numel, p.num_selects, p.num_samples = n, k, n // 97
    p.upper_count, p.lower_count = int(k * 1.3), int(np.ceil(0.8 * k))
    p.upper, p.lower, p.max_iters, p.resample, p.masking = 1.3, 0.8, 10, 1, 1
    p.vdtype, p.idtype, p.update_memory = 0, 0, 0
    vals = torch.empty(k, device=dev)
    idx = torch.empty(k, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    info = torch.zeros(_lib.INFO_BYTES, dtype=torch.uint8, device=dev)
    wsz = L.dgc_select_workspace(n, k)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for _ in range(reps):
        ev[0].record()
        _lib.check(L.dgc_select(vec.data_ptr(), None, t0.data_ptr(), ctypes.byref(p), vals.data_ptr(),
                                idx.data_ptr(), cnt.data_ptr(), info.data_ptr(), ws.data_ptr(), wsz,
                                _lib.SYNC_DEVICE, _lib.stream_of(dev)), "dgc_select")
        ev[1].record()
        torch.cuda.synchronize()
        times.append(ev[0].elapsed_time(ev[1]))
    inf = _lib.SelectInfo.from_buffer_copy(info.cpu().numpy().tobytes())
    return dict(n=n, k=k, candidates=inf.candidates, branch=_lib.BRANCHES[inf.branch],
                tie_rule=_lib.TIE_RULES[inf.tie_rule], select_ms=min(times))


def model_candidates(model):
    from dgc import workloads
    from dgc.batch import DGCBatch
    comp, _ = workloads.split(getattr(workloads, model)())
    b = DGCBatch(comp, compress_ratio=1e-3, device="cuda:0", seed=42)
    gen = torch.Generator(device="cuda:0")
    out = []
    for s in range(6):
        gen.manual_seed(100 + s)
        for off, n in zip(b.offsets, b.numels):
            b.grad_flat[off: off + n] = torch.randn(n, generator=gen, device="cuda:0") * 1e-3
        b.compress()
        torch.cuda.synchronize()
        out.append(sorted(((i["candidates"], b.attrs[t][0]) for t, i in enumerate(b.infos())
                           if i["branch"] == "resample"), reverse=True)[:6])
    return out


def main():
    L = _lib.lib()
    cases = [(400_000, 400, 2_000), (1_000_000, 1000, 6_000), (2_000_000, 2000, 12_000),
             (4_000_000, 2360, 30_000), (4_000_000, 2360, 45_000), (4_000_000, 2360, 57_000),
             (10_000_000, 10_000, 100_000), (50_000_000, 20_000, 500_000),
             (100_000_000, 102_761, 1_000_000)]
    for n, k, target in cases:
        print(json.dumps(select_case(L, n, k, target)), flush=True)
    if os.environ.get("K5_MODELS", "1") == "1":
        for model in ("resnet50", "vgg16_bn"):
            print(json.dumps({model: model_candidates(model)}), flush=True)


if __name__ == "__main__":
    main()
