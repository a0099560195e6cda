"""Why a resample does or does not take the multi-workgroup set path (k_bigset_*):
the scenario of tests/test_gpu_batch.py::test_batch_index_order_big_resample, one line
per step for the big tensor — branch, candidates, tie rule, and from the velocity the
k-th largest key against t_cur (the coarse bin it falls in, 4096 key units each, and
the keys in that bin; the path needs bin < 2047 and <= 65536 keys there).

  python tools/bigset_probe.py [steps] [numel]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]

import torch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    numel = int(float(sys.argv[2])) if len(sys.argv) > 2 else 20_000_000
    from dgc.batch import DGCBatch
    dev = torch.device("cuda:0")
    shapes = [("big", (numel,)), ("small", (300, 1000))]
    b = DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, device=dev, seed=5, resample_order="index")
    gen = torch.Generator(device=dev)
    for s in range(steps):
        gen.manual_seed(77 + s % 2)
        g = torch.zeros(b.flat_numel, device=dev)
        for off, n in zip(b.offsets, b.numels):
            g[off: off + n] = torch.randn(n, generator=gen, device=dev) * 1e-3
        b.grad_flat.copy_(g)
        b.compensate()
        v = b._vec_flat[b.offsets[0]: b.offsets[0] + numel].abs().clone()   # before the masking
        b.select()
        b.decompress()
        torch.cuda.synchronize()
        inf = b.infos()[0]
        row = {"step": s, "branch": inf["branch"], "candidates": inf["candidates"], "tie_rule": inf["tie_rule"],
               "threshold": inf["threshold"]}
        if inf["branch"] == "resample":
            k = b.attrs[0][0]
            keys = v.view(torch.int32)
            tkey = int(torch.tensor([inf["threshold"]], dtype=torch.float32).view(torch.int32).item())
            kth = int(torch.topk(keys, k).values.min().item())
            b0 = (kth - tkey) >> 12
            inbin = int(((keys >= tkey + (b0 << 12)) & (keys < tkey + ((b0 + 1) << 12))).sum().item())
            row.update(kth_over_t=float(torch.tensor([kth], dtype=torch.int32).view(torch.float32).item()
                                        / inf["threshold"]), coarse_bin=b0, keys_in_bin=inbin,
                       ties_at_kth=int((keys == kth).sum().item()))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
