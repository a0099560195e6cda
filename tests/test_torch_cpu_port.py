"""Pin ``oracle/torch_cpu.py`` (the timed CPU-baseline port in bench.py) to the
reference's golden fixtures: every compress case, step by step — thresholds are
implied by the selected indices, which must equal the reference's IN ORDER (the
port calls the same torch.topk as dgc/compression.py:134-137), plus values, the
momentum / velocity digests and the decompressed dense gradient."""
import random

import numpy as np
import torch

from oracle import synth
from oracle import torch_cpu as T


def test_torch_cpu_port_matches_reference_goldens(golden_compress):
    meta, arrays = golden_compress
    torch.set_num_threads(1)       # index_put_(accumulate) in input order, like the goldens
    for name, case in meta.items():
        N = case["N"]
        numel, k, S, ks, stride = case["attrs"]
        mmt, vec, out = torch.zeros(N), torch.zeros(N), torch.empty(N)
        random.seed(42)
        kw = dict(resample=case["resample"], max_iters=case["extra"].get("max_adaptation_iters", 10))
        for s, step in enumerate(case["per_step"]):
            g = torch.from_numpy(synth.gradient(step["seed"], N, case["kind"], case["scale"]))
            start = random.randint(0, stride - 1) if numel != S else 0
            T.compensate(g, mmt, vec, 0.9, case["nesterov"])
            values, idx = T.sparsify(vec, numel, k, S, ks, stride, start, **kw)
            values = values.clone()
            T.update(mmt, vec, idx, case["masking"])
            key = f"{name}/s{s}"
            ref_idx = arrays[key + "/indices"].astype(np.int64)
            assert np.array_equal(idx.numpy(), ref_idx), key
            wv = values.numpy().astype(np.float16) if case["fp16"] else values.numpy()
            assert np.array_equal(wv.view(np.uint8), arrays[key + "/values"].view(np.uint8)), key
            assert synth.digest(mmt.numpy()) == step["mmt_sha"], key
            assert synth.digest(vec.numpy()) == step["vec_sha"], key
            dense = T.decompress(torch.from_numpy(wv.astype(np.float32)), idx, out, 1).numpy()
            nz = np.flatnonzero(dense.view(np.uint32))
            assert np.array_equal(nz, arrays[key + "/dec_nz_idx"]), key
            assert np.array_equal(dense[nz].view(np.uint32), arrays[key + "/dec_nz_val"].view(np.uint32)), key
