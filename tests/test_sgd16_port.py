"""DGCSGD.step on bf16 / fp16 parameters: the numpy restatement (oracle.dgcsgd_step16:
every ATen op rounded to the dtype, the CPU kernels' vector body / scalar tail) against
the reference's own run (tests/golden/sgd16.*) — the formula the K7-16 kernel follows."""
import importlib.util
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import dgc_oracle as O


def sgd16_module():
    spec = importlib.util.spec_from_file_location("make_goldens", os.path.join(GOLDEN, "make_goldens.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


CASES = json.load(open(os.path.join(GOLDEN, "sgd16.json")))


@pytest.mark.parametrize("label", sorted(CASES))
def test_sgd16_restatement_matches_reference(label):
    mg = sgd16_module()
    cfg = CASES[label]
    arrays = np.load(os.path.join(GOLDEN, "sgd16.npz"))
    ci = [c[0] for c in mg.SGD16_CASES].index(label)
    dt = getattr(torch, cfg["dtype"])
    init, grads = mg.sgd16_inputs(torch.Generator().manual_seed(4000 + ci), dt)
    ps = [t.float().numpy().reshape(-1) for t in init]
    bufs = [None] * len(ps)
    for s in range(cfg["steps"]):
        for j, (name, _) in enumerate(mg.SGD16_SHAPES):
            g = grads[s][j].float().numpy().reshape(-1)
            ps[j], bufs[j] = O.dgcsgd_step16(ps[j], g, bufs[j], cfg["lr"], cfg["momentum"], cfg["dampening"],
                                             cfg["weight_decay"], cfg["nesterov"], cfg["dtype"])
            want = torch.from_numpy(arrays[f"{label}/s{s}/p/{name}"]).view(dt).float().numpy().reshape(-1)
            assert np.array_equal(ps[j].view(np.uint32), want.view(np.uint32)), (label, s, name)
    for j, (name, _) in enumerate(mg.SGD16_SHAPES):
        key = f"{label}/buf/{name}"
        if key in arrays:
            want = torch.from_numpy(arrays[key]).view(dt).float().numpy().reshape(-1)
            assert np.array_equal(bufs[j].view(np.uint32), want.view(np.uint32)), (label, name)
