"""K7-16: DGCSGD.step on bf16 / fp16 CUDA parameters through the fused kernel
(dgc_sgd_step16) reproduces the reference's own 16-bit run (tests/golden/sgd16.*: the
reference DGCSGD on CPU, one thread) bit for bit — parameters after every step and the
momentum buffers — over lengths that exercise the CPU kernels' vector body and scalar
tail, nesterov / plain, dampening, weight decay with and without momentum."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from test_sgd16_port import sgd16_module

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CASES = json.load(open(os.path.join(GOLDEN, "sgd16.json")))


@pytest.mark.parametrize("label", sorted(CASES))
def test_dgcsgd_16bit_fused_matches_reference(label, monkeypatch):
    from dgc import _lib
    from dgc.optim import DGCSGD
    mg = sgd16_module()
    cfg = CASES[label]
    arrays = np.load(os.path.join(GOLDEN, "sgd16.npz"))
    ci = [c[0] for c in mg.SGD16_CASES].index(label)
    dt = getattr(torch, cfg["dtype"])
    init, grads = mg.sgd16_inputs(torch.Generator().manual_seed(4000 + ci), dt)
    params = [torch.nn.Parameter(t.to(DEV)) for t in init]
    opt = DGCSGD(params, lr=cfg["lr"], momentum=cfg["momentum"], dampening=cfg["dampening"],
                 weight_decay=cfg["weight_decay"], nesterov=cfg["nesterov"])
    launched = []
    L = _lib.lib()
    real = L.dgc_sgd_step16

    def spy(*a):
        launched.append(a[5])
        return real(*a)
    monkeypatch.setattr(L, "dgc_sgd_step16", spy)
    for s in range(cfg["steps"]):
        for p, g in zip(params, grads[s]):
            p.grad = g.to(DEV)
        opt.step()
        for (name, _), p in zip(mg.SGD16_SHAPES, params):
            got = p.detach().cpu().view(torch.int16).numpy()
            assert np.array_equal(got, arrays[f"{label}/s{s}/p/{name}"]), (label, s, name)
    assert launched == [len(params)] * cfg["steps"]   # one fused launch per step, no ATen fallback
    for (name, _), p in zip(mg.SGD16_SHAPES, params):
        key = f"{label}/buf/{name}"
        if key in arrays:
            got = opt.state[p]["momentum_buffer"].cpu().view(torch.int16).numpy()
            assert np.array_equal(got, arrays[key]), (label, name)
