"""CPU: the torch-CPU restatement of the reference's op sequence (oracle/torch_cpu.py)
on bf16 / fp16 parameters reproduces the reference's own 16-bit fixtures
(tests/golden/half.*, made by make_goldens.py's gen_half from /root/reference): the
transmitted indices in order, values, thresholds' counts, the 16-bit state and the
decompressed gradient of the rank-order concatenation. This pins the oracle the GPU
test (test_gpu_half.py) compares against."""
import random

import numpy as np
import torch

from oracle import synth
from oracle import torch_cpu as TC


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({4: np.uint32, 2: np.uint16, 8: np.uint64}[a.dtype.itemsize])


def run_case(case, fn_rank=None):
    """Replays one half.json case through oracle.torch_cpu; yields per (step, rank)
    (indices, values as float32, mmt, vec) and per step the dense output."""
    dt = getattr(torch, case["dtype"])
    N, W = case["N"], case["W"]
    numel, k, S, ks, stride = case["attrs"]
    mm = [torch.zeros(N, dtype=dt) for _ in range(W)]
    vv = [torch.zeros(N, dtype=dt) for _ in range(W)]
    random.seed(42)
    for s, step in enumerate(case["per_step"]):
        rstate = random.getstate()
        payload = []
        for q, rk in enumerate(step["ranks"]):
            random.setstate(rstate)
            start = random.randint(0, stride - 1) if numel != S else 0
            g = torch.from_numpy(synth.gradient(rk["seed"], N, case["kind"], case["scale"]).copy()).to(dt)
            TC.compensate(g, mm[q], vv[q], 0.9, case["nesterov"])
            vals, idx = TC.sparsify(vv[q], numel, k, S, ks, stride, start, resample=case["resample"])
            TC.update(mm[q], vv[q], idx, case["masking"])
            if case["fp16"]:
                vals = vals.to(torch.float16)
            if case["int32"]:
                idx = idx.to(torch.int32)
            payload.append((vals, idx))
            yield ("rank", s, q, idx, vals, mm[q], vv[q])
        cat_v = torch.cat([p[0] for p in payload]).to(dt)
        cat_i = torch.cat([p[1] for p in payload]).to(torch.int64)
        out = TC.decompress(cat_v, cat_i, torch.empty(N, dtype=dt), W)
        yield ("dense", s, None, out, None, None, None)


def test_torch_cpu_port_matches_half_goldens(golden_half):
    meta, arrays = golden_half
    for name, case in meta.items():
        for kind, s, q, a, b, m, v in run_case(case):
            if kind == "rank":
                key = f"{name}/s{s}/r{q}"
                assert np.array_equal(a.numpy(), arrays[key + "/indices"]), key
                assert np.array_equal(bits(b.float().numpy()), bits(arrays[key + "/values"])), key
                rk = case["per_step"][s]["ranks"][q]
                assert synth.digest(m.float().numpy()) == rk["mmt_sha"], key
                assert synth.digest(v.float().numpy()) == rk["vec_sha"], key
            else:
                flat = a.float().numpy()
                assert synth.digest(flat) == case["per_step"][s]["dense_sha"], (name, s)
