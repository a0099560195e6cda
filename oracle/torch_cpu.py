"""torch-CPU restatement of the reference op sequence — the CPU BASELINE leg.

TEST/BENCH INFRASTRUCTURE ONLY (``bench.py``'s ``cpu_baseline`` leg and tests).
The reference itself cannot travel to the GPU box, so ``bench.py`` times this
restatement instead (``cpu_baseline.kind = "port"``). It issues the same ATen ops
in the same order as the reference, so its cost profile is the reference's:

* compensate          dgc/memory.py:50-63   (add_/mul_ passes)
* _sparsify           dgc/compression.py:109-153 (abs, strided slice, topk, ge,
                      nonzero, adaptation loop, gather)
* update              dgc/memory.py:72-77   (index_fill_)
* decompress          dgc/compression.py:179-194 (zero_, index_put_ accumulate, mul_)

Validated against the numpy oracle and the reference goldens in
tests/test_oracle_golden.py / tests/test_torch_cpu_port.py.
"""
import math

import torch

__all__ = ["compensate", "sparsify", "update", "decompress", "cpu_step"]


def compensate(grad, mmt, vec, momentum, nesterov, accumulate=True):
    if nesterov:
        mmt.add_(grad).mul_(momentum)
        if accumulate:
            vec.add_(mmt).add_(grad)
            return vec
        return mmt.add(grad)
    mmt.mul_(momentum).add_(grad)
    if accumulate:
        vec.add_(mmt)
        return vec
    return mmt.clone()


def sparsify(vec, numel, k, S, ks, stride, start, upper=1.3, lower=0.8, max_iters=10, resample=True):
    flat = vec.view(-1)
    imp = flat.abs()
    samples = imp if numel == S else imp[start::stride]
    thr = torch.topk(samples, ks, 0, largest=True, sorted=False)[0].min()
    idx = torch.ge(imp, thr).nonzero().view(-1)
    n = idx.numel()
    if numel > S:
        for _ in range(max_iters):
            if n > k:
                if n > k * upper:
                    if resample:
                        idx = idx[torch.topk(imp[idx], k, 0, largest=True, sorted=False)[1]]
                        break
                    thr = thr * upper
                else:
                    break
            elif n < lower * k:
                thr = thr * lower
            else:
                break
            idx = torch.ge(imp, thr).nonzero().view(-1)
            n = idx.numel()
    idx = idx[:k]
    return flat[idx], idx


def update(mmt, vec, idx, masking=True):
    if masking:
        mmt.view(-1).index_fill_(0, idx, 0)
    vec.view(-1).index_fill_(0, idx, 0)


def decompress(values, indices, out, world_size):
    out.zero_().index_put_([indices], values, accumulate=True)
    out.mul_(1.0 / world_size)
    return out


def cpu_step(grad, mmt, vec, out, attrs, start, momentum=0.9, nesterov=True, masking=True):
    """One DGC step for one rank at W=1: compensate -> sparsify -> update -> decompress."""
    numel, k, S, ks, stride = attrs
    compensate(grad, mmt, vec, momentum, nesterov)
    values, idx = sparsify(vec, numel, k, S, ks, stride, start)
    update(mmt, vec, idx, masking)
    decompress(values, idx, out, 1)
    return idx.numel()


def attributes(numel, ratio, sample_ratio=0.01):
    pct = int(math.ceil(numel * sample_ratio))
    cpr = int(math.ceil(2 / ratio))
    if numel <= cpr:
        stride, S = 1, numel
    else:
        need = max(pct, cpr)
        stride = int(math.ceil(numel / need / 32)) * 32 + 1
        S = numel // stride
        while S < need:
            stride -= 8
            S = numel // stride
    return numel, int(math.ceil(numel * ratio)), S, int(math.ceil(S * ratio)), stride
