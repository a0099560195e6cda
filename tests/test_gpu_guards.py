"""The resample replay's multi-workgroup phase, recovered within the same step.

K5 replays torch's nth_element exactly; above ~100k candidates its global steps run
over G co-resident workgroups with cross-workgroup barriers (introselect.hpp). A
barrier that times out after the residency consensus voted GO leaves the queue's
partitions unreliable; k_nth_select then rebuilds the queue from the gather's candidate
keys and replays the whole nth_element on one workgroup in the same call (k5_status
DGC_K5_FALLBACK | DGC_K5_RECOVERED), so the step's payload is still the reference's.
A barrier cannot be made to time out on purpose, so DGC_K5_FORCE_BROKEN=1 sends every
replayed tensor down that path (its queue first overwritten with garbage): DGCBucket,
DGCBatch and DistributedOptimizer(batch=True) must produce exactly the healthy run's
outputs and state, in the same step, with no raise.
"""
import random

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _tied(n, m, step, seed):
    """Small noise plus m elements tied at one large value: the sampled threshold lands on
    the tie, m > 1.3 k candidates -> the resample branch on K5's path (m < 64 k), with
    the k boundary inside the tie (the exact replay, not the set path)."""
    gen = torch.Generator(device=DEV).manual_seed(seed + 17 * step)
    g = torch.randn(n, generator=gen, device=DEV) * 1e-3
    idx = torch.randperm(n, generator=gen, device=DEV)[:m]
    g[idx] = 5.0 + step
    return g


def _bits(t):
    return t.detach().contiguous().view(torch.int32).cpu()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("m", [60_000, 150_000], ids=["one-workgroup", "global-phase"])
def test_batch_recovers_broken_replay(m, monkeypatch):
    _need_gpu()
    from dgc.batch import DGCBatch

    def run(force):
        if force:
            monkeypatch.setenv("DGC_K5_FORCE_BROKEN", "1")
        else:
            monkeypatch.delenv("DGC_K5_FORCE_BROKEN", raising=False)
        b = DGCBatch([("w", (2000, 1000)), ("v", (5000,))], compress_ratio=0.01, device=DEV, seed=1)
        outs, infos = [], []
        for s in range(3):
            b.grad_flat.zero_()
            b.grad("w").copy_(_tied(2_000_000, m, s, 5).view(2000, 1000))
            b.grad("v").copy_(torch.randn(5000, generator=torch.Generator(device=DEV).manual_seed(s), device=DEV))
            outs.append(_bits(b.step()))
            infos.append(b.infos())   # raises on an unrecovered DGC_K5_BROKEN
        b.status.check(sync=True)
        return outs, infos, _bits(b.vec_flat), _bits(b.mmt_flat)

    healthy, forced = run(False), run(True)
    for s, (h, f) in enumerate(zip(healthy[0], forced[0])):
        assert torch.equal(h, f), s
    assert torch.equal(healthy[2], forced[2]) and torch.equal(healthy[3], forced[3])
    replayed = 0
    for hi, fi in zip(healthy[1], forced[1]):
        w_h, w_f = hi[0], fi[0]
        assert w_h["branch"] == w_f["branch"] and not w_h["k5_recovered"], (w_h, w_f)
        if w_h["branch"] == "resample" and w_h["tie_rule"] == "exact":   # step 0: the tie holds the boundary
            replayed += 1
            assert w_f["k5_recovered"], w_f
    assert replayed >= 1


@pytest.mark.timeout(180)
def test_bucket_recovers_broken_replay(monkeypatch):
    _need_gpu()
    from dgc.bucket import DGCBucket
    n = 2_000_000

    def run(force):
        if force:
            monkeypatch.setenv("DGC_K5_FORCE_BROKEN", "1")
        else:
            monkeypatch.delenv("DGC_K5_FORCE_BROKEN", raising=False)
        b = DGCBucket(n, compress_ratio=0.01, device=DEV, seed=3)
        out = torch.empty(n, device=DEV)
        res = []
        for s in range(3):
            b.step(_tied(n, 150_000, s, 9), out)
            info = b.last_info()   # raises on an unrecovered DGC_K5_BROKEN
            res.append((_bits(out), info))
        b.status.check(sync=True)
        return res, _bits(b.vec), _bits(b.mmt)

    healthy, forced = run(False), run(True)
    replayed = 0
    for (ho, hi), (fo, fi) in zip(healthy[0], forced[0]):
        assert torch.equal(ho, fo)
        assert hi["branch"] == fi["branch"] and not hi["k5_recovered"]
        if hi["branch"] == "resample" and hi["tie_rule"] == "exact":
            replayed += 1
            assert fi["k5_recovered"], fi
    assert replayed >= 1
    assert torch.equal(healthy[1], forced[1]) and torch.equal(healthy[2], forced[2])


@pytest.mark.timeout(180)
def test_batched_optimizer_recovers_broken_replay(monkeypatch):
    """DistributedOptimizer(batch=True) at W = 1 (HOROVOD_ELASTIC=1 registers the hooks,
    dgc/horovod/optimizer.py:79-80): the weight's gradient holds a tied group that
    resamples on K5's path (the first step); the forced recovery yields the same weights."""
    _need_gpu()
    from dgc.compression import DGCCompressor
    from dgc.horovod import DistributedOptimizer
    from dgc.memory import DGCSGDMemory
    monkeypatch.setenv("HOROVOD_ELASTIC", "1")

    def run(force):
        if force:
            monkeypatch.setenv("DGC_K5_FORCE_BROKEN", "1")
        else:
            monkeypatch.delenv("DGC_K5_FORCE_BROKEN", raising=False)
        torch.manual_seed(0)
        random.seed(0)   # the sample starts: the reference's Python-global random.randint draws
        model = torch.nn.Linear(2000, 1000).to(DEV)
        comp = DGCCompressor(0.01, memory=DGCSGDMemory(momentum=0.9))
        comp.memory.initialize(model.named_parameters())
        comp.initialize([(n, p) for n, p in model.named_parameters() if p.dim() > 1])
        opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1),
                                   named_parameters=model.named_parameters(), compression=comp, batch=True)
        recovered = []
        for s in range(3):
            opt.zero_grad()
            model.weight.grad = _tied(2_000_000, 150_000, s, 11).view(1000, 2000)
            model.bias.grad = torch.full((1000,), 0.01 * (s + 1), device=DEV)
            for _, hook in reversed(opt._hook_fns):
                hook()
            opt.step()
            b = opt._batched._plan["batch"]
            b.status.check(sync=True)
            inf = b.infos()[0]
            recovered.append(inf["k5_recovered"])
            if s == 0:   # the tie holds the k boundary: the exact replay
                assert inf["branch"] == "resample" and inf["tie_rule"] == "exact", inf
        assert recovered[0] == force and (force or not any(recovered)), recovered
        return _bits(model.weight), _bits(model.bias)

    assert all(torch.equal(a, b) for a, b in zip(run(False), run(True)))
