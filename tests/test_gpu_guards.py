"""The engines' per-step check of the resample replay's health (DGC_K5_BROKEN).

DGCBucket, DGCBatch and DistributedOptimizer(batch=True) run DGC_SYNC_DEVICE: no host
synchronisation per step, so the multi-workgroup replay's status (dgc_select_info.
k5_status) is never read on the way. The library stores a broken status into the
engine's pinned host word (status_sink); the next step reads it and raises. A barrier
cannot be made to time out on purpose, so DGC_K5_FORCE_BROKEN=1 makes the finish report
every resampled tensor as broken: the path from the kernel's status to the raise is the
one a real timeout takes. Without it, the same runs never raise.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _tied(n, step):
    # every element equal: the sampled threshold selects all n > 1.3 k -> the resample branch
    return torch.full((n,), 1.0 + step, device=DEV)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("force", [False, True], ids=["healthy", "forced-broken"])
def test_batch_raises_on_broken_replay(force, monkeypatch):
    _need_gpu()
    from dgc.batch import DGCBatch
    if force:
        monkeypatch.setenv("DGC_K5_FORCE_BROKEN", "1")
    b = DGCBatch([("w", (200, 1000)), ("v", (5000,))], compress_ratio=0.001, device=DEV, seed=1)
    for s in range(2):
        b.grad_flat.zero_()
        b.grad("w").copy_(_tied(200_000, s).view(200, 1000))
        b.grad("v").copy_(torch.randn(5000, device=DEV))
        if force and s == 1:
            with pytest.raises(RuntimeError, match="resample replay"):
                b.step()
            return
        b.step()
        torch.cuda.synchronize()   # the host may run ahead of the GPU: the check sees finished steps
        infos = {n: i for n, i in zip(b.names, b.infos())} if not force else None
        if infos is not None:
            assert infos["w"]["branch"] == "resample"
    torch.cuda.synchronize()
    b.status.check()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("force", [False, True], ids=["healthy", "forced-broken"])
def test_bucket_raises_on_broken_replay(force, monkeypatch):
    _need_gpu()
    from dgc.bucket import DGCBucket
    if force:
        monkeypatch.setenv("DGC_K5_FORCE_BROKEN", "1")
    n = 1 << 20
    b = DGCBucket(n, compress_ratio=0.001, device=DEV)
    out = torch.empty(n, device=DEV)
    b.step(_tied(n, 0), out)
    if force:
        with pytest.raises(RuntimeError, match="resample replay"):
            b.last_info()
        with pytest.raises(RuntimeError, match="resample replay"):
            b.step(_tied(n, 1), out)
    else:
        assert b.last_info()["branch"] == "resample"
        b.step(_tied(n, 1), out)
        torch.cuda.synchronize()
        b.status.check()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("force", [False, True], ids=["healthy", "forced-broken"])
def test_batched_optimizer_raises_on_broken_replay(force, monkeypatch):
    """DistributedOptimizer(batch=True) at W = 1 (HOROVOD_ELASTIC=1 registers the hooks,
    dgc/horovod/optimizer.py:79-80): a Linear layer whose weight gradient is all ones
    (loss = sum of the outputs of an all-ones input) resamples every step."""
    _need_gpu()
    from dgc.compression import DGCCompressor
    from dgc.horovod import DistributedOptimizer
    from dgc.memory import DGCSGDMemory
    monkeypatch.setenv("HOROVOD_ELASTIC", "1")
    if force:
        monkeypatch.setenv("DGC_K5_FORCE_BROKEN", "1")
    torch.manual_seed(0)
    model = torch.nn.Linear(1000, 300).to(DEV)
    comp = DGCCompressor(0.001, memory=DGCSGDMemory(momentum=0.9))
    comp.memory.initialize(model.named_parameters())
    comp.initialize(model.named_parameters())
    opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), named_parameters=model.named_parameters(),
                               compression=comp, batch=True)
    x = torch.ones(4, 1000, device=DEV)
    for step in range(3):
        opt.zero_grad()
        model(x).sum().backward()
        if force and step == 1:
            with pytest.raises(RuntimeError, match="resample replay"):
                opt.step()
            return
        opt.step()
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    opt._batched._plan["batch"].status.check()
    assert os.environ.get("DGC_K5_FORCE_BROKEN") is None
