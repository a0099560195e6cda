"""Host-side logic of the drop-in classes (no GPU): attribute tuples, warmup
schedule, adaptation bounds, and the loud failure of the product path on CPU."""
import math

import pytest
import torch

from dgc.compression import DGCCompressor
from dgc.memory import DGCSGDMemory, Memory


def quiet(fn, *a, **kw):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **kw)


def test_attributes_match_reference(golden_attributes):
    rows = golden_attributes["rows"]
    by_cfg = {}
    for r in rows:
        by_cfg.setdefault((r["sample_ratio"], r["ratio"]), []).append(r)
    for (sr, ratio), group in by_cfg.items():
        comp = quiet(DGCCompressor, 0.001, sample_ratio=sr)
        comp.compress_ratio = ratio
        quiet(comp.initialize, [(f"t{r['numel']}", (r["numel"], [r["numel"]])) for r in group])
        for r in group:
            numel, shape, k, S, ks, stride = comp.attributes[f"t{r['numel']}"]
            assert [numel, k, S, ks, stride] == r["attrs"], (sr, ratio, r)
            assert shape == [r["numel"]]


def test_warmup_matches_reference(golden_attributes):
    for label, sched in golden_attributes["schedules"].items():
        comp = quiet(DGCCompressor, sched["base_ratio"], **sched["kwargs"])
        quiet(comp.initialize, [("w", (1000000, [1000, 1000]))])
        for epoch, (ratio, attrs) in enumerate(sched["per_epoch"]):
            quiet(comp.warmup_compress_ratio, epoch)
            assert comp.compress_ratio == ratio, (label, epoch)
            assert list(comp.attributes["w"][2:]) == attrs, (label, epoch)


def test_select_params_bounds():
    comp = quiet(DGCCompressor, 0.001)
    quiet(comp.initialize, [("w", (1000000, [1000000])), ("v", (3000, [3000]))])
    p = comp._select_params("w", True, True)
    assert (p.num_selects, p.upper_count, p.lower_count) == (1000, 1300, 800)
    assert p.upper == pytest.approx(1.3) and p.max_iters == 10 and p.resample == 1
    q = comp._select_params("v", False, False)
    k = 3
    assert q.upper_count == math.floor(k * 1.3) and q.lower_count == math.ceil(0.8 * k)


def test_int32_default_off_and_dtypes():
    comp = quiet(DGCCompressor, 0.01, fp16_values=True, int32_indices=True)
    quiet(comp.initialize, [("w", (5000, [5000]))])
    p = comp._select_params("w", True, True)
    assert (p.vdtype, p.idtype) == (1, 1)


def test_product_path_refuses_cpu_tensors():
    mem = DGCSGDMemory(momentum=0.9)
    comp = quiet(DGCCompressor, 0.01, memory=mem)
    w = torch.zeros(5000)
    quiet(mem.initialize, [("w", w)])
    quiet(comp.initialize, [("w", w)])
    with pytest.raises(RuntimeError, match="MI355X"):
        comp.compress(torch.randn(5000), "w")
    with pytest.raises(RuntimeError, match="MI355X"):
        mem.compensate(torch.randn(5000), "w")


def test_dense_branch_passthrough_and_memory_api():
    comp = quiet(DGCCompressor, 0.01, fp16_values=True)
    t = torch.randn(10)
    out, ctx = comp.compress(t, "bias")         # not in attributes -> dense path
    assert out.dtype == torch.float16 and ctx == ("bias", None, None, torch.float32, None, None)
    assert Memory.compensate(t) is t and Memory.state_dict() is None
    mem = DGCSGDMemory()
    quiet(mem.initialize, [("a", torch.zeros(3))])
    sd = mem.state_dict()
    mem2 = DGCSGDMemory()
    quiet(mem2.initialize, [("a", torch.ones(3))])
    mem2.load_state_dict(sd)
    assert mem2.momentums["a"] is sd["momentums"]["a"]


def test_distributed_optimizer_default_picks_batched_only_when_equivalent():
    """DistributedOptimizer's default batch="auto" (dgc.horovod.batched.auto) takes the
    batched step only where it computes what the per-tensor hooks would: not for host
    parameters, an overriding subclass, an op other than Average, mixed dtypes or a
    non-DGC compressor (the gloo CPU tests' oracle doubles keep their per-tensor calls)."""
    from dgc.comm import Average, Sum
    from dgc.horovod import batched

    class Sub(DGCCompressor):
        def compress(self, tensor, name):
            return super().compress(tensor, name)

    mem = DGCSGDMemory(momentum=0.9)
    comp = quiet(DGCCompressor, 0.01, memory=mem)
    cpu = [("w", torch.nn.Parameter(torch.zeros(4, 4)))]
    assert not batched.auto(comp, cpu, Average)                    # host parameters
    assert not batched.auto(quiet(Sub, 0.01, memory=mem), cpu, Average)
    assert not batched.auto(comp, cpu, Sum)
    assert not batched.auto(quiet(DGCCompressor, 0.01), cpu, Average)   # Memory, not DGCSGDMemory
    assert not batched.auto(quiet(DGCCompressor, 0.01, memory=mem, strided_sample=False), cpu, Average)
