"""DistributedOptimizer(batch=True) at W = 1 against the reference's per-tensor hook path
(dgc/horovod/optimizer.py:91-187), on the same gradients and sample starts.

The batched step reads every gradient where autograd left it (K1's pointer table), runs
the dense tensors through one multi-tensor compensate (fp16 wire rounding fused) and
decompresses into its own output buffer, whose views become p.grad. Everything it
produces — the gradients handed to the wrapped optimizer, the momentum and velocity
state — must equal the per-tensor path's bit for bit, whatever autograd's gradients look
like: fresh tensors (zero_grad(set_to_none=True), torch's default), the previous step's
output views zeroed in place (set_to_none=False), a gradient that is not 16-B aligned
(copied first), or one whose hook never fired (compressed in synchronize(), after the
others, as the reference does). (A non-contiguous gradient is not one the reference
takes: its compress keeps `tensor.data.view(numel)`, dgc/compression.py:167.)
"""
import random

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

SHAPES = [("conv.weight", (64, 3, 7, 7)), ("bn.weight", (64,)), ("bn.bias", (64,)),
          ("odd.weight", (333, 7)), ("fc.weight", (1000, 512)), ("fc.bias", (1000,)), ("tiny.weight", (3, 5)),
          ("big.weight", (512, 512, 3, 3)), ("late.weight", (16, 16))]


def _run(batch, fp16, modes, monkeypatch, dtype=torch.float32, on_step=None):
    """The steps ``modes`` through DistributedOptimizer(batch=...); ``on_step(opt, grads)``
    after each synchronize(), with the gradients autograd handed over."""
    from dgc.compression import DGCCompressor
    from dgc.horovod import DistributedOptimizer
    from dgc.memory import DGCSGDMemory
    monkeypatch.setenv("HOROVOD_ELASTIC", "1")
    named = [(n, torch.nn.Parameter(torch.zeros(s, device=DEV, dtype=dtype))) for n, s in SHAPES]
    comp = DGCCompressor(0.01, memory=DGCSGDMemory(momentum=0.9, nesterov=True), fp16_values=fp16,
                         int32_indices=fp16)
    comp.memory.initialize(named)
    comp.initialize([(n, p) for n, p in named if p.dim() > 1])
    opt = DistributedOptimizer(torch.optim.SGD([p for _, p in named], lr=0.0), named_parameters=named,
                               compression=comp, batch=batch)
    random.seed(7)
    gen = torch.Generator(device=DEV).manual_seed(11)
    hooks = list(reversed(opt._hook_fns))
    late = dict(named)["late.weight"]
    out = []
    for step, mode in enumerate(modes):
        for i, (n, p) in enumerate(named):
            g = torch.randn(p.shape, generator=gen, device=DEV) * (1e-3 * (1 + i))
            if step % 2:   # a heavy-tailed step: the adaptation loop and the resample run
                g = g * torch.rand(p.shape, generator=gen, device=DEV).pow(8) * 50
            g = g.to(dtype)
            if mode == "inplace" and p.grad is not None:
                p.grad.add_(g)          # zero_grad(set_to_none=False) then backward's accumulation
            elif mode == "unaligned" and n in ("fc.weight", "bn.bias"):
                buf = torch.empty(p.numel() + 1, device=DEV, dtype=dtype)
                buf[1:].copy_(g.view(-1))
                p.grad = buf[1:].view(p.shape)   # 4-B aligned only
            else:
                p.grad = g.clone()
        grads = {n: p.grad.clone() for n, p in named} if on_step else None
        for p, hook in hooks:
            if p is not late:   # late.weight's hook never fires
                hook()
        opt.synchronize()
        torch.cuda.synchronize()
        if on_step:
            on_step(opt, grads)
        res = {n: (p.grad.clone() if p.grad is not None else None) for n, p in named}
        st = comp.memory.state_dict()
        res.update({f"m:{n}": t.clone() for n, t in st["momentums"].items()})
        res.update({f"v:{n}": t.clone() for n, t in st["velocities"].items()})
        out.append(res)
        opt.zero_grad(set_to_none=(modes[step + 1] != "inplace") if step + 1 < len(modes) else True)
    return out


def _bits(t):
    return t.contiguous().view(torch.int32 if t.element_size() == 4 else torch.int16)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16], ids=["fp32", "bf16", "f16"])
@pytest.mark.parametrize("fp16", [False, True], ids=["wire-dtype-int64", "wire-fp16-int32"])
@pytest.mark.parametrize("batch", [True, "sparse"], ids=["batch", "batch-sparse"])
def test_batched_optimizer_equals_per_tensor(batch, fp16, dtype, monkeypatch):
    """16-bit parameters (bf16 / fp16) run the batch's 16-bit engine (K1-16, the
    selection on the velocity's fp32 image, the 16-bit masking and decompress; "sparse"
    falls back to the dense zero_() there); the per-tensor path they are compared with is
    pinned to the reference's own 16-bit fixtures (test_gpu_half.py)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    modes = ["fresh", "fresh", "inplace", "inplace", "unaligned", "fresh", "fresh"]
    want = _run(False, fp16, modes, monkeypatch, dtype)
    got = _run(batch, fp16, modes, monkeypatch, dtype)
    for step, (w, g) in enumerate(zip(want, got)):
        assert w.keys() == g.keys()
        for k in w:
            assert w[k] is not None and g[k] is not None, (step, k)
            assert torch.equal(_bits(w[k]), _bits(g[k])), (step, modes[step], k)
