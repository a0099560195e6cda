"""DGC's SGD step — drop-in for the reference ``dgc/optim/sgd.py`` (``DGCSGD``, :9-71).

The gradient's momentum is already applied by ``DGCSGDMemory.compensate``, so the
optimizer keeps momentum only for the weight-decay term: with weight decay wd,
``d = wd * p``; ``buf = momentum * buf + (1 - dampening) * d`` (``buf = d`` on the
first step); ``d = d + momentum * buf`` (nesterov) or ``d = buf``; then
``p -= lr * (d + grad)``. Without weight decay ``p -= lr * grad``.

On the MI355X every parameter group is ONE fused pass per dtype (``dgc_sgd_step``,
K7 in ``csrc/sgd.hip``, for fp32; ``dgc_sgd_step16`` for bf16 / fp16): read p, grad
(+ the momentum buffer), write p (+ buffer), with the reference's torch-CPU rounding
(fp32: ``add(alpha)`` is one fused multiply-add; 16-bit: every op rounds to the
dtype, alpha too, with the CPU kernels' vector body / scalar tail — oracle
``dgcsgd_step16``, pinned to tests/golden/sgd16.*), so the weights are bit-identical to
the reference's. For 16-bit parameters "the reference's" means what the fixtures pin: a
ONE-thread CPU run on the AVX2 kernels (32-element vector body; tests/golden/
make_goldens.py sets torch.set_num_threads(1)). A multi-threaded CPU run gives every
parallel chunk of a tensor over 32768 elements its own scalar tail, the AVX512 kernels
a 64-element body, and a CUDA run one rounding with an fp32 alpha — parity with those
is unpinned. Every other parameter — on the CPU (the gloo plumbing tests), or on
the GPU but not a contiguous fp32 / bf16 / fp16 tensor with a contiguous gradient of
its dtype (channels_last convolutions, a non-contiguous view) — takes the reference's
own torch op sequence, as the reference accepts any of them. The optimizer state keeps
the reference's layout (``state[p]["momentum_buffer"]``).
"""
import ctypes

import torch
from torch.optim.optimizer import Optimizer, required

__all__ = ["DGCSGD"]


class DGCSGD(Optimizer):
    def __init__(self, params, lr=required, momentum=0, dampening=0, weight_decay=0, nesterov=False):
        if lr is not required and lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov))

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    _DTYPES = (torch.float32, torch.bfloat16, torch.float16)

    @staticmethod
    def _fusable(p):
        """A parameter K7 serves: contiguous CUDA weight and gradient of one dtype (fp32,
        bf16 or fp16; and, when it exists, momentum buffer) on one device."""
        g = p.grad
        return (p.is_cuda and p.dtype in DGCSGD._DTYPES and p.data.is_contiguous() and g.is_cuda
                and g.dtype == p.dtype and g.is_contiguous() and g.device == p.device)

    @staticmethod
    def _cpu_param(p, d_p, group, state):
        """The reference's op sequence (dgc/optim/sgd.py:50-68), for a parameter K7 does
        not serve (any device, dtype or layout)."""
        wd, mom = group["weight_decay"], group["momentum"]
        if wd == 0:
            p.add_(d_p, alpha=-group["lr"])
            return
        d = wd * p.data
        if mom != 0:
            buf = state.get("momentum_buffer")
            if buf is None:
                buf = state["momentum_buffer"] = d
            else:
                buf.mul_(mom).add_(d, alpha=1 - group["dampening"])
            d = d.add(buf, alpha=mom) if group["nesterov"] else buf
        p.add_(d.add(d_p), alpha=-group["lr"])

    def _fused_group(self, group, params):
        """One dgc_sgd_step(16) launch (per 48 tensors) over the group's CUDA parameters
        of one device and dtype."""
        from dgc import _lib
        wd, mom = float(group["weight_decay"]), float(group["momentum"])
        use_buf = wd != 0 and mom != 0
        n = len(params)
        dt = params[0].dtype
        P, G, B = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
        N, F = (ctypes.c_int64 * n)(), (ctypes.c_int32 * n)()
        keep = []
        for i, p in enumerate(params):
            g = p.grad
            if _lib.require_cuda_float(p.data, "DGCSGD.step") != dt or g.dtype != dt:
                raise ValueError("DGCSGD.step: a fused launch takes parameters and gradients of one dtype")
            _lib.require_cuda_float(g, "DGCSGD.step")
            if g.device != p.device:
                raise ValueError("DGCSGD.step: parameter and gradient on different devices")
            P[i], G[i], N[i] = p.data.data_ptr(), g.data_ptr(), p.numel()
            if use_buf:
                state = self.state[p]
                buf = state.get("momentum_buffer")
                F[i] = int(buf is None)
                if buf is None:
                    buf = state["momentum_buffer"] = torch.empty_like(p.data)
                if _lib.require_cuda_float(buf, "DGCSGD.step") != dt:
                    raise ValueError("DGCSGD.step: momentum buffer of another dtype")
                B[i] = buf.data_ptr()
            keep.append(g)
        dev = params[0].device
        L = _lib.lib()
        args = (P, G, B, N, F, n, float(group["lr"]), mom, float(group["dampening"]), wd, int(bool(group["nesterov"])))
        if dt == torch.float32:
            _lib.check(L.dgc_sgd_step(*args, _lib.stream_of(dev)), "dgc_sgd_step")
        else:
            _lib.check(L.dgc_sgd_step16(*args, _lib.VD[dt], _lib.stream_of(dev)), "dgc_sgd_step16")

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            by_dev = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                buf = self.state[p].get("momentum_buffer") if p in self.state else None
                if self._fusable(p) and (buf is None or (buf.dtype == p.dtype and buf.is_contiguous()
                                                         and buf.device == p.device)):
                    by_dev.setdefault((p.device, p.dtype), []).append(p)
                else:
                    self._cpu_param(p, p.grad, group, self.state[p])
            for params in by_dev.values():
                self._fused_group(group, params)
        return loss
