"""DGC's SGD step (dgc/optim/sgd.py:9-71).

The gradient's momentum is already applied by ``DGCSGDMemory.compensate``, so the
optimizer keeps momentum only for the weight-decay term: with weight decay wd,
``d = wd * p``; ``buf = momentum * buf + (1 - dampening) * d`` (``buf = d`` on the
first step); ``d = d + momentum * buf`` (nesterov) or ``d = buf``; then
``p -= lr * (d + grad)``. Without weight decay ``p -= lr * grad``.

This step sits after the hot path; it runs as torch ops.
"""
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

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            wd, mom = group["weight_decay"], group["momentum"]
            damp, nest, lr = group["dampening"], group["nesterov"], group["lr"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if wd == 0:
                    p.add_(p.grad, alpha=-lr)
                    continue
                d = wd * p.data
                if mom != 0:
                    state = self.state[p]
                    buf = state.get("momentum_buffer")
                    if buf is None:
                        buf = state["momentum_buffer"] = d
                    else:
                        buf.mul_(mom).add_(d, alpha=1 - damp)
                    d = d.add(buf, alpha=mom) if nest else buf
                p.add_(d.add(p.grad), alpha=-lr)
        return loss
