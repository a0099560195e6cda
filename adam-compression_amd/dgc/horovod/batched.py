"""One grouped exchange per optimizer step for ``DistributedOptimizer(..., batch=True)``.

The reference compresses and exchanges tensor by tensor from the grad-accumulator
hooks (dgc/horovod/optimizer.py:91-155): per compressed tensor a compress, two
Horovod allgathers and a decompress; per dense tensor an allreduce and a
``compensate(accumulate=False)`` (dgc/compression.py:155-212). ``BatchedStep`` keeps
those numerics and runs the whole step as

    compressed tensors   dgc.batch.DGCBatch: ONE K1 launch over all of them, the
                         selections together, ONE packed payload -> ONE allgather
                         (RCCL over xGMI) -> ONE decompress, written back into the
                         gradients (the reference's decompress writes into p.grad)
    dense tensors        ONE flat allreduce (Average; fp16 on the wire when the
                         compressor casts) -> ONE compensate(accumulate=False)

with no host synchronisation. It does so by laying the parameters' state out flat:

* every compressed parameter's ``p.grad``, ``memory.momentums[name]`` and
  ``memory.velocities[name]`` become views of the batch's three flat buffers;
* every dense parameter's ``p.grad`` and momentum become views of two dense flat
  buffers; the dense result goes to a second gradient buffer (the reference's
  ``p.grad.set_(compensate(...))`` of a new tensor), and the two alternate by step.

Anything that rebinds those tensors (``zero_grad(set_to_none=True)`` followed by a
backward, ``memory.load_state_dict``, ``compressor.initialize``) is detected at the
next step and copied back into the flat layout, so the results never depend on it;
keeping the views (``zero_grad(set_to_none=False)``; torch's and so the wrapper's
default is ``set_to_none=True``) just avoids that copy.

Sample starts: one ``random.randint(0, stride - 1)`` per sampled compressed tensor,
drawn from Python's global ``random`` in the order the hooks fired — the order in
which the reference's hooks call ``compress`` (dgc/compression.py:118) — so the
selections, and the weights, are the reference's bit for bit.
"""
import math
import random

import torch

from .. import _lib
from .. import comm
from ..batch import DGCBatch
from ..comm import Average
from ..compression import DGCCompressor
from ..memory import DGCSGDMemory

__all__ = ["BatchedStep", "supported"]


def supported(compression):
    """The batched step covers DGCCompressor + DGCSGDMemory with strided sampling and no
    gradient clipping (everything else keeps the per-tensor path)."""
    mem = getattr(compression, "memory", None)
    return (isinstance(compression, DGCCompressor) and isinstance(mem, DGCSGDMemory)
            and compression.strided_sample and mem.gradient_clipping is None)


class BatchedStep:
    def __init__(self, compression, named_parameters):
        self.comp = compression
        self.mem = compression.memory
        self.named = [(n, p) for n, p in named_parameters if p.requires_grad]
        bad = sorted({str(p.dtype) for _, p in self.named if p.dtype != torch.float32})
        if bad:   # the engines (dgc_batch_*) are fp32; 16-bit parameters take the per-tensor path
            raise NotImplementedError(f"DistributedOptimizer(batch=True): fp32 parameters only (got {', '.join(bad)}); "
                                      "bf16 / fp16 parameters run with batch=False")
        self._plan = None
        self.mem._before_read.append(self.flush)

    # ------------------------------------------------------------------ layout
    def _plan_key(self):
        c = self.comp
        names = tuple(n for n, _ in self.named if c.compress_ratio < 1.0 and n in c.attributes)
        return (c.compress_ratio, names)

    def _build(self, key):
        """(Re)lays out the flat buffers, moving the current momentum / velocity / grad
        contents in (a no-op copy when they already live there)."""
        c, mem = self.comp, self.mem
        ratio, comp_names = key
        old_batch = self._plan["batch"] if self._plan else None
        if old_batch is not None:
            old_batch.flush()
        params = dict(self.named)
        dev = self.named[0][1].device
        plan = {"key": key, "batch": None, "comp": [], "dense": [], "parity": 0}
        if comp_names:
            shapes = [(n, tuple(params[n].shape)) for n in comp_names]
            b = DGCBatch(shapes, compress_ratio=ratio, momentum=mem.momentum, nesterov=mem.nesterov,
                         momentum_masking=mem.momentum_masking, sample_ratio=c.sample_ratio,
                         compress_upper_bound=c.compress_upper_bound, compress_lower_bound=c.compress_lower_bound,
                         max_adaptation_iters=c.max_adaptation_iters, resample=c.resample,
                         fp16_values=c.fp16_values, int32_indices=c.int32_indices, device=dev,
                         world_size=comm.size(), deferred_masking=True)
            for i, n in enumerate(comp_names):
                numel, _, k, S, ks, stride = c.attributes[n]
                if (k, S, ks, stride) != tuple(b.attrs[i]):
                    raise RuntimeError(f"batched DGC: attributes of {n} differ from the compressor's")
            plan["batch"] = b
            for n in comp_names:
                p = params[n]
                mv, vv, gv = b._view(b._mmt_flat, n), b._view(b._vec_flat, n), b._view(b.grad_flat, n)
                mv.copy_(mem.momentums[n])
                vv.copy_(mem.velocities[n])
                if p.grad is not None:
                    gv.copy_(p.grad)
                mem.momentums[n], mem.velocities[n] = mv, vv
                p.grad = gv
                plan["comp"].append((n, p))
        dense = [(n, p) for n, p in self.named if n not in set(comp_names)]
        if dense:
            offs, end = [], 0
            for _, p in dense:
                offs.append(end)
                end += -(-p.numel() // 4) * 4   # 16-B aligned views
            bufs = [torch.zeros(end, dtype=torch.float32, device=dev) for _ in range(3)]   # grad A, grad B, mmt
            plan["dense_bufs"], plan["dense_numel"] = bufs, end
            for (n, p), o in zip(dense, offs):
                mv = bufs[2][o: o + p.numel()].view(p.shape)
                mv.copy_(mem.momentums[n])
                mem.momentums[n] = mv
                gv = bufs[0][o: o + p.numel()].view(p.shape)
                if p.grad is not None:
                    gv.copy_(p.grad)
                p.grad = gv
                plan["dense"].append((n, p, o))
            if c.fp16_values:
                plan["dense_wire"] = torch.empty(end, dtype=torch.float16, device=dev)
        self._plan = plan

    def flush(self):
        """Applies a deferred momentum masking (before anyone reads the memory)."""
        if self._plan and self._plan["batch"] is not None:
            self._plan["batch"].flush()

    def _rebind(self):
        """Moves back into the flat layout whatever was rebound since the last step."""
        plan, mem = self._plan, self.mem
        b = plan["batch"]
        if b is not None:
            for n, p in plan["comp"]:
                for store, flat in ((mem.momentums, b._mmt_flat), (mem.velocities, b._vec_flat)):
                    view = b._view(flat, n)
                    if store[n].data_ptr() != view.data_ptr():
                        b.flush()
                        view.copy_(store[n])
                        store[n] = view
                gv = b._view(b.grad_flat, n)
                self._own_grad(p, gv)
        if plan["dense"]:
            cur = plan["dense_bufs"][plan["parity"]]
            for n, p, o in plan["dense"]:
                mv = plan["dense_bufs"][2][o: o + p.numel()].view(p.shape)
                if mem.momentums[n].data_ptr() != mv.data_ptr():
                    mv.copy_(mem.momentums[n])
                    mem.momentums[n] = mv
                self._own_grad(p, cur[o: o + p.numel()].view(p.shape))

    @staticmethod
    def _own_grad(p, view):
        if p.grad is None:
            view.zero_()
        elif p.grad.data_ptr() != view.data_ptr():
            view.copy_(p.grad)
        else:
            return
        p.grad = view

    # ------------------------------------------------------------------ step
    def step(self, hook_order):
        """compress -> exchange -> decompress for every parameter; ``hook_order`` lists
        the parameters in the order their hooks fired (the reference's compress order)."""
        key = self._plan_key()
        if self._plan is None or self._plan["key"] != key:
            self._build(key)
        self._rebind()
        plan = self._plan
        b = plan["batch"]
        handle = None
        if b is not None:
            index = {n: i for i, n in enumerate(b.names)}
            starts = [0] * len(b.names)
            seen = set()
            for n in list(hook_order) + [n for n, _ in plan["comp"]]:
                i = index.get(n)
                if i is None or i in seen:
                    continue
                seen.add(i)
                numel, _, _, S, _, stride = self.comp.attributes[n]
                if numel != S:
                    starts[i] = random.randint(0, stride - 1)   # dgc/compression.py:118
            b.compensate(starts)
            b.select()
            if b.world > 1:
                handle = comm.allgather_packed_async(b.payload, out=b.gathered)
        dense_handle = None
        if plan["dense"]:
            cur = plan["dense_bufs"][plan["parity"]]
            wire = plan.get("dense_wire")
            if wire is not None:
                wire.copy_(cur)   # compress: tensor.type(float16) (dgc/compression.py:175-177)
            dense_handle = comm.allreduce_async_(wire if wire is not None else cur, op=Average)
        if b is not None:
            if handle is not None:
                handle.wait()
            b.decompress(out_flat=b.grad_flat)   # into p.grad, as dgc/compression.py:191-194
        if dense_handle is not None:
            red = comm.synchronize(dense_handle)
            src = red.float() if red.dtype != torch.float32 else red
            nxt = plan["dense_bufs"][1 - plan["parity"]]
            mem = self.mem
            L = _lib.lib()
            _lib.check(L.dgc_compensate(_lib.ptr(src), _lib.ptr(plan["dense_bufs"][2]), None, _lib.ptr(nxt),
                                        plan["dense_numel"], float(mem.momentum), int(bool(mem.nesterov)), 0,
                                        None, 0, 1, 0, _lib.stream_of(nxt.device)), "dgc_compensate")
            for n, p, o in plan["dense"]:   # p.grad.set_(compensate(accumulate=False)) (:195-198)
                p.grad = nxt[o: o + p.numel()].view(p.shape)
            plan["parity"] = 1 - plan["parity"]

    def zero_grads(self):
        """zero_() of every gradient in place (the views stay bound)."""
        plan = self._plan
        if plan is None:
            return False
        if plan["batch"] is not None:
            plan["batch"].grad_flat.zero_()
        if plan["dense"]:
            plan["dense_bufs"][plan["parity"]].zero_()
        return True
