"""Momentum-correction memory for DGC — drop-in for the reference ``dgc/memory.py``.

Same classes, constructor arguments, methods and state layout as the reference
(``Memory`` static API, dgc/memory.py:9-28; ``DGCSGDMemory``, dgc/memory.py:31-88).
The arithmetic runs in ``libdgc_hip.so`` on the MI355X:

* ``compensate``  -> ``dgc_compensate`` (K1: one fused streaming pass, fp32 with the
  reference's two separate roundings, no FMA contraction);
* ``update``      -> ``dgc_mask_indices`` (the same masking that ``dgc_compress``
  fuses into its emit kernel when the compressor drives this memory).

``momentums`` / ``velocities`` stay plain param-shaped tensors of the parameter's dtype
keyed by name, so ``state_dict`` / ``load_state_dict`` and checkpoints are unchanged.
bf16 / fp16 parameters run ``dgc_compensate16`` / ``dgc_mask_indices16``: every op of
the reference rounds to the dtype, as ATen does on a 16-bit tensor.
"""
import ctypes

import torch

from . import _lib
from . import comm

__all__ = ["Memory", "DGCSGDMemory"]


class Memory:
    """No-op memory (dgc/memory.py:9-28)."""

    @staticmethod
    def initialize(*args, **kwargs):
        pass

    @staticmethod
    def compensate(tensor, *args, **kwargs):
        return tensor

    @staticmethod
    def update(*args, **kwargs):
        pass

    @staticmethod
    def state_dict():
        return None

    @staticmethod
    def load_state_dict(state_dict):
        pass


class DGCSGDMemory(Memory):
    """Memory for momentum correction in DGC for momentum SGD (dgc/memory.py:31-88)."""

    def __init__(self, momentum=0.9, nesterov=False, gradient_clipping=None, momentum_masking=True):
        self.gradient_clipping = gradient_clipping
        self.momentum_masking = momentum_masking
        self.momentum = momentum
        self.nesterov = nesterov
        self.momentums = {}
        self.velocities = {}
        self._status = {}   # device -> StatusSink: update() with an index outside the state
        # callables run before the state is read or replaced: a batched step
        # (dgc/horovod/batched.py) applies a deferred momentum masking there
        self._before_read = []

    def _sync(self):
        for fn in self._before_read:
            fn()
        self.check()

    def check(self, sync=False):
        """Raises if an ``update`` issued earlier got an index outside [-n, n) (the
        reference's index_fill_ raises there, dgc/memory.py:76-77): the kernel stores a
        flag in pinned host memory, read here for free at every call (``sync=True``
        waits for the stream first)."""
        for sink in self._status.values():
            sink.check(sync)

    def initialize(self, named_parameters):
        """zeros_like per parameter (dgc/memory.py:43-48)."""
        if comm.rank() == 0:
            print("=> initializing dgc sgd memory")
        self._sync()
        for name, param in named_parameters:
            self.momentums[name] = torch.zeros_like(param.data)
            self.velocities[name] = torch.zeros_like(param.data)

    # ------------------------------------------------------------------ K1
    def _clip(self, grad):
        return self.gradient_clipping(grad) if self.gradient_clipping is not None else grad

    def state_of(self, name, like, accumulate=True, what="DGCSGDMemory.compensate"):
        """(momentum, velocity or None) of ``name``, checked before their pointers reach a
        kernel: contiguous tensors of ``like``'s dtype, device and size. ``load_state_dict``
        rebinds them to whatever the checkpoint holds (a CPU map_location, fp32 state for a
        16-bit parameter); the reference's ATen ops would raise on the device mismatch and
        promote the dtype, the kernels would fault or misread — so this raises instead."""
        out = []
        for kind, store in (("momentum", self.momentums), ("velocity", self.velocities if accumulate else None)):
            if store is None:
                out.append(None)
                continue
            t = store[name]
            _lib.require_cuda_float(t, f"{what} ({kind} of {name})")
            if t.dtype != like.dtype or t.device != like.device or t.numel() != like.numel():
                raise TypeError(f"{what}: {kind} of {name} is {t.dtype} [{t.numel()}] on {t.device}, the gradient "
                                f"{like.dtype} [{like.numel()}] on {like.device}; load the state with the "
                                "parameter's dtype and device")
            out.append(t)
        return out[0], out[1]

    def compensate(self, grad, name, accumulate=True):
        """Momentum correction + local accumulation (dgc/memory.py:50-70).

        accumulate=True returns ``velocities[name]`` itself (updated in place);
        accumulate=False (dense tensors) returns a new tensor."""
        self._sync()
        grad = self._clip(grad)
        g = grad.contiguous()
        dt = _lib.require_cuda_float(g, "DGCSGDMemory.compensate")
        mmt, _ = self.state_of(name, g, accumulate)
        L = _lib.lib()
        stream = _lib.stream_of(g.device)
        if dt in _lib.HALF:
            return self._compensate16(g, name, accumulate)
        if accumulate:
            vec = self.velocities[name]
            _lib.check(L.dgc_compensate(_lib.ptr(g), _lib.ptr(mmt), _lib.ptr(vec), None, mmt.numel(),
                                        float(self.momentum), int(bool(self.nesterov)), 1, None, 0, 1, 0,
                                        stream), "dgc_compensate")
            return vec
        out = torch.empty_like(mmt)
        _lib.check(L.dgc_compensate(_lib.ptr(g), _lib.ptr(mmt), None, _lib.ptr(out), mmt.numel(),
                                    float(self.momentum), int(bool(self.nesterov)), 0, None, 0, 1, 0,
                                    stream), "dgc_compensate")
        return out

    def _compensate16(self, g, name, accumulate, vec32=None):
        """compensate on a bf16 / fp16 state (K1-16); vec32: optional fp32 image of the
        new velocity for the selection (the compressor's fused path)."""
        mmt, _ = self.state_of(name, g, accumulate)
        L = _lib.lib()
        dt = _lib.VD[g.dtype]
        stream = _lib.stream_of(g.device)
        if accumulate:
            vec = self.velocities[name]
            _lib.check(L.dgc_compensate16(_lib.ptr(g), _lib.ptr(mmt), _lib.ptr(vec), None, _lib.ptr(vec32),
                                          mmt.numel(), float(self.momentum), int(bool(self.nesterov)), 1, dt,
                                          stream), "dgc_compensate16")
            return vec
        out = torch.empty_like(mmt)
        _lib.check(L.dgc_compensate16(_lib.ptr(g), _lib.ptr(mmt), None, _lib.ptr(out), None, mmt.numel(),
                                      float(self.momentum), int(bool(self.nesterov)), 0, dt, stream),
                   "dgc_compensate16")
        return out

    def update(self, name, ctx):
        """Zero the transmitted slots (dgc/memory.py:72-77)."""
        self._sync()
        indices = ctx[0]
        vec = self.velocities[name]
        dt = _lib.require_cuda_float(vec, "DGCSGDMemory.update")
        mmt, _ = self.state_of(name, vec, False, "DGCSGDMemory.update")
        idx = indices.reshape(-1)
        if idx.dtype not in _lib.ID:
            idx = idx.to(torch.int64)
        idx = idx.contiguous()
        sink = self._status.get(vec.device)
        if sink is None:
            sink = self._status[vec.device] = _lib.StatusSink("DGCSGDMemory.update", vec.device)
        L = _lib.lib()
        fn = L.dgc_mask_indices16 if dt in _lib.HALF else L.dgc_mask_indices
        _lib.check(fn(_lib.ptr(mmt) if self.momentum_masking else None, _lib.ptr(vec),
                      vec.numel(), _lib.ptr(idx), _lib.ID[idx.dtype], idx.numel(),
                      ctypes.c_void_p(sink.index_flag), _lib.stream_of(vec.device)), "dgc_mask_indices")

    def state_dict(self):
        self._sync()
        return dict(momentums=self.momentums, velocities=self.velocities)

    def load_state_dict(self, state_dict):
        self._sync()
        momentums = state_dict["momentums"]
        velocities = state_dict["velocities"]
        for name in self.momentums.keys():
            if name in momentums:
                self.momentums[name] = momentums[name]
                self.velocities[name] = velocities[name]
