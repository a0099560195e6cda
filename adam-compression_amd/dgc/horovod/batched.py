"""One grouped exchange per optimizer step for ``DistributedOptimizer(..., batch=True)``.

The reference compresses and exchanges tensor by tensor from the grad-accumulator
hooks (dgc/horovod/optimizer.py:91-155): per compressed tensor a compress, two
Horovod allgathers and a decompress; per dense tensor an allreduce and a
``compensate(accumulate=False)`` (dgc/compression.py:155-212). ``BatchedStep`` keeps
those numerics and runs the whole step as

    compressed tensors   dgc.batch.DGCBatch: ONE K1 launch over all of them, reading
                         every gradient where autograd left it (a table of p.grad
                         pointers in the kernel arguments, no copy), the selections
                         together, ONE packed payload -> ONE allgather (RCCL over xGMI)
                         -> ONE decompress into the batch's output buffer, whose views
                         become the new p.grad (the reference's decompress writes into
                         p.grad, dgc/compression.py:191-194)
    dense tensors        W = 1: ONE multi-tensor compensate(accumulate=False) straight
                         from the gradients (the fp16 wire's rounding fused); W > 1: ONE
                         gather (+ fp16 cast) into the TAIL of the same packed payload, so
                         the step's one allgather carries them too -> ONE compensate from
                         the gathered rows (dgc_compensate_ranks: the Average as the
                         rank-order sum / W in the wire dtype, the order the reference's
                         Horovod Average is restated in — an allreduce would sum in the
                         backend's order). A split exchange, or a step with no compressed
                         tensor, allgathers the dense values on their own.

with no host synchronisation and no per-parameter launch. The momentums and
velocities become views of the batch's flat buffers (``memory.momentums[name]`` /
``velocities[name]``); anything that rebinds them (``memory.load_state_dict``,
``compressor.initialize``) is detected at the next step and copied back in.

Gradients: whatever ``p.grad`` is at ``step()`` — a fresh tensor from backward after
the default ``zero_grad(set_to_none=True)``, or the previous step's output view zeroed
in place and accumulated into (``set_to_none=False``) — is read in place when it is a
contiguous, 16-B aligned fp32 tensor on the device (else copied into the batch's flat
gradient buffer first; a missing one counts as zeros).

The zero_() before the scatter (dgc/compression.py:191): ``fill="inline"`` (the
default) zeroes the whole output, as the reference does. ``fill="sparse"`` re-zeroes
only the previous step's gathered indices of the output when nothing wrote it since
(same storage, torch version counter unchanged — an in-place op on a p.grad view bumps
it); writes through ``p.grad.data`` or raw pointers do not, so only a training loop
that never writes the gradients that way (torch's optimizers, clip_grad_norm_ and
zero_grad do not) should opt in.

Sample starts: one ``random.randint(0, stride - 1)`` per sampled compressed tensor,
drawn from Python's global ``random`` in the order the hooks fired — the order in
which the reference's hooks call ``compress`` (dgc/compression.py:118) — so the
selections, and the weights, are the reference's bit for bit.
"""
import ctypes
import random

import torch

from .. import _lib
from .. import comm
from .._lib import glue as _glue
from ..batch import DGCBatch
from ..comm import Average
from ..compression import DGCCompressor
from ..memory import DGCSGDMemory

__all__ = ["BatchedStep", "supported", "auto"]


def supported(compression):
    """The batched step covers DGCCompressor + DGCSGDMemory with strided sampling and no
    gradient clipping (everything else keeps the per-tensor path)."""
    mem = getattr(compression, "memory", None)
    return (isinstance(compression, DGCCompressor) and isinstance(mem, DGCSGDMemory)
            and compression.strided_sample and mem.gradient_clipping is None)


def auto(compression, named_parameters, op):
    """``DistributedOptimizer(batch="auto")``, the default: the batched step whenever it
    computes exactly what the per-tensor hooks would — ``supported``, Average, the
    compressor's and memory's own compress / decompress / communicate / synchronize /
    compensate / update (a subclass that overrides one keeps the per-tensor calls it
    expects), and the trainable parameters on the MI355X sharing one dtype of fp32, bf16
    or fp16. Anything else runs per tensor, as the reference does."""
    if op != Average or not supported(compression):
        return False
    for base, obj, names in ((DGCCompressor, compression, ("compress", "decompress", "communicate", "synchronize")),
                             (DGCSGDMemory, compression.memory, ("compensate", "update"))):
        if any(getattr(type(obj), n) is not getattr(base, n) for n in names):
            return False
    params = [p for _, p in named_parameters if p.requires_grad]
    dts = {p.dtype for p in params}
    return (bool(params) and all(p.is_cuda for p in params) and len(dts) == 1
            and dts <= {torch.float32, torch.bfloat16, torch.float16})


def _draw():
    """random.randint(0, stride - 1) of dgc/compression.py:118, as the function that
    consumes the generator the same way (randint(0, b) = randrange(0, b + 1) = the
    generator's _randbelow(b + 1)) at a third of the call cost; randint where the
    module lacks it."""
    rb = getattr(getattr(random, "_inst", None), "_randbelow", None)
    return rb if rb is not None else (lambda s: random.randint(0, s - 1))


class BatchedStep:
    def __init__(self, compression, named_parameters, fill="inline"):
        if fill not in ("inline", "sparse"):
            raise ValueError(f"batched DGC: fill must be 'inline' or 'sparse', not {fill!r}")
        self.comp = compression
        self.mem = compression.memory
        self.fill = fill
        self.named = [(n, p) for n, p in named_parameters if p.requires_grad]
        dts = sorted({str(p.dtype) for _, p in self.named})
        if len(dts) > 1 or any(p.dtype not in (torch.float32,) + _lib.HALF for _, p in self.named):
            # one flat layout per step: fp32, or bf16 / fp16 throughout (mixed dtypes: batch=False)
            raise NotImplementedError(f"DistributedOptimizer(batch=True): the parameters must share one dtype of "
                                      f"fp32, bf16 or fp16 (got {', '.join(dts)}); mixed dtypes run with batch=False")
        self.dtype = self.named[0][1].dtype if self.named else torch.float32
        self.half = self.dtype in _lib.HALF
        self._plan = None
        self.mem._before_read.append(self.flush)
        _lib.glue()   # the host glue must be there (fails loudly, like the library)

    # ------------------------------------------------------------------ layout
    def _plan_key(self):
        c = self.comp
        return (c.compress_ratio, c.layout_epoch, len(c.attributes))

    def _build(self, key):
        """(Re)lays out the flat buffers, moving the current momentum / velocity contents
        in (a no-op copy when they already live there)."""
        c, mem = self.comp, self.mem
        old_batch = self._plan["batch"] if self._plan else None
        if old_batch is not None:
            old_batch.flush()
        comp_names = [n for n, _ in self.named if c.compress_ratio < 1.0 and n in c.attributes]
        params = dict(self.named)
        dev = self.named[0][1].device
        plan = {"key": key, "batch": None, "comp": [], "dense": [], "dev": dev, "state": [], "dense_state": []}
        dense = [(n, p) for n, p in self.named if n not in set(comp_names)]
        offs, end = [], 0
        for _, p in dense:
            offs.append(end)
            end += -(-p.numel() // 4) * 4   # 16-B aligned views
        # fp32 parameters exchanging (W > 1): the dense wire values ride in the packed
        # payload's tail, summed in rank order after the ONE allgather (dgc_compensate_ranks)
        exchanging = comm.size() > 1 or comm.one_rank_collectives()
        wire_dt = torch.float16 if c.fp16_values else torch.float32
        dense_bytes = end * torch.empty(0, dtype=wire_dt).element_size() if dense and exchanging and not self.half else 0
        if comp_names:
            shapes = [(n, tuple(params[n].shape)) for n in comp_names]
            b = DGCBatch(shapes, compress_ratio=c.compress_ratio, momentum=mem.momentum, nesterov=mem.nesterov,
                         momentum_masking=mem.momentum_masking, sample_ratio=c.sample_ratio,
                         compress_upper_bound=c.compress_upper_bound, compress_lower_bound=c.compress_lower_bound,
                         max_adaptation_iters=c.max_adaptation_iters, resample=c.resample,
                         fp16_values=c.fp16_values, int32_indices=c.int32_indices, device=dev,
                         world_size=comm.size(), deferred_masking=True, fill=self.fill, dtype=self.dtype,
                         payload_extra=dense_bytes)
            for i, n in enumerate(comp_names):
                numel, _, k, S, ks, stride = c.attributes[n]
                if (k, S, ks, stride) != tuple(b.attrs[i]):
                    raise RuntimeError(f"batched DGC: attributes of {n} differ from the compressor's")
            plan["batch"] = b
            for n in comp_names:
                p = params[n]
                mv, vv = b._view(b._mmt_flat, n), b._view(b._vec_flat, n)
                mv.copy_(mem.momentums[n])
                vv.copy_(mem.velocities[n])
                mem.momentums[n], mem.velocities[n] = mv, vv
                plan["comp"].append((n, p, b.out(n), b.grad(n)))
                plan["state"].append((n, mv, vv))
            plan["comp_params"] = [e[1] for e in plan["comp"]]
            plan["comp_views"] = [e[2] for e in plan["comp"]]
            plan["index"] = {n: i for i, n in enumerate(b.names)}
            plan["ptrs"] = (ctypes.c_void_p * len(comp_names))()
            plan["sampled"] = {n: c.attributes[n][5] for n in comp_names if c.attributes[n][0] != c.attributes[n][3]}
            plan["order"] = None
        if dense:
            out = torch.zeros(end, dtype=self.dtype, device=dev)
            mmt = torch.zeros(end, dtype=self.dtype, device=dev)
            for (n, p), o in zip(dense, offs):
                mv = mmt[o: o + p.numel()].view(p.shape)
                mv.copy_(mem.momentums[n])
                mem.momentums[n] = mv
                plan["dense"].append((n, p, o, out[o: o + p.numel()].view(p.shape)))
                plan["dense_state"].append((n, mv))
            plan["dense_out"], plan["dense_mmt"], plan["dense_numel"] = out, mmt, end
            plan["dense_params"] = [e[1] for e in plan["dense"]]
            plan["dense_views"] = [e[3] for e in plan["dense"]]
            T = len(dense)
            plan["dense_ptrs"] = (ctypes.c_void_p * T)()
            plan["dense_numels"] = (ctypes.c_int64 * T)(*[p.numel() for _, p in dense])
            plan["dense_offs"] = (ctypes.c_int64 * T)(*offs)
            if dense_bytes:
                plan["wire_dtype"] = wire_dt
                b = plan["batch"]
                if b is None or b.extra_off is None:
                    # no compressed tensor (a ratio-1 warmup epoch) or a split exchange: the
                    # wire values go in an allgather of their own, summed the same way
                    plan["dense_wire"] = torch.empty(dense_bytes, dtype=torch.uint8, device=dev)
                    plan["dense_gathered"] = torch.empty(comm.size() * dense_bytes, dtype=torch.uint8, device=dev)
            if self.half:   # the gathered 16-bit gradients (K1-16's dense branch reads one buffer)
                plan["dense_in"] = torch.zeros(end, dtype=self.dtype, device=dev)
            plan["zeros"] = torch.zeros(max((p.numel() for _, p in dense), default=1), dtype=self.dtype,
                                        device=dev)
        self._plan = plan

    def flush(self):
        """Applies a deferred momentum masking (before anyone reads the memory)."""
        if self._plan and self._plan["batch"] is not None:
            self._plan["batch"].flush()

    def _rebind_state(self):
        """Moves back into the flat layout whatever state was rebound since the last step
        (``load_state_dict`` puts the checkpoint's tensors into the memory's dicts)."""
        plan, mem = self._plan, self.mem
        moms, vels = mem.momentums, mem.velocities
        for n, mv, vv in plan["state"]:
            for store, view in ((moms, mv), (vels, vv)):
                if store[n] is not view:
                    plan["batch"].flush()
                    view.copy_(store[n])
                    store[n] = view
        for n, mv in plan["dense_state"]:
            if moms[n] is not mv:
                mv.copy_(moms[n])
                moms[n] = mv

    # ------------------------------------------------------------------ step
    def step(self, hook_order):
        """compress -> exchange -> decompress for every parameter; ``hook_order`` lists
        the parameters in the order their hooks fired (the reference's compress order)."""
        glue = _glue()
        key = self._plan_key()
        if self._plan is None or self._plan["key"] != key:
            self._build(key)
        self._rebind_state()
        plan = self._plan
        b = plan["batch"]
        dev = plan["dev"]
        if b is not None:
            if plan["order"] != hook_order:
                # the sample-start draw sequence of this hook order (backward's order is
                # the same step after step): the hooked tensors in their order, then the
                # rest in the model's order (synchronize() compresses those after)
                index, sampled, seq, seen = plan["index"], plan["sampled"], [], set()
                for n in list(hook_order) + [e[0] for e in plan["comp"]]:
                    if n in index and n not in seen:
                        seen.add(n)
                        if n in sampled:
                            seq.append((index[n], sampled[n]))
                plan["order"], plan["seq"] = list(hook_order), seq
            starts = [0] * len(plan["comp"])
            draw = _draw()
            for i, stride in plan["seq"]:
                starts[i] = draw(stride)   # dgc/compression.py:118
            ptrs = plan["ptrs"]
            # autograd (and the p.grad setter) keep dtype, device and size those of the
            # parameter: only the layout needs a look (K1 reads 16-B aligned rows)
            for i in glue.grad_table(plan["comp_params"], ctypes.addressof(ptrs), 2 if self.half else 16):
                _, p, _, gflat = plan["comp"][i]
                if p.grad is None:
                    gflat.zero_()   # no gradient this step: zeros
                else:
                    gflat.copy_(p.grad)
                ptrs[i] = gflat.data_ptr()
            b.compensate(starts, grad_ptrs=ptrs)
            b.select()
        dense_handle = None
        if plan["dense"]:
            dptrs = plan["dense_ptrs"]
            for i in glue.grad_table(plan["dense_params"], ctypes.addressof(dptrs), 2 if self.half else 4):
                g = plan["dense"][i][1].grad
                if g is None:
                    g = plan["zeros"]
                else:
                    g = g.contiguous()
                    plan.setdefault("keep", []).append(g)
                dptrs[i] = g.data_ptr()
            L = _lib.lib()
            st = _lib.stream_of(dev)
            if self.half:
                dense_handle = self._dense16_exchange(plan, L, st)
            elif "wire_dtype" in plan:
                # compress: tensor.type(torch.float16) (dgc/compression.py:175-177), into the
                # payload's tail (or the dense allgather's own buffer)
                own = plan.get("dense_wire")
                dst = own.data_ptr() if own is not None else b.payload.data_ptr() + b.extra_off
                _lib.check(L.dgc_gather_cast(dptrs, plan["dense_numels"], plan["dense_offs"], len(plan["dense"]),
                                             ctypes.c_void_p(dst), _lib.VD[plan["wire_dtype"]], st), "dgc_gather_cast")
                if own is not None:
                    dense_handle = comm.allgather_packed_async(own, out=plan["dense_gathered"])
        if b is not None:
            b.send()   # the allgather (or its parts), waited for in b.decompress()
            b.decompress()   # into the batch's output, then p.grad (dgc/compression.py:191-194)
            glue.bind_grads(plan["comp_params"], plan["comp_views"])
        if plan["dense"]:
            mem = self.mem
            L = _lib.lib()
            st = _lib.stream_of(dev)
            out, mmt = plan["dense_out"], plan["dense_mmt"]
            if self.half:
                src = plan["dense_in"]
                if dense_handle is not None:   # decompress: tensor.type(vdtype) (dgc/compression.py:196-197)
                    src = comm.synchronize(dense_handle).to(self.dtype)
                _lib.check(L.dgc_compensate16(_lib.ptr(src), _lib.ptr(mmt), None, _lib.ptr(out), None,
                                              plan["dense_numel"], float(mem.momentum), int(bool(mem.nesterov)), 0,
                                              _lib.VD[self.dtype], st), "dgc_compensate16")
            elif "wire_dtype" in plan:
                # Average = the rank-order sum / W of the gathered wire values, then
                # compensate(accumulate=False) (dgc/compression.py:195-198, 205-206)
                if dense_handle is not None:
                    src, stride = comm.synchronize(dense_handle).data_ptr(), plan["dense_wire"].numel()
                else:
                    src, stride = b.gathered.data_ptr() + b.extra_off, b.rank_stride
                _lib.check(L.dgc_compensate_ranks(ctypes.c_void_p(src), _lib.VD[plan["wire_dtype"]], comm.size(),
                                                  stride, _lib.ptr(mmt), _lib.ptr(out), plan["dense_numel"],
                                                  float(mem.momentum), int(bool(mem.nesterov)), st),
                           "dgc_compensate_ranks")
            else:   # one rank: the allreduce is the identity, the fp16 wire a rounding
                rnd = torch.float16 if self.comp.fp16_values else torch.float32
                _lib.check(L.dgc_compensate_multi(plan["dense_ptrs"], plan["dense_numels"], plan["dense_offs"],
                                                  len(plan["dense"]), _lib.VD[rnd], _lib.ptr(mmt), _lib.ptr(out),
                                                  float(mem.momentum), int(bool(mem.nesterov)), st),
                           "dgc_compensate_multi")
            # p.grad.set_(compensate(accumulate=False)) (dgc/compression.py:195-198)
            glue.bind_grads(plan["dense_params"], plan["dense_views"])
            plan.pop("keep", None)

    def _dense16_exchange(self, plan, L, st):
        """16-bit dense tensors: the gradients gathered into one buffer (2-B copies),
        then compress's wire cast (fp16 for fp16_values, dgc/compression.py:175-177) and
        the allreduce, or at W = 1 the cast's rounding alone (the allreduce is the
        identity). Returns the allreduce handle (None at W = 1). Not on a benched path:
        the casts are ATen's."""
        dense_in = plan["dense_in"]
        _lib.check(L.dgc_gather16(plan["dense_ptrs"], plan["dense_numels"], plan["dense_offs"], len(plan["dense"]),
                                  _lib.ptr(dense_in), st), "dgc_gather16")
        wire = dense_in.to(torch.float16) if self.comp.fp16_values else dense_in
        if comm.size() > 1 or comm.one_rank_collectives():
            return comm.allreduce_async_(wire, op=Average)
        if wire is not dense_in:
            dense_in.copy_(wire)   # the fp16 round trip of a bf16 gradient
        return None

    def release_grads(self, param_groups):
        """zero_grad(set_to_none=True): every gradient of the wrapped optimizer's params
        dropped (torch's zero_grad does the same, per call with a profiler scope)."""
        key = (id(param_groups), len(param_groups), sum(len(g["params"]) for g in param_groups))
        if getattr(self, "_params_key", None) != key:
            self._params_key = key
            self._params = [p for g in param_groups for p in g["params"]]
        _glue().release_grads(self._params)
        return True

    def zero_grads(self):
        """zero_() of every gradient in place (the output views stay bound)."""
        plan = self._plan
        if plan is None:
            return False
        if plan["batch"] is not None:
            plan["batch"].out_flat.zero_()
        if plan["dense"]:
            plan["dense_out"].zero_()
        for _, p, out, _ in plan["comp"]:     # anything rebound since: zeroed in place too
            if p.grad is not None and p.grad is not out:
                p.grad.zero_()
        for _, p, _, view in plan["dense"]:
            if p.grad is not None and p.grad is not view:
                p.grad.zero_()
        return True
