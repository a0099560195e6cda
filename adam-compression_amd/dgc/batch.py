"""Every compressed tensor of a training step through ONE set of launches.

The reference compresses tensor by tensor, from one autograd hook per parameter,
with two Horovod allgathers per tensor (dgc/horovod/optimizer.py:116-155,
dgc/compression.py:155-212). ``DGCBatch`` keeps the per-tensor numerics exactly —
the same attributes (dgc/compression.py:56-89), one ``random.randint(0, stride - 1)``
per tensor and step in the tensors' order (dgc/compression.py:118), the same
compensate / threshold / adaptation / resample / masking per tensor — but lays the
tensors side by side in three flat fp32 buffers (gradients, momentums, velocities;
each tensor at a 1024-element-aligned offset) and runs

    dgc_batch_compress   K1 over all tensors, K3 for all thresholds, the selection
                         chain with per-tensor state, one packed payload
    one allgather        the packed payload, RCCL over xGMI (gloo stages via the host)
    decompress           dgc_decompress_packed (zero fill + scatter) over the flat output
                         (``fill="auto"``/``"inline"``, the default), or — opted in with
                         ``fill="sparse"`` by a caller that owns the output and never writes
                         it — dgc_decompress_packed_over: only the previous step's gathered
                         indices are re-zeroed, as in ``DGCBucket`` (writes through ``.data``
                         or raw pointers do not bump torch's version counter, so the
                         re-zero cannot see them: see dgc/bucket.py)

with O(1) launches per phase and no host synchronisation. The payload carries flat
indices (tensor offset + index in the tensor), tensor after tensor.

``grad(name)`` / ``momentum(name)`` / ``velocity(name)`` / ``out(name)`` are views in
the flat buffers (the parameter-shaped tensors the reference keeps per name).
"""
import ctypes
import math
import random

import torch
import torch.distributed as dist

from . import _lib
from . import comm
from .exchange import SplitExchange, split_parts

__all__ = ["DGCBatch"]

SEG = 1024   # tensors start at multiples of this many elements (the kernels' segment)


def _attributes(numel, ratio, sample_ratio):
    """(num_selects, num_samples, top_k_samples, sample_stride): dgc/compression.py:56-89."""
    from .compression import DGCCompressor
    stride, samples = DGCCompressor._stride_and_samples(numel, ratio, sample_ratio)
    return int(math.ceil(numel * ratio)), samples, int(math.ceil(samples * ratio)), stride


class DGCBatch:
    def __init__(self, named_shapes, compress_ratio=0.001, momentum=0.9, nesterov=False, momentum_masking=True,
                 sample_ratio=0.01, compress_upper_bound=1.3, compress_lower_bound=0.8, max_adaptation_iters=10,
                 resample=True, fp16_values=False, int32_indices=False, device=None, world_size=None, seed=None,
                 deferred_masking=True, fill="auto", dtype=torch.float32, exchange_parts="auto",
                 resample_order="index", payload_extra=0):
        if fill not in ("auto", "inline", "sparse"):
            raise ValueError(f"fill must be 'auto', 'inline' or 'sparse', not {fill!r}")
        if dtype not in (torch.float32,) + _lib.HALF:
            raise NotImplementedError(f"DGCBatch: fp32, bf16 or fp16 parameters (got {dtype})")
        self.dtype = dtype
        self.half = dtype in _lib.HALF
        if fill == "auto" or self.half:   # the dense zero_() is always right; the re-zero is opt-in (fp32)
            fill = "inline"
        self.fill = fill
        self.exchange_parts = exchange_parts
        if resample_order not in ("index", "topk"):
            raise ValueError(f"resample_order must be 'index' or 'topk', not {resample_order!r}")
        # "index": a resampled tensor whose k-th largest candidate is untied lists its
        # top-k set in index order (the decompress and the memory update depend on the
        # set only; dgc_select_params.resample_order); "topk": torch.topk's order always
        self.resample_order = resample_order
        # bytes appended to every rank's payload (after the packed entries): the batched
        # optimizer's dense wire values ride in the same allgather (``extra_off``; None
        # when the exchange is split, which carries the sparse entries only)
        self.payload_extra = int(payload_extra)
        self.device = torch.device(device or "cuda")
        self.names = [n for n, _ in named_shapes]
        self.shapes = {n: tuple(s) for n, s in named_shapes}
        self.numels = [math.prod(self.shapes[n]) for n in self.names]
        self.momentum, self.nesterov, self.momentum_masking = float(momentum), bool(nesterov), bool(momentum_masking)
        self.sample_ratio = min(max(sample_ratio, 0.01), 1.0)
        self.upper, self.lower = float(compress_upper_bound), float(compress_lower_bound)
        self.max_iters, self.resample = int(max_adaptation_iters), bool(resample)
        self.vdtype = torch.float16 if fp16_values else dtype
        self.idtype = torch.int32 if int32_indices else torch.int64
        self.world = world_size or (dist.get_world_size() if dist.is_initialized() else 1)
        self.rng = random.Random(seed) if seed is not None else random   # the reference draws from `random`
        offs, end = [], 0
        for n in self.numels:
            offs.append(end)
            end += -(-n // SEG) * SEG
        self.offsets = offs
        self.flat_numel = max(end, SEG)
        dev = self.device
        self.grad_flat = torch.zeros(self.flat_numel, dtype=dtype, device=dev)
        self._mmt_flat = torch.zeros(self.flat_numel, dtype=dtype, device=dev)
        self._vec_flat = torch.zeros(self.flat_numel, dtype=dtype, device=dev)
        # 16-bit: K1-16 (dgc_compensate16) rounds every op to the dtype and writes the new
        # velocity's exact fp32 image, which the selection reads (dgc_batch_select); the
        # 16-bit state is masked from the payload (dgc_mask_packed16)
        self._vec32 = torch.zeros(self.flat_numel, dtype=torch.float32, device=dev) if self.half else None
        self.deferred_masking = bool(deferred_masking) and not self.half
        self._pending = False
        self.out_flat = torch.zeros(self.flat_numel, dtype=dtype, device=dev)
        self._L = _lib.lib()
        self.info = torch.zeros(len(self.names) * _lib.INFO_BYTES, dtype=torch.uint8, device=dev)
        # DGC_K5_BROKEN and the decompress's bad index / gathered count (a peer's payload
        # corrupted in transit), written by the kernels into pinned words, checked every step
        self.status = _lib.StatusSink("DGCBatch", dev)
        self.set_ratio(compress_ratio)

    # ---------------------------------------------------------------- layout
    def set_ratio(self, compress_ratio):
        """(Re-)derive every tensor's attributes for a compress ratio and write the
        device tables — ``DGCCompressor.initialize`` (dgc/compression.py:56-89), also
        what ``warmup_compress_ratio`` re-runs on a ratio change (:91-107)."""
        ratio = compress_ratio if compress_ratio <= 1.0 else 1.0 / compress_ratio
        self.flush()   # a pending masking lives in the old workspace
        self.ratio = ratio
        T = len(self.names)
        self.attrs = [_attributes(n, ratio, self.sample_ratio) for n in self.numels]
        arr = lambda xs: (ctypes.c_int64 * T)(*xs)   # noqa: E731
        self._arrays = [arr(self.numels), arr(self.offsets), arr([a[0] for a in self.attrs]),
                        arr([a[1] for a in self.attrs]), arr([a[2] for a in self.attrs]), arr([a[3] for a in self.attrs])]
        d = _lib.BatchDesc()
        d.count = T
        d.numel, d.offset, d.num_selects, d.num_samples, d.top_k_samples, d.sample_stride = self._arrays
        d.flat_numel = self.flat_numel
        d.upper_bound, d.lower_bound = self.upper, self.lower
        d.max_iters, d.resample, d.momentum_masking = self.max_iters, int(self.resample), int(self.momentum_masking)
        d.fp16_values, d.int32_indices = int(self.vdtype == torch.float16), int(self.idtype == torch.int32)
        d.nesterov, d.momentum, d.spec_margin = int(self.nesterov), self.momentum, _lib.SPEC_MARGIN
        d.deferred_masking = int(self.deferred_masking)
        d.dtype = _lib.VD[self.dtype]
        d.status_sink = self.status.address
        d.resample_order = 1 if self.resample_order == "index" else 0
        self.desc = d
        L = self._L
        wsz = L.dgc_batch_workspace(ctypes.byref(d))
        if wsz == 0:
            raise RuntimeError(f"dgc_batch_workspace: {L.dgc_last_error().decode()}")
        self.ws = torch.empty(wsz, dtype=torch.uint8, device=self.device)
        _lib.check(L.dgc_batch_init(ctypes.byref(d), self.ws.data_ptr(), wsz, _lib.stream_of(self.device)),
                   "dgc_batch_init")
        self.capacity = sum(a[0] for a in self.attrs)
        from .compression import _layout
        self.rank_stride, self.voff, self.ioff = _layout(self.capacity, self.vdtype, self.idtype)
        # W > 1, fp32: the allgather in parts, each scattered as it lands (dgc/exchange.py)
        # (W = 1 exchanges too when comm.one_rank_collectives(): the RCCL tests' one-rank group)
        self.exchanging = self.world > 1 or comm.one_rank_collectives()
        self.parts = 1 if self.half else split_parts(self.world, self.capacity, self.exchange_parts)
        self.extra_off = None
        if self.payload_extra > 0 and self.parts == 1:
            self.extra_off = self.rank_stride
            self.rank_stride = -(-(self.rank_stride + self.payload_extra) // 256) * 256
        # fill="sparse": two payload / gather buffers, so the previous step's gathered
        # indices stay readable for the re-zero; a new layout forgets them
        nbuf = 2 if self.fill == "sparse" else 1
        self._payloads = [torch.zeros(self.rank_stride, dtype=torch.uint8, device=self.device) for _ in range(nbuf)]
        self.xchg = None
        self._inflight = None
        if self.parts > 1:
            self.xchg = SplitExchange(self.capacity, self.flat_numel, self.world, self.parts, self.vdtype,
                                      self.idtype, self.device, nbuf)
            self._gathers = self.xchg.gathers
        else:
            self._gathers = ([torch.zeros(self.world * self.rank_stride, dtype=torch.uint8, device=self.device)
                              for _ in range(nbuf)] if self.exchanging else self._payloads)
        self._par = 0
        self._last_out = None
        self._last_gathered = None
        self.dec_ws = (torch.empty(L.dgc_decompress_packed_workspace(self.flat_numel, self.world, self.capacity),
                                   dtype=torch.uint8, device=self.device) if self.xchg is None else None)
        self.status.bind(self.dec_ws if self.xchg is None else self.xchg.ws)

    @property
    def payload(self):
        """This rank's packed payload of the current step."""
        return self._payloads[self._par % len(self._payloads)]

    @property
    def gathered(self):
        """The allgather buffer of the current step (the payload itself at W = 1)."""
        return self._gathers[self._par % len(self._gathers)]

    def flush(self):
        """Applies a deferred masking now (no-op when none is pending)."""
        if self._pending:
            _lib.check(self._L.dgc_batch_flush(ctypes.byref(self.desc), self._mmt_flat.data_ptr(),
                                               self._vec_flat.data_ptr(), self.ws.data_ptr(), self.ws.numel(),
                                               _lib.stream_of(self.device)), "dgc_batch_flush")
            self._pending = False

    @property
    def mmt_flat(self):
        """Flat momentum buffer, masking applied."""
        self.flush()
        return self._mmt_flat

    @property
    def vec_flat(self):
        """Flat velocity buffer, masking applied."""
        self.flush()
        return self._vec_flat

    def _view(self, flat, name):
        i = self.names.index(name)
        return flat[self.offsets[i]: self.offsets[i] + self.numels[i]].view(self.shapes[name])

    def grad(self, name):
        return self._view(self.grad_flat, name)

    def momentum_of(self, name):
        return self._view(self.mmt_flat, name)

    def velocity_of(self, name):
        return self._view(self.vec_flat, name)

    def out(self, name):
        return self._view(self.out_flat, name)

    # ---------------------------------------------------------------- phases
    def draw_starts(self):
        """random.randint(0, stride - 1) per sampled tensor, in the tensors' order (dgc/compression.py:118)."""
        starts = []
        for n, (k, S, ks, stride) in zip(self.numels, self.attrs):
            starts.append(self.rng.randint(0, stride - 1) if n != S else 0)
        return starts

    def _arrays16(self):
        if not hasattr(self, "_g16"):
            T = len(self.names)
            self._g16 = ((ctypes.c_int64 * T)(*self.numels), (ctypes.c_int64 * T)(*self.offsets))
        return self._g16

    def compensate(self, starts=None, grad_ptrs=None):
        """K1 over every tensor: compensate + strided samples + candidate lists (and any
        masking the previous select left pending). The gradients come from ``grad_flat``,
        or — ``grad_ptrs``, a ctypes array of T device pointers, each to the tensor's
        numel contiguous fp32 elements, 16-B aligned — from wherever they are (the
        batched optimizer's p.grad tensors, read in place). Raises first if a previous
        step's resample replay reported DGC_K5_BROKEN, or its decompress met an index
        or a gathered count out of range (``status``)."""
        self.status.check()
        starts = self.draw_starts() if starts is None else starts
        self.starts = starts
        self._par += 1   # a step starts: the other payload / gather buffer
        arr = (ctypes.c_int64 * len(starts))(*starts)
        self._starts_arr = arr
        L, st = self._L, _lib.stream_of(self.device)
        if self.half:
            if grad_ptrs is not None:   # the 16-bit gradients into the flat buffer (2-B gather)
                numels, offs = self._arrays16()
                _lib.check(L.dgc_gather16(grad_ptrs, numels, offs, len(self.names), self.grad_flat.data_ptr(), st),
                           "dgc_gather16")
            _lib.check(L.dgc_compensate16(self.grad_flat.data_ptr(), self._mmt_flat.data_ptr(),
                                          self._vec_flat.data_ptr(), None, self._vec32.data_ptr(), self.flat_numel,
                                          self.momentum, int(self.nesterov), 1, _lib.VD[self.dtype], st),
                       "dgc_compensate16")
            return
        if grad_ptrs is None:
            _lib.check(L.dgc_batch_compress_begin(ctypes.byref(self.desc), self.grad_flat.data_ptr(),
                                                  self._mmt_flat.data_ptr(), self._vec_flat.data_ptr(), arr,
                                                  self.ws.data_ptr(), self.ws.numel(), st), "dgc_batch_compress_begin")
        else:
            _lib.check(L.dgc_batch_compress_begin_ptrs(ctypes.byref(self.desc), grad_ptrs, self._mmt_flat.data_ptr(),
                                                       self._vec_flat.data_ptr(), arr, self.ws.data_ptr(),
                                                       self.ws.numel(), st), "dgc_batch_compress_begin_ptrs")
        self._pending = False

    def select(self):
        """K3 thresholds + selection / adaptation / resample / pack / masking of every tensor."""
        if self.half:
            L, st = self._L, _lib.stream_of(self.device)
            _lib.check(L.dgc_batch_select(ctypes.byref(self.desc), self._vec32.data_ptr(), None, self._starts_arr,
                                          self.payload.data_ptr(), self.info.data_ptr(), self.ws.data_ptr(),
                                          self.ws.numel(), _lib.SYNC_DEVICE, st), "dgc_batch_select")
            _lib.check(L.dgc_mask_packed16(self.payload.data_ptr(), self.capacity, _lib.VD[self.vdtype],
                                           _lib.ID[self.idtype],
                                           self._mmt_flat.data_ptr() if self.momentum_masking else None,
                                           self._vec_flat.data_ptr(), self.flat_numel, st), "dgc_mask_packed16")
            return
        _lib.check(self._L.dgc_batch_compress_finish(ctypes.byref(self.desc), self._mmt_flat.data_ptr(),
                                                     self._vec_flat.data_ptr(), self.payload.data_ptr(),
                                                     self.info.data_ptr(), self.ws.data_ptr(), self.ws.numel(),
                                                     _lib.SYNC_DEVICE, _lib.stream_of(self.device)),
                   "dgc_batch_compress_finish")
        self._pending = self.deferred_masking

    def compress(self, starts=None):
        """Every tensor: compensate -> sample -> threshold -> select -> pack -> masking."""
        self.compensate(starts)
        self.select()

    def send(self):
        """Issues the exchange of this step's payload (W > 1): one allgather, or one per
        part (split); ``decompress`` waits for it. Nothing is issued in between, so a
        single allgather goes out on the current stream (``comm.COLLECTIVE_ISSUE``)."""
        if self.exchanging:
            if self.xchg is not None:
                self._inflight = self.xchg.send(self.payload, self.gathered)
            else:
                self._inflight = [comm.allgather_packed_async(self.payload, out=self.gathered, wait=True)]

    def exchange(self):
        """The exchange; a single allgather is also waited for here, a split one part by
        part in ``decompress``."""
        self.send()
        if self.xchg is None and self._inflight:
            self._inflight.pop().wait()
            self._inflight = None

    def decompress(self, out_flat=None):
        """out = the rank-order sum of the gathered entries / W, +0.0 elsewhere (every tensor).

        fill="sparse": when ``out`` still holds exactly the previous decompress's result
        (same storage, torch version counter unchanged — our writes are raw-pointer
        writes) and is not the gradient buffer (the batched optimizer decompresses into
        p.grad, rewritten by every backward), the zero_() re-zeroes only the previous
        step's gathered indices (dgc_decompress_packed_over) instead of the whole
        buffer: identical result, W * capacity slots instead of flat_numel."""
        out = self.out_flat if out_flat is None else out_flat
        if _lib.require_cuda_float(out, "DGCBatch.decompress") != self.dtype or out.numel() != self.flat_numel \
                or out.device != self.device:
            raise ValueError(f"DGCBatch.decompress: out_flat must be a contiguous {self.dtype} tensor of "
                             f"{self.flat_numel} elements on {self.device} (got {out.dtype} [{out.numel()}] on "
                             f"{out.device})")
        L = self._L
        st = _lib.stream_of(self.device)
        cur = self.gathered
        handles, self._inflight = self._inflight or [], None
        if self.xchg is None:
            for h in handles:
                h.wait()
        elif self.exchanging and not handles:
            raise RuntimeError("DGCBatch: decompress of a split exchange before send() / exchange()")
        if self.half:   # zero_(), the runs in rank order (each add rounded), the 1/W scale
            _lib.check(L.dgc_decompress_packed16(cur.data_ptr(), self.world, self.rank_stride, self.capacity,
                                                 _lib.VD[self.vdtype], _lib.ID[self.idtype], out.data_ptr(),
                                                 _lib.VD[self.dtype], self.flat_numel, 1.0 / self.world,
                                                 ctypes.c_void_p(self.status.decompress_words), st),
                       "dgc_decompress_packed16")
            return out
        aliased = out.untyped_storage().data_ptr() == self.grad_flat.untyped_storage().data_ptr()
        reusable = (self.fill == "sparse" and not aliased and self._last_gathered is not None
                    and self._last_gathered is not cur
                    and self._last_out == (out.data_ptr(), out.numel(), out._version))
        if self.xchg is not None:   # zero_() first (it runs under the first part's collective)
            if reusable:
                self.xchg.clear(self._last_gathered, out, st)
            else:
                _lib.check(L.dgc_fill_zero(out.data_ptr(), self.flat_numel, st), "dgc_fill_zero")
            self.xchg.scatter(cur, handles, out, 1.0 / self.world, reusable)
        else:
            args = (self.world, self.rank_stride, self.capacity, _lib.VD[self.vdtype], _lib.ID[self.idtype],
                    out.data_ptr(), self.flat_numel, 1.0 / self.world, self.dec_ws.data_ptr(), self.dec_ws.numel(), st)
            if reusable:
                _lib.check(L.dgc_decompress_packed_over(cur.data_ptr(), self._last_gathered.data_ptr(), *args),
                           "dgc_decompress_packed_over")
            else:
                # the zero fill and the scatter in one call: the fill also resets the scatter's status words
                _lib.check(L.dgc_decompress_packed(cur.data_ptr(), *args), "dgc_decompress_packed")
        if aliased:
            self._last_out = self._last_gathered = None
        else:
            self._last_out = (out.data_ptr(), out.numel(), out._version)
            self._last_gathered = cur
        return out

    def step(self, starts=None):
        self.compress(starts)
        self.exchange()
        return self.decompress()

    # ---------------------------------------------------------------- results
    def infos(self):
        self.status.check(sync=True)
        raw = self.info.cpu().numpy().tobytes()
        out = []
        for t in range(len(self.names)):
            i = _lib.SelectInfo.from_buffer_copy(raw[t * _lib.INFO_BYTES:(t + 1) * _lib.INFO_BYTES])
            out.append(_lib.info_dict(i, f"DGCBatch tensor {self.names[t]}"))
        return out

    def transmitted(self, rank_payload=None):
        """{name: (values, indices)} of one rank's payload (this rank's by default), with
        indices relative to the tensor — what the reference's compress returns."""
        p = self.payload if rank_payload is None else rank_payload
        total = int(p[:8].view(torch.int64).item())
        vb = torch.empty(0, dtype=self.vdtype).element_size()
        ib = torch.empty(0, dtype=self.idtype).element_size()
        vals = p[self.voff: self.voff + total * vb].view(self.vdtype)
        idxs = p[self.ioff: self.ioff + total * ib].view(self.idtype)
        counts = [i["count"] for i in self.infos()]
        res, pos = {}, 0
        for name, off, c in zip(self.names, self.offsets, counts):
            res[name] = (vals[pos: pos + c], idxs[pos: pos + c].to(torch.int64) - off)
            pos += c
        return res
