"""Deep Gradient Compression compressor — drop-in for the reference ``dgc/compression.py``.

``DGCCompressor`` keeps the reference's constructor, ``attributes`` tuples,
``initialize``, ``warmup_compress_ratio``, ``compress``, ``decompress``,
``communicate`` and ``synchronize`` (dgc/compression.py:17-212), including the
Python-global ``random.randint`` draw of the sample start at the same call point
(dgc/compression.py:118). All tensor work runs in ``libdgc_hip.so`` on the MI355X:

  compress    ``dgc_compress``: K1 compensate with the strided sample fused in,
              K3 radix-select threshold, K4 select / adaptation loop / resample /
              pack / momentum masking. One host synchronisation per call, to
              return exact-length ``[n, 1]`` tensors as the reference does.
  communicate one RCCL ``all_gather_into_tensor`` of the packed per-rank payload
              ``[count | values | indices]`` (fixed capacity = num_selects).
  decompress  ``dgc_decompress(_packed)``: deterministic rank-order scatter-add.

Wire casts follow the reference (fp16 values, int32 indices). int32 indices are
refused for tensors above 2^31 - 1 elements, where the reference's cast wraps.
"""
import math
import random

import torch

from . import _lib
from . import comm
from .comm import Average
from .memory import DGCSGDMemory, Memory

__all__ = ["DGCCompressor"]


class _Gathered(list):
    """``synchronize`` output: ``[values[sum n_r, 1], indices[sum n_r, 1]]`` like the
    reference's list of two allgathers, carrying the packed buffer for decompress."""
    packed = None
    world = 1
    rank_stride = 0
    capacity = 0
    run_offsets = None
    distinct_runs = False   # every run's indices distinct (payloads this compressor emitted)


class _PackedHandle:
    def __init__(self, handle, name, capacity, vdtype, idtype, stride, voff, ioff):
        self.handle = handle
        self.name = name
        self.capacity = capacity
        self.vdtype = vdtype
        self.idtype = idtype
        self.stride = stride
        self.voff = voff
        self.ioff = ioff


_OURS = 0x444743454D495454   # payload header word 1 of a compress-emitted payload ("DGCEMITT")


def _layout(capacity, vdtype, idtype):
    import ctypes
    voff, ioff = ctypes.c_int64(), ctypes.c_int64()
    stride = _lib.lib().dgc_payload_layout(capacity, _lib.VD[vdtype], _lib.ID[idtype],
                                           ctypes.byref(voff), ctypes.byref(ioff))
    return stride, voff.value, ioff.value


class DGCCompressor:
    def __init__(self, compress_ratio, memory=None,
                 sample_ratio=0.01, strided_sample=True,
                 compress_upper_bound=1.3, compress_lower_bound=0.8, max_adaptation_iters=10, resample=True,
                 fp16_values=False, int32_indices=False,
                 warmup_epochs=-1, warmup_coeff=None):
        # dgc/compression.py:18-54
        self.world_size = comm.size()
        self.op = Average
        self.fp16_values = fp16_values
        self.int32_indices = int32_indices
        ratio = compress_ratio if compress_ratio <= 1.0 else 1.0 / compress_ratio
        self.base_compress_ratio = self.compress_ratio = ratio
        self.memory = Memory if memory is None else memory
        self.warmup_epochs = warmup_epochs
        if warmup_epochs > 0:
            if warmup_coeff is None:
                self.warmup_coeff = self.base_compress_ratio ** (1.0 / (warmup_epochs + 1))
            elif isinstance(warmup_coeff, (tuple, list)):
                assert len(warmup_coeff) >= warmup_epochs
                for wc in warmup_coeff:
                    assert 0 < wc <= 1
                self.warmup_coeff = warmup_coeff
            else:
                assert 0 < warmup_coeff <= 1
                self.warmup_coeff = warmup_coeff
        else:
            self.warmup_coeff = 1
        self.sample_ratio = min(max(sample_ratio, 0.01), 1.0)
        self.strided_sample = strided_sample
        self.compress_upper_bound = compress_upper_bound
        self.compress_lower_bound = compress_lower_bound
        self.max_adaptation_iters = max_adaptation_iters
        self.resample = resample
        self.attributes = {}
        self._ws = _lib.Workspace()
        self._params = {}
        self._payloads = {}
        self._status = {}      # device -> StatusSink: bad indices / gathered counts in the decompress
        self._bound_ws = {}    # device -> the decompress workspace bound to that sink
        self._spec = {}        # name -> device float: speculative list threshold (dgc_compress)
        self.layout_epoch = 0  # bumped by initialize(): the batched step re-derives its layout

    # ------------------------------------------------------------------ host math
    @staticmethod
    def _stride_and_samples(numel, ratio, sample_ratio):
        """(sample_stride, num_samples) of dgc/compression.py:66-83."""
        if sample_ratio >= 1.0:
            return 1, numel
        pct = int(math.ceil(numel * sample_ratio))
        cpr = int(math.ceil(2 / ratio))
        if numel <= cpr:
            return 1, numel
        need = max(pct, cpr)
        stride = int(math.ceil(numel / need / 32)) * 32 + 1
        while numel // stride < need:
            stride -= 8
        return stride, numel // stride

    def initialize(self, named_parameters):
        """Per-tensor (numel, shape, num_selects, num_samples, top_k_samples, sample_stride)
        (dgc/compression.py:56-89)."""
        if comm.rank() == 0:
            print("=> initializing dgc compressor")
        self.layout_epoch += 1
        for name, param in named_parameters:
            if torch.is_tensor(param):
                numel, shape = param.numel(), list(param.size())
            else:
                assert isinstance(param, (list, tuple))
                numel, shape = param[0], param[1]
            stride, samples = self._stride_and_samples(numel, self.compress_ratio, self.sample_ratio)
            if comm.rank() == 0 and self.sample_ratio < 1.0 and samples == numel and stride == 1 \
                    and numel <= int(math.ceil(2 / self.compress_ratio)):
                print(f"Warning: {name} with {numel} elements transmits 1 gradient element")
            top_k_samples = int(math.ceil(samples * self.compress_ratio))
            num_selects = int(math.ceil(numel * self.compress_ratio))
            self.attributes[name] = (numel, shape, num_selects, samples, top_k_samples, stride)
            self._params = {key: v for key, v in self._params.items() if key[0] != name}
            self._spec.pop(name, None)
            if comm.rank() == 0:
                how = f"at stride {stride}" if self.strided_sample else "uniformly"
                print(f"   {name:<25}: transmit {num_selects} / {numel} elements of shape {shape}\n"
                      f"   {' ' * 25}  threshold {top_k_samples} / {samples} samples {how}")

    def warmup_compress_ratio(self, epoch):
        """dgc/compression.py:91-107."""
        if self.warmup_epochs > 0 and epoch < self.warmup_epochs:
            if isinstance(self.warmup_coeff, (tuple, list)):
                ratio = self.warmup_coeff[epoch]
            else:
                ratio = max(self.warmup_coeff ** (epoch + 1), self.base_compress_ratio)
        else:
            ratio = self.base_compress_ratio
        if ratio != self.compress_ratio:
            if comm.rank() == 0:
                print(f"update compress ratio: {ratio}")
            self.compress_ratio = ratio
            self.initialize(self.attributes.items())

    # ------------------------------------------------------------------ errors
    def _sink(self, device):
        """This compressor's StatusSink on ``device``: the decompress kernels store an
        out-of-range index or a gathered count outside [0, capacity] there (the
        reference's index_put_ raises, dgc/compression.py:191)."""
        sink = self._status.get(device)
        if sink is None:
            sink = self._status[device] = _lib.StatusSink("DGCCompressor", device)
        return sink

    def _dec_ws(self, device, nbytes):
        ws = self._ws.get(device, nbytes, "decompress")
        if self._bound_ws.get(device) is not ws:
            self._sink(device).bind(ws)
            self._bound_ws[device] = ws
        return ws

    def check(self, sync=False):
        """Raises if a decompress issued earlier met a bad index or gathered count (read
        from pinned host words: free; ``sync=True`` waits for the stream first). Runs at
        every compress / decompress / synchronize, so an error surfaces one call later
        than the reference's, which raises inside its index_put_."""
        for sink in self._status.values():
            sink.check(sync)

    # ------------------------------------------------------------------ kernels
    def _select_params(self, name, masking, update_memory, dtype=torch.float32):
        key = (name, bool(masking), bool(update_memory), dtype)
        p = self._params.get(key)
        if p is None:
            numel, _, k, S, _, _ = self.attributes[name]
            p = _lib.SelectParams()
            p.numel, p.num_selects, p.num_samples = numel, k, S
            # n > k * upper  and  n < lower * k compare an int with a Python double
            p.upper_count = math.floor(k * self.compress_upper_bound)
            p.lower_count = math.ceil(self.compress_lower_bound * k)
            p.upper, p.lower = float(self.compress_upper_bound), float(self.compress_lower_bound)
            p.max_iters = int(self.max_adaptation_iters)
            p.resample = int(bool(self.resample))
            p.masking = int(bool(masking))
            p.vdtype = _lib.VD[torch.float16 if self.fp16_values else dtype]
            p.thr_dtype = _lib.VD[dtype]   # threshold *= bound rounds to the tensor's dtype
            p.idtype = _lib.ID[torch.int32 if self.int32_indices else torch.int64]
            p.update_memory = int(bool(update_memory))
            self._params[key] = p
        return p

    def _new_payload(self, name, device, dtype=torch.float32):
        k = self.attributes[name][2]
        vdt = torch.float16 if self.fp16_values else dtype
        idt = torch.int32 if self.int32_indices else torch.int64
        stride, voff, ioff = _layout(k, vdt, idt)
        payload = torch.empty(stride, dtype=torch.uint8, device=device)
        return payload, (k, vdt, idt, stride, voff, ioff)

    def _views(self, payload, lay, n):
        k, vdt, idt, stride, voff, ioff = lay
        vb, ib = torch.empty(0, dtype=vdt).element_size(), torch.empty(0, dtype=idt).element_size()
        values = payload[voff: voff + n * vb].view(vdt).view(-1, 1)
        indices = payload[ioff: ioff + n * ib].view(idt).view(-1, 1)
        return values, indices

    def _sample_start(self, name):
        numel, _, _, S, _, stride = self.attributes[name]
        if numel == S or not self.strided_sample:
            return 0
        return random.randint(0, stride - 1)         # dgc/compression.py:118

    def _sparsify(self, tensor, name, payload=None, lay=None, update_memory=False):
        """dgc/compression.py:109-153 on an already-compensated tensor. Returns
        (values, indices, numel, shape, num_selects) with exact-length 1-D outputs.
        A bf16 / fp16 tensor is selected on its exact fp32 image (dgc_widen16)."""
        vec = tensor.reshape(-1)
        dt = _lib.require_cuda_float(vec, "DGCCompressor._sparsify")
        if dt in _lib.HALF:
            if update_memory:
                raise ValueError("DGCCompressor._sparsify: a 16-bit state is masked by DGCSGDMemory.update")
            img = self._ws.get(vec.device, 4 * vec.numel(), "img16")[: 4 * vec.numel()].view(torch.float32)
            _lib.check(_lib.lib().dgc_widen16(_lib.ptr(vec), _lib.ptr(img), vec.numel(), _lib.VD[dt],
                                              _lib.stream_of(vec.device)), "dgc_widen16")
            vec = img
        return self._select_on(vec, name, dt, payload, lay, update_memory)

    def _select_on(self, vec, name, dt, payload, lay, update_memory):
        """Sample, threshold and select over the fp32 tensor (or 16-bit image) vec of
        a tensor of dtype dt (dgc/compression.py:113-153)."""
        numel, shape, k, S, ks, stride = self.attributes[name]
        L = _lib.lib()
        dev = vec.device
        stream = _lib.stream_of(dev)
        if numel == S:
            samples, m = vec, numel
        elif self.strided_sample:
            start = self._sample_start(name)
            m = (numel - start + stride - 1) // stride
            samples = torch.empty(m, dtype=torch.float32, device=dev)
            _lib.check(L.dgc_sample_strided(_lib.ptr(vec), numel, start, stride, _lib.ptr(samples), m, stream),
                       "dgc_sample_strided")
        else:                                           # dgc/compression.py:120-121
            idx = torch.randint(0, numel, (S,), device=dev)
            m = S
            samples = torch.empty(m, dtype=torch.float32, device=dev)
            _lib.check(L.dgc_sample_gather(_lib.ptr(vec), _lib.ptr(idx), m, _lib.ptr(samples), stream),
                       "dgc_sample_gather")
        thr = torch.empty(64, dtype=torch.float32, device=dev)
        kws = L.dgc_kth_largest_workspace(m)
        kbuf = self._ws.get(dev, kws, "kth")
        _lib.check(L.dgc_kth_largest(_lib.ptr(samples), m, ks, _lib.ptr(thr), _lib.ptr(kbuf), kws, stream),
                   "dgc_kth_largest")
        if payload is None:
            payload, lay = self._new_payload(name, dev, dt)
        k_, vdt, idt, pstride, voff, ioff = lay
        masking = isinstance(self.memory, DGCSGDMemory) and self.memory.momentum_masking
        params = self._select_params(name, masking, update_memory, dt)
        # pure selection emits fp32 / int64; the wire casts happen in compress
        sws = L.dgc_select_workspace(numel, k)
        sbuf = self._ws.get(dev, sws, "select")
        info = torch.empty(_lib.INFO_BYTES, dtype=torch.uint8, device=dev)
        mmt = self.memory.momentums[name] if update_memory and masking else None
        base = payload.data_ptr()
        _lib.check(L.dgc_select(_lib.ptr(vec), _lib.ptr(mmt), _lib.ptr(thr), params,
                                base + voff, base + ioff, base, _lib.ptr(info), _lib.ptr(sbuf), sws,
                                _lib.SYNC_HOST, stream), "dgc_select")
        n = self._count(info)
        values, indices = self._views(payload, lay, n)
        self._last_info = info
        return values.view(-1), indices.view(-1), numel, shape, k

    def compress(self, tensor, name):
        """dgc/compression.py:155-177."""
        self.check()
        if self.compress_ratio < 1.0 and name in self.attributes:
            numel, shape, k, S, ks, stride = self.attributes[name]
            mem = self.memory
            dev = tensor.device
            dt = _lib.require_cuda_float(tensor, "DGCCompressor.compress", contiguous=False)
            payload, lay = self._new_payload(name, dev, dt)
            if isinstance(mem, DGCSGDMemory) and dt in _lib.HALF:
                # 16-bit state: K1-16 writes the velocity's fp32 image, the selection runs
                # on it (pure), then DGCSGDMemory.update masks the 16-bit state
                grad = mem._clip(tensor).reshape(-1).contiguous()
                mem._sync()
                mem.state_of(name, grad, True, "DGCCompressor.compress")
                img = self._ws.get(dev, 4 * numel, "img16")[: 4 * numel].view(torch.float32)
                mem._compensate16(grad, name, True, vec32=img)
                _, idx, _, _, _ = self._select_on(img, name, dt, payload, lay, False)
                mem.update(name, (idx,))
                values, indices = self._views(payload, lay, idx.numel())
            elif isinstance(mem, DGCSGDMemory) and self.strided_sample:
                # fused path: K1 (+sample) -> K3 -> K4 (+update) in one library call
                grad = mem._clip(tensor).reshape(-1)
                _lib.require_cuda_f32(grad, "DGCCompressor.compress")
                mem._sync()
                mmt, vec = mem.state_of(name, grad, True, "DGCCompressor.compress")
                start = self._sample_start(name)
                params = self._select_params(name, mem.momentum_masking, True)
                L = _lib.lib()
                wsz = L.dgc_compress_workspace(numel, k, S)
                ws = self._ws.get(dev, wsz, name)
                spec = self._spec.get(name)
                if spec is None or spec.device != dev:
                    spec = self._spec[name] = torch.full((8,), float("inf"), dtype=torch.float32, device=dev)
                info = torch.empty(_lib.INFO_BYTES, dtype=torch.uint8, device=dev)
                base = payload.data_ptr()
                voff, ioff = lay[4], lay[5]
                _lib.check(L.dgc_compress(_lib.ptr(grad), _lib.ptr(mmt), _lib.ptr(vec), float(mem.momentum),
                                          int(bool(mem.nesterov)), start, stride, ks, params, _lib.ptr(spec),
                                          _lib.SPEC_MARGIN, base + voff, base + ioff, base, _lib.ptr(info),
                                          _lib.ptr(ws), wsz, _lib.SYNC_HOST, _lib.stream_of(dev)), "dgc_compress")
                n = self._count(info)
                values, indices = self._views(payload, lay, n)
                self._last_info = info
            else:
                # generic path: any Memory, or uniform (non-strided) sampling
                compensated = mem.compensate(tensor, name, accumulate=True)
                _, idx, _, _, _ = self._sparsify(compensated, name, payload, lay, update_memory=False)
                mem.update(name, (idx.to(torch.int64) if idx.dtype != torch.int64 else idx,))
                values, indices = self._views(payload, lay, idx.numel())
            # header word 1: "emitted by compress" (distinct indices), read by every rank's
            # synchronize with the counts, so a peer's foreign payload is never taken for one
            payload[8:16].view(torch.int64).fill_(_OURS)
            self._payloads[name] = (payload, lay)
            ctx = (name, numel, shape, dt, torch.int64, tensor.data.view(numel))
            return (values, indices), ctx
        ctx = (name, None, None, tensor.dtype, None, None)
        if self.fp16_values and tensor.dtype.is_floating_point:
            tensor = tensor.type(torch.float16)
        return tensor, ctx

    @staticmethod
    def _count(info):
        """The emitted count, read with the whole selection record in ONE device-to-host
        copy (the one host sync the exact-length [n, 1] outputs need); raises if the
        resample replay reported a broken multi-workgroup phase."""
        return _lib.info_dict(_lib.SelectInfo.from_buffer_copy(info.cpu().numpy().tobytes()),
                              "DGCCompressor.compress")["count"]

    def last_info(self):
        """Selection record of the last compress (branch, counts, thresholds) — diagnostics."""
        return _lib.info_dict(_lib.SelectInfo.from_buffer_copy(self._last_info.cpu().numpy().tobytes()),
                              "DGCCompressor")

    def decompress(self, tensor, ctx):
        """dgc/compression.py:179-198. An index outside the gradient (or a gathered
        count outside the payload's capacity) is reported through this compressor's
        StatusSink and raised at the next call (``check``)."""
        self.check()
        name, numel, shape, vdtype, idtype, grad = ctx
        if self.compress_ratio < 1.0 and name in self.attributes:
            assert isinstance(tensor, (list, tuple))
            gdt = _lib.require_cuda_float(grad, "DGCCompressor.decompress")
            L = _lib.lib()
            dev = grad.device
            scale = 1.0 / self.world_size if self.op == Average else 1.0
            stream = _lib.stream_of(dev)
            if gdt in _lib.HALF:
                return self._decompress16(tensor, grad, numel, shape, scale)
            if isinstance(tensor, _Gathered) and tensor.packed is not None:
                p = tensor
                wsz = L.dgc_decompress_packed_workspace(numel, p.world, p.capacity)
                ws = self._dec_ws(dev, wsz)
                vd = _lib.VD[p.vdtype]
                idd = _lib.ID[p.idtype]
                _lib.check(L.dgc_decompress_packed(_lib.ptr(p.packed), p.world, p.rank_stride, p.capacity, vd,
                                                   idd, _lib.ptr(grad), numel, scale, _lib.ptr(ws), wsz,
                                                   stream), "dgc_decompress_packed")
                return grad.view(shape)
            values, indices = tensor
            values = values.reshape(-1).contiguous()
            indices = indices.reshape(-1).contiguous()
            if values.dtype not in _lib.VD:
                values = values.to(torch.float32)
            if indices.dtype not in _lib.ID:
                indices = indices.to(torch.int64)
            # index_put_ wraps a negative index (>= -numel); the kernels take [0, numel)
            indices = torch.where(indices < 0, indices + numel, indices)
            offs = getattr(tensor, "run_offsets", None)
            import ctypes
            if offs is not None:
                arr = (ctypes.c_int64 * len(offs))(*offs)
                nruns = len(offs) - 1
                wsz = L.dgc_decompress_workspace(numel, nruns)
            else:
                arr, nruns = None, 0
                wsz = L.dgc_decompress_workspace(numel, 64)
            ws = self._dec_ws(dev, wsz)
            status = L.dgc_decompress(_lib.ptr(values), _lib.VD[values.dtype], _lib.ptr(indices),
                                      _lib.ID[indices.dtype], values.numel(), arr, nruns, _lib.ptr(grad), numel,
                                      scale, _lib.ptr(ws), wsz, stream)
            if status == 6:   # DGC_ERR_UNSORTED: many descending runs -> one stable-sorted run
                order = torch.sort(indices, stable=True).indices
                values, indices = values[order].contiguous(), indices[order].contiguous()
                arr = (ctypes.c_int64 * 2)(0, values.numel())
                status = L.dgc_decompress(_lib.ptr(values), _lib.VD[values.dtype], _lib.ptr(indices),
                                          _lib.ID[indices.dtype], values.numel(), arr, 1, _lib.ptr(grad), numel,
                                          scale, _lib.ptr(ws), wsz, stream)
            _lib.check(status, "dgc_decompress")
            return grad.view(shape)
        if self.fp16_values and vdtype.is_floating_point:
            tensor = tensor.type(vdtype)
        return self.memory.compensate(tensor, name, accumulate=False)

    def _decompress16(self, tensor, grad, numel, shape, scale):
        """dgc/compression.py:179-194 into a bf16 / fp16 gradient (dgc_decompress16):
        runs (ranks) in rank order, every add and the 1/W scale rounded to its dtype."""
        import ctypes
        values, indices = tensor
        values = values.reshape(-1).contiguous()
        indices = indices.reshape(-1).contiguous()
        if values.dtype not in _lib.VD:
            values = values.to(grad.dtype)
        if indices.dtype not in _lib.ID:
            indices = indices.to(torch.int64)
        offs = getattr(tensor, "run_offsets", None)
        if offs is None or not getattr(tensor, "distinct_runs", False):
            # input whose runs may repeat an index (the reference's list format, or
            # foreign payloads): one stably sorted run, each index folded in input order
            # (index_put_'s serial order; as the fp32 path's unsorted fallback). Negative
            # indices wrap as in index_put_: normalised first, so -1 and n - 1 fold together
            indices = torch.where(indices < 0, indices + numel, indices)
            order = torch.sort(indices, stable=True).indices
            values, indices = values[order].contiguous(), indices[order].contiguous()
            offs, nruns = [0, values.numel()], -1
        else:
            nruns = len(offs) - 1
        arr = (ctypes.c_int64 * len(offs))(*[int(o) for o in offs])
        dev = grad.device
        bad = ctypes.c_void_p(self._sink(dev).decompress_words)   # 1: an index outside the gradient
        _lib.check(_lib.lib().dgc_decompress16(_lib.ptr(values), _lib.VD[values.dtype], _lib.ptr(indices),
                                               _lib.ID[indices.dtype], arr, nruns, _lib.ptr(grad),
                                               _lib.VD[grad.dtype], numel, scale, bad,
                                               _lib.stream_of(dev)), "dgc_decompress16")
        return grad.view(shape)

    # ------------------------------------------------------------------ collectives
    def communicate(self, tensor_compressed, name, op):
        """dgc/compression.py:200-206: sparse payload -> one packed allgather;
        dense tensors -> allreduce (Average)."""
        self.op = op
        if self.compress_ratio < 1.0 and name in self.attributes:
            values, indices = tensor_compressed
            packed = self._payloads.get(name)
            payload, lay = packed if packed is not None else (None, None)
            ours = payload is not None and values.data_ptr() == payload.data_ptr() + lay[4]
            if not ours:
                payload, lay = self._pack_foreign(name, values, indices)
            k, vdt, idt, stride, voff, ioff = lay
            handle = comm.allgather_packed_async(payload)
            return _PackedHandle(handle, name, k, vdt, idt, stride, voff, ioff)
        return comm.allreduce_async_(tensor_compressed, name=name, op=op)

    def _pack_foreign(self, name, values, indices):
        """Pack (values, indices) that did not come from this compressor's compress."""
        payload, lay = self._new_payload(name, values.device)
        n = values.numel()
        payload[:16].view(torch.int64).copy_(torch.tensor([n, 0], dtype=torch.int64))
        v, i = self._views(payload, lay, n)
        v.copy_(values.reshape(-1, 1))
        i.copy_(indices.reshape(-1, 1))
        return payload, lay

    def synchronize(self, handle):
        """dgc/compression.py:208-212. A gathered header whose count is outside [0,
        capacity] (a payload corrupted in transit, README.md:132) raises here."""
        self.check()
        if isinstance(handle, _PackedHandle):
            gathered = handle.handle.wait()
            W = gathered.numel() // handle.stride
            rows = gathered.view(W, handle.stride)
            head = rows[:, :16].contiguous().view(torch.int64).view(W, 2).tolist()
            counts = [c for c, _ in head]
            bad = [r for r, c in enumerate(counts) if not 0 <= c <= handle.capacity]
            if bad:
                raise RuntimeError(f"DGCCompressor.synchronize: {handle.name}: the payload gathered from rank(s) {bad} "
                                   f"holds count(s) {[counts[r] for r in bad]} outside [0, {handle.capacity}] "
                                   "(corrupted in transit?)")
            vb = torch.empty(0, dtype=handle.vdtype).element_size()
            ib = torch.empty(0, dtype=handle.idtype).element_size()
            vals = [rows[r, handle.voff: handle.voff + c * vb].view(handle.vdtype) for r, c in enumerate(counts)]
            idxs = [rows[r, handle.ioff: handle.ioff + c * ib].view(handle.idtype) for r, c in enumerate(counts)]
            out = _Gathered([torch.cat(vals).view(-1, 1), torch.cat(idxs).view(-1, 1)])
            out.packed = gathered
            out.world = W
            out.rank_stride = handle.stride
            out.capacity = handle.capacity
            out.vdtype, out.idtype = handle.vdtype, handle.idtype
            offs = [0]
            for c in counts:
                offs.append(offs[-1] + c)
            out.run_offsets = offs
            # every rank's run came from compress (distinct indices): the per-run scatter;
            # a foreign payload anywhere sends the 16-bit decompress to its sorted fold
            out.distinct_runs = all(mark == _OURS for _, mark in head)
            return out
        if isinstance(handle, (tuple, list)):
            return [comm.synchronize(h) for h in handle]
        return comm.synchronize(handle)
