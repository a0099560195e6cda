"""Flat-bucket DGC step with no host synchronisation (the padded fast path).

One fp32 gradient bucket per rank goes through the whole DGC step of the
reference — compensate -> sample -> threshold -> select/adapt/resample -> update
(dgc/memory.py:50-77, dgc/compression.py:109-177) -> allgather
(dgc/compression.py:200-212) -> decompress (dgc/compression.py:179-194) — with
every decision kept on the device:

* the payload is fixed-capacity: ``[count | values(k) | indices(k)]`` per rank
  (``dgc_payload_layout``), so the RCCL allgather needs no size exchange and the
  decompress reads each rank's count on the device;
* the selection runs in ``DGC_SYNC_DEVICE`` mode (adaptation recounts and the
  resample chain are launched and early-exit on a device flag);
* the decompress is ``grad.zero_()`` (dgc/compression.py:191) as a one-shot
  ``dgc_fill_zero`` followed by a sparse scatter of the gathered entries.
  ``fill="allgather"`` issues the fill on a side stream right after the RCCL
  allgather is enqueued (ordered after the selection), so at W > 1 the 4 B/elem
  zero fill runs under the xGMI transfer instead of after it; the decompress then
  only scatters. ``"inline"`` runs fill + scatter after the allgather.
  ``"sparse"`` (opt-in) treats ``out`` as a persistent output
  bucket: when it is the tensor the previous step decompressed into and nobody has
  written it since (same storage, same torch version counter), it is +0.0 except at
  the previous step's W*k gathered indices, so ``zero_()`` is a sparse re-zero of
  those slots — W*k scattered stores instead of a 4 B/elem stream, issued on a side
  stream at the start of the step so they run under K1 (``dgc_clear_packed``, then
  ``dgc_scatter_packed_cleared``; ``decompress`` alone does both in one call,
  ``dgc_decompress_packed_over``); the dense result is the same, bit for bit. Any other ``out``
  (first step, a new tensor, one modified in place) gets the dense fill. The
  payload (W = 1) / gather buffer (W > 1) alternates between two buffers so the
  previous step's indices survive the current step.
* at W > 1 with a large step (``exchange_parts``, dgc/exchange.py) the allgather goes
  out in parts and each part is scattered as it lands, so only the last part's share
  of the W-dependent scatter is exposed after the exchange.
  **What "sparse" cannot see**: writes through ``out.data`` (the reference's own idiom,
  e.g. ``grad.data.mul_``) and raw-pointer writes do not bump torch's version counter,
  so after one the re-zero would leave stale values. Only a caller that owns ``out``
  and never writes it (the bench) should opt in; ``"auto"`` (the default) is the dense
  fill ``"inline"``.

The numerics are those of the drop-in ``DGCCompressor`` + ``DGCSGDMemory`` (same
kernels); the sample start is drawn from a ``random.Random`` seeded identically on
every rank, one draw per step, like the reference's global ``random`` call.
"""
import ctypes
import math
import random

import torch
import torch.distributed as dist

from . import _lib
from . import comm
from .exchange import SplitExchange, split_parts

__all__ = ["DGCBucket", "algorithmic_bytes"]


def algorithmic_bytes(numel, k, num_samples, world, vbytes=4, ibytes=8):
    """Bytes one rank must move per step:
    compensate 20N + select re-read 4N + dense decompress write 4N, the samples 4S,
    masking 8k, payload written k(vb+ib) + gathered W*k(vb+ib) read, scatter RMW 8Wk."""
    return (28 * numel + 4 * num_samples + 8 * k + (1 + world) * k * (vbytes + ibytes) + 8 * world * k)


class DGCBucket:
    def __init__(self, numel, compress_ratio=0.001, momentum=0.9, nesterov=True, momentum_masking=True,
                 sample_ratio=0.01, compress_upper_bound=1.3, compress_lower_bound=0.8,
                 max_adaptation_iters=10, resample=True, fp16_values=False, int32_indices=False,
                 device=None, world_size=None, seed=42, fill="auto", deferred_masking=True, exchange_parts="auto",
                 resample_order="topk"):
        from .compression import DGCCompressor, _layout
        self.device = torch.device(device or "cuda")
        self.numel = N = int(numel)
        ratio = compress_ratio if compress_ratio <= 1.0 else 1.0 / compress_ratio
        sample_ratio = min(max(sample_ratio, 0.01), 1.0)
        self.stride, self.num_samples = DGCCompressor._stride_and_samples(N, ratio, sample_ratio)
        self.top_k_samples = int(math.ceil(self.num_samples * ratio))
        self.k = int(math.ceil(N * ratio))
        self.momentum, self.nesterov = float(momentum), bool(nesterov)
        self.world = world_size or (dist.get_world_size() if dist.is_initialized() else 1)
        self.vdtype = torch.float16 if fp16_values else torch.float32
        self.idtype = torch.int32 if int32_indices else torch.int64
        self.rng = random.Random(seed)

        p = _lib.SelectParams()
        p.numel, p.num_selects, p.num_samples = N, self.k, self.num_samples
        p.upper_count = math.floor(self.k * compress_upper_bound)
        p.lower_count = math.ceil(compress_lower_bound * self.k)
        p.upper, p.lower = float(compress_upper_bound), float(compress_lower_bound)
        p.max_iters, p.resample, p.masking = int(max_adaptation_iters), int(bool(resample)), int(bool(momentum_masking))
        # update_memory 2: the first-k branches' DGCSGDMemory.update zeroing rides in the
        # next step's K1, which streams vec/mmt anyway (mmt/vec below flush it on read)
        p.vdtype, p.idtype = _lib.VD[self.vdtype], _lib.ID[self.idtype]
        p.update_memory = 2 if deferred_masking else 1
        # "index" (opt-in): an untied resample lists its set in index order (DGCBatch's
        # default); a flat bucket's resample (up to 64k candidates) mostly exceeds the
        # one-workgroup set path, so it keeps torch.topk's order by default
        if resample_order not in ("index", "topk"):
            raise ValueError(f"resample_order must be 'index' or 'topk', not {resample_order!r}")
        p.resample_order = 1 if resample_order == "index" else 0
        self.status = _lib.StatusSink("DGCBucket", self.device)   # DGC_K5_BROKEN, checked every step
        p.status_sink = self.status.address
        self.params = p

        dev = self.device
        self._mmt = torch.zeros(N, dtype=torch.float32, device=dev)
        self._vec = torch.zeros(N, dtype=torch.float32, device=dev)
        self._pending = False
        L = _lib.lib()
        self.sampled = N != self.num_samples
        # zero-filled: per-tensor state (deferred masking, spill and window counts) lives in it
        self.ws = torch.zeros(L.dgc_compress_workspace(N, self.k, self.num_samples), dtype=torch.uint8,
                              device=dev)
        self.spec = torch.full((8,), float("inf"), dtype=torch.float32, device=dev)
        self.info = torch.zeros(_lib.INFO_BYTES, dtype=torch.uint8, device=dev)
        self.rank_stride, self.voff, self.ioff = _layout(self.k, self.vdtype, self.idtype)
        if fill not in ("auto", "inline", "allgather", "sparse"):
            raise ValueError(f"fill must be 'auto', 'inline', 'allgather' or 'sparse', not {fill!r}")
        if fill == "auto":   # the dense zero_() is always right; the re-zero is opt-in (see above)
            fill = "inline"
        self.fill = fill
        nbuf = 2 if fill == "sparse" else 1   # the previous step's gathered indices stay readable
        self._payloads = [torch.zeros(self.rank_stride, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        # (W = 1 exchanges too when comm.one_rank_collectives(): the RCCL tests' one-rank group)
        self.exchanging = self.world > 1 or comm.one_rank_collectives()
        self._gathers = ([torch.zeros(self.world * self.rank_stride, dtype=torch.uint8, device=dev)
                          for _ in range(nbuf)] if self.exchanging else self._payloads)
        # W > 1: the allgather in parts, each scattered as it lands (dgc/exchange.py)
        self.parts = split_parts(self.world, self.k, exchange_parts)
        self.xchg = None
        if self.parts > 1:
            self.xchg = SplitExchange(self.k, N, self.world, self.parts, self.vdtype, self.idtype, dev, nbuf)
            self._gathers = self.xchg.gathers
        self._inflight = None
        self._par = 0
        self._last_out = None   # (data_ptr, numel, _version) of the output after the last decompress
        self._last_gathered = None
        self.dec_ws = (torch.empty(L.dgc_decompress_packed_workspace(N, self.world, self.k), dtype=torch.uint8,
                                   device=dev) if self.xchg is None else None)
        # a bad index or gathered count in the decompress lands in ``status`` (raised next step)
        self.status.bind(self.dec_ws if self.xchg is None else self.xchg.ws)
        self.scale = 1.0 / self.world
        self._L = L
        if fill in ("allgather", "sparse"):
            self.side = torch.cuda.Stream(device=dev)
            self._ev_go = torch.cuda.Event()
            self._ev_filled = torch.cuda.Event()

    # ---------------------------------------------------------------- state
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
            _lib.check(self._L.dgc_compress_flush(self._vec.data_ptr(), self._mmt.data_ptr(), self.stride,
                                                  ctypes.byref(self.params), self.ws.data_ptr(), self.ws.numel(),
                                                  _lib.stream_of(self.device)), "dgc_compress_flush")
            self._pending = False

    @property
    def mmt(self):
        """Momentum (DGCSGDMemory.momentums), masking applied."""
        self.flush()
        return self._mmt

    @property
    def vec(self):
        """Velocity (DGCSGDMemory.velocities), masking applied."""
        self.flush()
        return self._vec

    # ---------------------------------------------------------------- phases
    def compensate(self, grad):
        """K1: compensate + fused strided sample + speculative candidate lists. Raises
        first if a previous step's resample replay reported DGC_K5_BROKEN, or its
        decompress met an index or a gathered count out of range (``status``)."""
        self.status.check()
        L = self._L
        self._par += 1   # a step starts: the other payload / gather buffer
        self.start = self.rng.randint(0, self.stride - 1) if self.sampled else 0
        _lib.check(L.dgc_compress_begin(grad.data_ptr(), self._mmt.data_ptr(), self._vec.data_ptr(), self.momentum,
                                        int(self.nesterov), self.start, self.stride, ctypes.byref(self.params),
                                        self.spec.data_ptr(), self.ws.data_ptr(), self.ws.numel(),
                                        _lib.stream_of(self.device)), "dgc_compress_begin")
        self.cnt = (self.numel - self.start + self.stride - 1) // self.stride if self.sampled else self.numel
        self._pending = False   # K1 applied it

    def select(self):
        """K3 threshold + K4 selection / adaptation / resample / emit + masking, into the payload."""
        L = self._L
        base = self.payload.data_ptr()
        self.params.order_out = base + 8   # header word 1: the W = 1 scatter's ascending-order flag
        self._pending = self.params.update_memory == 2
        _lib.check(L.dgc_compress_finish(self._vec.data_ptr(), self._mmt.data_ptr(), self.start, self.stride,
                                         self.top_k_samples, ctypes.byref(self.params), self.spec.data_ptr(),
                                         _lib.SPEC_MARGIN, base + self.voff, base + self.ioff, base,
                                         self.info.data_ptr(), self.ws.data_ptr(), self.ws.numel(),
                                         _lib.SYNC_DEVICE, _lib.stream_of(self.device)), "dgc_compress_finish")

    def exchange(self):
        """The packed allgather (RCCL over xGMI; gloo stages through the host). Split
        (``parts`` > 1): the parts' collectives are only issued; decompress waits for
        each as it scatters it."""
        if self.exchanging:
            if self.xchg is not None:
                self._inflight = self.xchg.send(self.payload, self.gathered)
            else:
                comm.allgather_packed_async(self.payload, out=self.gathered, wait=True).wait()

    def _decompress_split(self, out, dense, cleared=False):
        """The split exchange's decompress: the zero_() (the dense fill, or the sparse
        re-zero of the previous step's entries) issued first, so it runs under the
        first part's collective, then one scatter per part as it lands."""
        if self._inflight is None:
            raise RuntimeError("DGCBucket: decompress of a split exchange before exchange()")
        handles, self._inflight = self._inflight, None
        cur = self.gathered
        if dense and not cleared:
            if self.fill == "sparse" and self._reusable(out) and self._last_gathered is not cur:
                self.xchg.clear(self._last_gathered, out, _lib.stream_of(self.device))
                cleared = True
            else:
                _lib.check(self._L.dgc_fill_zero(out.data_ptr(), self.numel, _lib.stream_of(self.device)),
                           "dgc_fill_zero")
        self.xchg.scatter(cur, handles, out, self.scale, cleared)
        self._remember(out, cur)

    def decompress(self, out, dense=True):
        """dense: out = scale * (rank-order sum of the gathered entries), zeros elsewhere.
        dense=False: out already holds +0.0 (see fill_zero); only the entries are written.
        fill="sparse": a dense decompress into the previous step's untouched output
        re-zeroes only the previous entries (see the module docstring)."""
        if self.xchg is not None:
            return self._decompress_split(out, dense)
        L = self._L
        cur = self.gathered
        args = self._dec_args(out)
        if dense and self.fill == "sparse" and self._reusable(out) and self._last_gathered is not cur:
            _lib.check(L.dgc_decompress_packed_over(cur.data_ptr(), self._last_gathered.data_ptr(), *args),
                       "dgc_decompress_packed_over")
        else:
            fn = L.dgc_decompress_packed if dense else L.dgc_scatter_packed
            _lib.check(fn(cur.data_ptr(), *args), "dgc_decompress_packed" if dense else "dgc_scatter_packed")
        self._remember(out, cur)

    def _dec_args(self, out):
        return (self.world, self.rank_stride, self.k, _lib.VD[self.vdtype], _lib.ID[self.idtype], out.data_ptr(),
                self.numel, self.scale, self.dec_ws.data_ptr(), self.dec_ws.numel(), _lib.stream_of(self.device))

    def _reusable(self, out):
        """out still holds exactly the last decompress's result: same storage, and no
        in-place write since (torch's version counter; ours are raw-pointer writes)."""
        return self._last_gathered is not None and self._last_out == (out.data_ptr(), out.numel(), out._version)

    def _remember(self, out, cur):
        self._last_out = (out.data_ptr(), out.numel(), out._version)
        self._last_gathered = cur

    def _clear_on_side(self, out):
        """The sparse re-zero of the previous step's entries, on the side stream at the
        start of the step (ordered after everything already issued, e.g. an optimizer
        reading out), so it runs under K1 instead of before the scatter."""
        self.side.wait_stream(torch.cuda.current_stream(self.device))
        if self.xchg is not None:
            self.xchg.clear(self._last_gathered, out, self.side.cuda_stream)
            self._ev_filled.record(self.side)
            return
        _lib.check(self._L.dgc_clear_packed(self._last_gathered.data_ptr(), self.world, self.rank_stride, self.k,
                                            _lib.VD[self.vdtype], _lib.ID[self.idtype], out.data_ptr(), self.numel,
                                            self.dec_ws.data_ptr(), self.dec_ws.numel(), self.side.cuda_stream),
                   "dgc_clear_packed")
        self._ev_filled.record(self.side)

    def _fill_on_side(self, out):
        """zero_() of the output on the side stream, ordered after the event recorded
        at the end of the selection (so it never races a reader of the previous step)."""
        self.side.wait_event(self._ev_go)
        _lib.check(self._L.dgc_fill_zero(out.data_ptr(), self.numel, self.side.cuda_stream), "dgc_fill_zero")
        self._ev_filled.record(self.side)

    def step(self, grad, out, events=None):
        """compensate -> threshold -> select -> allgather -> decompress into ``out``;
        ``events`` maps a phase name to a (start, end) pair of torch.cuda.Event recorded
        around it on the current stream."""
        ev = events or {}
        self.status.check()   # before anything of this step is issued
        # an output that shares storage with the gradient (the reference's in-place
        # layout) is rewritten with each new gradient: always the dense fill there
        aliased = out.untyped_storage().data_ptr() == grad.untyped_storage().data_ptr()
        if aliased:
            self._last_out = None
        cleared = self.fill == "sparse" and not aliased and self._reusable(out)
        if cleared:
            self._clear_on_side(out)

        def decompress():
            if cleared:   # the entries onto the re-zeroed output
                torch.cuda.current_stream(self.device).wait_event(self._ev_filled)
                if self.xchg is not None:
                    self._decompress_split(out, True, cleared=True)
                    return
                cur = self.gathered
                _lib.check(self._L.dgc_scatter_packed_cleared(cur.data_ptr(), *self._dec_args(out)),
                           "dgc_scatter_packed_cleared")
                self._remember(out, cur)
            elif self.fill != "allgather":
                self.decompress(out)
                if aliased:
                    self._last_out = None
            else:
                torch.cuda.current_stream(self.device).wait_event(self._ev_filled)
                self.decompress(out, dense=False)

        for name, fn in (("compensate", lambda: self.compensate(grad)), ("select", self.select),
                         ("allgather", self.exchange), ("decompress", decompress)):
            pair = ev.get(name)
            if pair:
                pair[0].record()
            fn()
            if pair:
                pair[1].record()
            if self.fill == "allgather":
                if name == "select":      # the fill may start once the selection is done ...
                    self._ev_go.record(torch.cuda.current_stream(self.device))
                elif name == "allgather":  # ... and is enqueued behind the RCCL launch
                    self._fill_on_side(out)

    def last_info(self):
        self.status.check(sync=True)
        raw = self.info.cpu().numpy().tobytes()
        return _lib.info_dict(_lib.SelectInfo.from_buffer_copy(raw), "DGCBucket")
