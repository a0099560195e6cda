"""Collective facade replacing ``horovod.torch`` / ``horovod.torch.mpi_ops`` on the DGC path.

The reference calls Horovod's ``size``, ``rank``, ``allgather_async``,
``allreduce_async_``, ``synchronize`` and ``Average`` (dgc/compression.py:3-10,
dgc/horovod/optimizer.py:24-27). Here they sit on ``torch.distributed``: backend
``nccl`` is RCCL on ROCm (one process per MI355X, xGMI inside a node); ``gloo``
serves the CPU plumbing tests. Without an initialised process group everything
behaves as a world of one rank.

Semantics kept from Horovod:
  * allgather concatenates along dim 0 in rank order, each rank may send a
    different number of rows;
  * allreduce with ``Average`` is the rank sum divided by the world size, in place —
    summed in RANK ORDER (an allgather, then ``dgc_rank_sum``), as the oracle restates
    Horovod's Average, for tensors up to ``RANK_ORDER_MAX`` elements (every dense DGC
    tensor: biases and BatchNorm vectors); a larger one (``Compression.none``, a ratio-1
    warmup epoch) is a backend allreduce, whose summation order is the backend's.

The DGC sparse payload itself does NOT go through the generic allgather: each
rank's (count, values, indices) is packed into one fixed-capacity byte buffer
(``dgc_payload_layout``) and exchanged with a single ``all_gather_into_tensor``
(see ``allgather_packed_async``), so no size exchange is needed.
"""
import os

import torch
import torch.distributed as dist

__all__ = ["Average", "Sum", "Adasum", "size", "rank", "local_rank", "is_initialized",
           "allreduce_async_", "allgather_async", "allgather_packed_async", "synchronize",
           "Handle"]

Average = "Average"
Sum = "Sum"
Adasum = "Adasum"


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def size():
    return dist.get_world_size() if is_initialized() else 1


def rank():
    return dist.get_rank() if is_initialized() else 0


def local_rank():
    import os
    return int(os.environ.get("LOCAL_RANK", rank()))


# A world of one rank returns its input without a collective. Cleared (tests), an
# initialised one-rank group runs the collective path itself — on a one-GPU box the
# only way to execute the RCCL branch (tests/test_gpu_rccl.py).
ONE_RANK_SHORTCUT = True


def _shortcut(W):
    return W == 1 and (ONE_RANK_SHORTCUT or not is_initialized())


def one_rank_collectives():
    """An initialised one-rank group with the shortcut cleared: the engines exchange
    through the collectives as at W > 1 (DGCBucket, DGCBatch, the split exchange)."""
    return is_initialized() and not ONE_RANK_SHORTCUT


def _backend_needs_host(t):
    """gloo moves host tensors only; keep GPU tensors on the GPU for nccl (RCCL)."""
    return t.is_cuda and dist.get_backend() != "nccl"


class Handle:
    """An in-flight collective. ``wait()`` returns its output (Horovod's synchronize)."""

    def __init__(self, work=None, finish=None, output=None):
        self._work = work
        self._finish = finish
        self._output = output
        self._done = work is None and finish is None

    def wait(self):
        if not self._done:
            if self._work is not None:
                self._work.wait()
            if self._finish is not None:
                self._output = self._finish()
            self._done = True
        return self._output


# Dense tensors up to this many elements are averaged in rank order through an allgather
# (W x the tensor's bytes in flight); larger ones take the backend's allreduce (a ring
# moves ~2x the bytes whatever W is). The dense tensors of the DGC configs are <= 4096
# elements each; DGC_RANK_ORDER_MAX overrides the cap (0: always the backend allreduce).
RANK_ORDER_MAX = int(os.environ.get("DGC_RANK_ORDER_MAX", str(1 << 20)))


def _rank_order_sum(rows, W, average):
    """acc = x_0; acc += x_1 ...; acc /= W on rows of a [W, n] host tensor (torch ops in
    the rows' dtype: the oracle's restatement of Horovod's Average)."""
    acc = rows[0].clone()
    for q in range(1, W):
        acc.add_(rows[q])
    if average:
        acc.div_(W)
    return acc


def allreduce_async_(tensor, name=None, op=Average):
    """In-place allreduce of ``tensor``; ``synchronize`` returns it (sum, /W for Average).

    The reference Average-allreduces its dense tensors through Horovod
    (dgc/compression.py:205-206). Its result is restated (tests/golden/make_goldens.py)
    as the RANK-ORDER sum divided by W, every op in the tensor's dtype; a backend
    allreduce sums in its own order, which decides the last bits from W = 3 on (fp16
    wire values above all). So the tensor is allgathered and summed in rank order: on
    the device by ``dgc_rank_sum`` (RCCL; gloo stages the bytes through the host), with
    torch ops for a host tensor (the gloo plumbing tests) or a dtype the kernel lacks."""
    if op not in (Average, Sum):
        raise NotImplementedError(f"allreduce op {op!r} (Adasum is out of scope)")
    W = size()
    if _shortcut(W):
        return Handle(output=tensor)
    src = tensor.contiguous().view(-1)
    n = src.numel()
    if n > RANK_ORDER_MAX:
        return _backend_allreduce(tensor, src, W, op == Average)
    device_sum = tensor.is_cuda and tensor.dtype in (torch.float32, torch.float16, torch.bfloat16)
    if _backend_needs_host(src) or not tensor.is_cuda:
        host = src.cpu()
        gathered = torch.empty(W * n, dtype=src.dtype)
        work = dist.all_gather_into_tensor(gathered, host, async_op=True)
    else:
        gathered = torch.empty(W * n, dtype=src.dtype, device=src.device)
        work = dist.all_gather_into_tensor(gathered, src, async_op=True)

    def finish():
        if device_sum:
            from . import _lib
            g = gathered.to(src.device) if not gathered.is_cuda else gathered
            dst = src if src.data_ptr() == tensor.data_ptr() else torch.empty_like(src)
            _lib.check(_lib.lib().dgc_rank_sum(_lib.ptr(g), _lib.VD[src.dtype], W, n * src.element_size(), n,
                                               int(op == Average), _lib.ptr(dst), _lib.stream_of(src.device)),
                       "dgc_rank_sum")
            if dst.data_ptr() != tensor.data_ptr():
                tensor.copy_(dst.view(tensor.shape))
        else:
            acc = _rank_order_sum(gathered.view(W, n), W, op == Average)
            tensor.copy_(acc.view(tensor.shape).to(tensor.device))
        return tensor

    return Handle(work, finish)


def _backend_allreduce(tensor, src, W, average):
    """A large dense tensor: the backend's SUM allreduce (RCCL's ring over xGMI on the
    device; gloo on a host copy), then ``div_(W)`` for Average — the reference's Horovod
    allreduce, in the backend's summation order (bit-equal to the rank-order restatement
    at W = 2, where fp addition commutes; parity unpinned from W = 3 on)."""
    buf = src.cpu() if _backend_needs_host(src) else src   # gloo moves host tensors
    work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, async_op=True)

    def finish():
        if average:
            buf.div_(W)
        if buf.data_ptr() != tensor.data_ptr():
            tensor.copy_(buf.view(tensor.shape))
        return tensor

    return Handle(work, finish)


def allgather_async(tensor, name=None):
    """Variable-length allgather along dim 0 (Horovod semantics)."""
    W = size()
    if _shortcut(W):
        return Handle(output=tensor)
    dev = tensor.device
    staged = tensor.cpu() if _backend_needs_host(tensor) else tensor
    rows = torch.tensor([staged.shape[0]], dtype=torch.int64, device=staged.device)
    all_rows = torch.empty(W, dtype=torch.int64, device=staged.device)
    dist.all_gather_into_tensor(all_rows, rows)
    counts = all_rows.tolist()
    cap = max(counts)
    padded = staged.new_zeros((cap,) + tuple(staged.shape[1:]))
    padded[: staged.shape[0]] = staged
    out = staged.new_empty((W * cap,) + tuple(staged.shape[1:]))
    work = dist.all_gather_into_tensor(out, padded, async_op=True)

    def finish():
        parts = [out[r * cap: r * cap + counts[r]] for r in range(W)]
        return torch.cat(parts, 0).to(dev)

    return Handle(work, finish)


# How a collective whose result the caller waits for at once is issued under RCCL:
# "current" (default) with async_op=False — torch then runs it on the caller's current
# stream, ordered like a kernel launch; "async" with async_op=True and wait() — on
# torch's collective stream, joined to the current stream by events, which costs a
# stream hand-off per collective (~35 us at one rank). DGC_COLLECTIVE_ISSUE
# selects; bench.py --rccl-one-rank times both.
COLLECTIVE_ISSUE = os.environ.get("DGC_COLLECTIVE_ISSUE", "current")


def allgather_packed_async(payload, out=None, wait=False):
    """Fixed-size byte allgather of one packed DGC payload per rank -> [W * P] bytes.
    ``wait=True``: the caller needs the result before its next launch (a single
    collective per step) — under RCCL it is issued on the current stream
    (``COLLECTIVE_ISSUE`` "current"), so the returned handle is already complete."""
    W = size()
    if out is None:
        out = torch.empty(W * payload.numel(), dtype=torch.uint8, device=payload.device)
    if _shortcut(W):
        if out.data_ptr() != payload.data_ptr():
            out.copy_(payload)
        return Handle(output=out)
    if _backend_needs_host(payload):
        host_in = payload.cpu()
        host_out = torch.empty(out.numel(), dtype=torch.uint8)
        work = dist.all_gather_into_tensor(host_out, host_in, async_op=True)
        return Handle(work, lambda: out.copy_(host_out))
    if wait and COLLECTIVE_ISSUE == "current":
        dist.all_gather_into_tensor(out, payload, async_op=False)
        return Handle(output=out)
    work = dist.all_gather_into_tensor(out, payload, async_op=True)
    return Handle(work, lambda: out)


def synchronize(handle):
    return handle.wait()
