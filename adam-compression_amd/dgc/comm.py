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
  * allreduce with ``Average`` is the rank sum divided by the world size, in place.

The DGC sparse payload itself does NOT go through the generic allgather: each
rank's (count, values, indices) is packed into one fixed-capacity byte buffer
(``dgc_payload_layout``) and exchanged with a single ``all_gather_into_tensor``
(see ``allgather_packed_async``), so no size exchange is needed.
"""
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


def allreduce_async_(tensor, name=None, op=Average):
    """In-place allreduce of ``tensor``; ``synchronize`` returns it (sum, /W for Average)."""
    if op not in (Average, Sum):
        raise NotImplementedError(f"allreduce op {op!r} (Adasum is out of scope)")
    W = size()
    if _shortcut(W):
        return Handle(output=tensor)
    staged = tensor.cpu() if _backend_needs_host(tensor) else tensor
    work = dist.all_reduce(staged, op=dist.ReduceOp.SUM, async_op=True)

    def finish():
        if staged is not tensor:
            tensor.copy_(staged)
        if op == Average:
            tensor.div_(W)
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


def allgather_packed_async(payload, out=None):
    """Fixed-size byte allgather of one packed DGC payload per rank -> [W * P] bytes."""
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
    work = dist.all_gather_into_tensor(out, payload, async_op=True)
    return Handle(work, lambda: out)


def synchronize(handle):
    return handle.wait()
