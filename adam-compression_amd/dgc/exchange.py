"""Split exchange: the packed allgather of a step (dgc/compression.py:200-212) in
``parts`` collectives, with the decompress (dgc/compression.py:179-194) of each part
scattered while the later parts are still in flight.

The W-dependent part of a flat step is the scatter of the W*k gathered entries: at
W = 8 and k = 1M it is ~0.3 ms, exposed after a single allgather. Split, the rank's
packed payload is re-laid out as ``parts`` part buffers (``dgc_payload_split``: the
entries in payload order, each part's header carrying the smallest index of the parts
after it), each part goes out in its own RCCL allgather on torch's NCCL stream, and
the compute stream waits for them one at a time: after part p it scatters every index
below the smallest such bound over the ranks (all of that index's entries have landed),
so only the last part's share is exposed. The dense result is the single-collective
decompress's bit for bit (same rank-order sums; tests/test_gpu_split.py).

Used by DGCBucket / DGCBatch (fp32 parameters) at W > 1; ``parts="auto"`` splits a
step of >= 2^21 gathered entries (2 parts at W <= 4, 4 at W = 8) and leaves smaller ones
to one allgather: each extra collective costs ~35 us of fixed hand-off
and hides at most its share of the scatter, which at 2M entries (flat-1B, W = 2: 0.07
ms) only breaks even and at VGG-16-BN's 1.1M (W = 8) loses.

``DGC_EXCHANGE_PARTS`` overrides ``"auto"``; every rank must issue the same collectives,
so an override is checked across the ranks when the layout is built (``agree``).
"""
import ctypes
import os

import torch

from . import _lib, comm

__all__ = ["SplitExchange", "split_parts"]


def split_parts(world, capacity, parts="auto"):
    """The number of collectives for a step of ``capacity`` entries per rank."""
    env = os.environ.get("DGC_EXCHANGE_PARTS")
    if parts == "auto" and env:
        parts = int(env)
    multi = world > 1 or comm.one_rank_collectives()
    if parts == "auto":
        if not multi or world * capacity < (1 << 21):
            return 1
        return 2 if world <= 4 else 4
    parts = int(parts)
    if not multi or parts <= 1:
        parts = 1
    elif parts > 8 or world * parts > 64:
        raise ValueError(f"exchange parts must be 1..8 with world * parts <= 64 (world {world}, parts {parts})")
    if env and multi:
        agree(parts)
    return parts


def agree(parts):
    """Raises unless every rank chose ``parts`` (a per-rank DGC_EXCHANGE_PARTS that
    differs would issue different collectives and hang or corrupt the exchange). One
    MAX-allreduce of (parts, -parts) over the process group, at layout time only."""
    import torch.distributed as dist
    if not comm.is_initialized():
        return
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([parts, -parts], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    hi, lo = int(t[0]), -int(t[1])
    if hi != parts or lo != parts:
        raise RuntimeError(f"DGC_EXCHANGE_PARTS differs across ranks (parts between {lo} and {hi}); set the "
                           "same value on every rank")


class SplitExchange:
    """The split payload of this rank, ``nbuf`` part-major gather buffers and the
    phase scatter's workspace."""

    def __init__(self, capacity, numel, world, parts, vdtype, idtype, device, nbuf):
        L = self._L = _lib.lib()
        self.capacity, self.numel, self.world, self.parts = int(capacity), int(numel), int(world), int(parts)
        self.vd, self.id = _lib.VD[vdtype], _lib.ID[idtype]
        pc = ctypes.c_int64(0)
        self.part_bytes = L.dgc_payload_split_layout(self.capacity, self.parts, self.vd, self.id, ctypes.byref(pc))
        self.part_capacity = pc.value
        nb = L.dgc_payload_split_bytes(self.capacity, self.parts, self.vd, self.id)
        if self.part_bytes <= 0 or nb <= 0:
            raise ValueError(f"dgc_payload_split_layout: capacity {capacity}, parts {parts}")
        self.split = torch.zeros(nb, dtype=torch.uint8, device=device)   # its scratch must start zero
        self.gathers = [torch.zeros(self.parts * self.world * self.part_bytes, dtype=torch.uint8, device=device)
                        for _ in range(nbuf)]
        wsz = L.dgc_decompress_split_workspace(self.numel, self.world, self.parts, self.capacity)
        if wsz == 0:
            raise ValueError(f"dgc_decompress_split_workspace: world {world}, parts {parts}")
        self.ws = torch.empty(wsz, dtype=torch.uint8, device=device)
        self.device = device

    def send(self, payload, gathered):
        """Splits this rank's payload and issues one allgather per part (in order on
        torch's collective stream, behind everything issued so far); returns the handles."""
        L, st = self._L, _lib.stream_of(self.device)
        _lib.check(L.dgc_payload_split(payload.data_ptr(), self.capacity, self.parts, self.vd, self.id,
                                       self.split.data_ptr(), st), "dgc_payload_split")
        pb, W = self.part_bytes, self.world
        return [comm.allgather_packed_async(self.split[p * pb:(p + 1) * pb],
                                            out=gathered[p * W * pb:(p + 1) * W * pb])
                for p in range(self.parts)]

    def scatter(self, gathered, handles, out, scale, cleared):
        """The phases: each waits for its part (a stream wait under RCCL) and scatters
        what has landed. ``out`` holds +0.0 (cleared: re-zeroed by ``clear`` on this
        workspace)."""
        L, st = self._L, _lib.stream_of(self.device)
        for p, h in enumerate(handles):
            h.wait()
            _lib.check(L.dgc_scatter_split(gathered.data_ptr(), self.world, self.parts, p, self.capacity, self.vd,
                                           self.id, out.data_ptr(), self.numel, scale, int(bool(cleared) and p == 0),
                                           self.ws.data_ptr(), self.ws.numel(), st), "dgc_scatter_split")

    def clear(self, prev_gathered, out, stream):
        """The previous step's entries re-zeroed in ``out`` (which holds exactly that
        step's result), on ``stream``; also resets the phase scatter's status words."""
        _lib.check(self._L.dgc_clear_split(prev_gathered.data_ptr(), self.world, self.parts, self.capacity, self.vd,
                                           self.id, out.data_ptr(), self.numel, self.ws.data_ptr(), self.ws.numel(),
                                           stream), "dgc_clear_split")
