"""World-size-2 gloo tests on CPU: the drop-in DistributedOptimizer, the packed
sparse allgather (communicate / synchronize) and dgc.comm collectives, checked
against the weights the REFERENCE produced for the same 3 training steps
(tests/golden/optimizer.npz)."""
import os

import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN
import dist_helpers as H


def run(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = H.free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    out = {}
    while not q.empty():
        rank, res = q.get()
        out[rank] = res
    assert sorted(out) == list(range(world))
    return out


@pytest.mark.timeout(300)
def test_distributed_optimizer_matches_reference_weights():
    out = run(H.optimizer_worker, 2, os.path.join(GOLDEN, "optimizer.npz"))
    for rank, mismatches in out.items():
        assert mismatches == [], (rank, mismatches)


@pytest.mark.timeout(300)
def test_resnet20_config0_matches_reference():
    """BASELINE configs[0]: ResNet-20, ratio 0.001, warmup 5, fp16 values, int32 indices, 2 ranks."""
    out = run(H.resnet20_worker, 2, GOLDEN)
    for rank, problems in out.items():
        assert problems == [], (rank, problems)


@pytest.mark.timeout(300)
def test_comm_collectives_gloo():
    out = run(H.comm_worker, 2)
    for rank, (gathered, avg, sm, (size, rk), big) in out.items():
        assert gathered == [0.0, 1.0, 10.0, 11.0, 12.0]       # rank order, ragged rows
        assert avg == [1.5, 1.5, 1.5] and sm == [3.0, 3.0]
        assert size == 2 and rk == rank
        # a tensor above comm.RANK_ORDER_MAX: one in-place backend allreduce, / W
        assert big == (True, True, {"all_reduce": 1, "all_gather_into_tensor": 0}), big


@pytest.mark.timeout(120)
def test_one_rank_shortcut_switch(monkeypatch):
    """Without a group a world of one never issues a collective; a one-rank group with
    comm.ONE_RANK_SHORTCUT cleared does (the RCCL tests' switch, here over gloo)."""
    import torch
    import torch.distributed as dist
    from dgc import comm
    assert comm.size() == 1 and not comm.one_rank_collectives()
    monkeypatch.setattr(comm, "ONE_RANK_SHORTCUT", False)
    assert not comm.one_rank_collectives()   # no group: still the shortcut
    h = comm.allreduce_async_(torch.ones(3))
    assert h._work is None
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{H.free_port()}", rank=0, world_size=1)
    try:
        assert comm.one_rank_collectives()
        t = torch.arange(6, dtype=torch.float32).view(3, 2)
        h = comm.allgather_async(t)
        assert h._work is not None and torch.equal(comm.synchronize(h), t)
        x = torch.full((4,), 3.0)
        h = comm.allreduce_async_(x, op=comm.Average)
        assert h._work is not None and torch.equal(comm.synchronize(h), torch.full((4,), 3.0))
        monkeypatch.setattr(comm, "ONE_RANK_SHORTCUT", True)
        assert not comm.one_rank_collectives() and comm.allreduce_async_(x)._work is None
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("label,world", [("w3_fp32", 3), ("w4_fp16_wm5o", 4), ("w8_fp16", 8)])
def test_dense_average_multi_rank_matches_reference(label, world):
    """W = 3 / 4 / 8 gloo ranks on CPU: the reference's weights (tests/golden/
    optimizer_multi.*), whose dense tensors' Average is the rank-order sum / W in the wire
    dtype — dgc.comm.allreduce_async_ as an allgather summed in rank order."""
    out = run(H.multi_worker, world, GOLDEN, label)
    for rank, problems in out.items():
        assert problems == [], (rank, problems)
