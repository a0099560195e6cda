"""The RCCL branch of the collective facade (dgc/comm.py), executed on one MI355X.

A one-GPU box cannot hold two RCCL ranks, so these tests initialise a one-rank `nccl`
process group (RCCL on ROCm) and clear `comm.ONE_RANK_SHORTCUT`: the collectives then
run `all_gather_into_tensor` on the device tensors themselves (no host staging — that
is gloo's branch), as at W > 1. Checked: the packed payload allgather, the variable-row
allgather and the Average (an allgather summed in rank order) return their inputs, and
the reference's per-tensor hook path (dgc/horovod/optimizer.py:116-187: compress ->
packed allgather -> decompress, dense tensors averaged) over RCCL equals the same steps
without a collective bit for bit.
"""
import socket

import pytest
import torch
import torch.distributed as dist

import test_gpu_dropin as dropin

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_one_rank(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dgc import comm
    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=DEV)
    monkeypatch.setattr(comm, "ONE_RANK_SHORTCUT", False)
    try:
        assert dist.get_backend() == "nccl" and comm.size() == 1
        yield comm
    finally:
        torch.cuda.synchronize()
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_comm_collectives_over_rccl(rccl_one_rank):
    comm = rccl_one_rank
    gen = torch.Generator(device=DEV).manual_seed(5)
    payload = torch.randint(0, 256, (4099,), dtype=torch.uint8, device=DEV, generator=gen)
    h = comm.allgather_packed_async(payload)
    assert h._work is not None   # a collective was issued (the shortcut returns the input)
    out = comm.synchronize(h)
    assert out.is_cuda and out.data_ptr() != payload.data_ptr()
    assert torch.equal(out, payload)
    rows = torch.randn(37, 3, device=DEV, generator=gen)
    assert torch.equal(comm.synchronize(comm.allgather_async(rows)), rows)
    x = torch.randn(1 << 16, device=DEV, generator=gen)
    want = x.clone()
    assert torch.equal(comm.synchronize(comm.allreduce_async_(x, op=comm.Average)), want)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fp16", [False, True], ids=["wire-dtype-int64", "wire-fp16-int32"])
def test_per_tensor_path_over_rccl(fp16, rccl_one_rank, monkeypatch):
    """The hook path with every payload through RCCL equals it with none."""
    modes = ["fresh", "fresh", "inplace", "fresh"]
    calls = {"all_gather_into_tensor": 0, "all_reduce": 0}

    def counted(name):
        fn = getattr(dist, name)

        def wrapper(*a, **kw):
            calls[name] += 1
            return fn(*a, **kw)
        return wrapper

    for name in calls:
        monkeypatch.setattr(rccl_one_rank.dist, name, counted(name))
    got = dropin._run(False, fp16, modes, monkeypatch)
    # every step: a packed allgather per compressed tensor and an allgather per dense one
    # (the Average summed in rank order by dgc_rank_sum) — no allreduce, whose order is RCCL's
    dense = sum(1 for _, s in dropin.SHAPES if len(s) <= 1)
    assert calls["all_gather_into_tensor"] >= len(modes) * (1 + dense) and calls["all_reduce"] == 0, calls
    monkeypatch.setattr(rccl_one_rank, "ONE_RANK_SHORTCUT", True)
    want = dropin._run(False, fp16, modes, monkeypatch)
    for step, (w, g) in enumerate(zip(want, got)):
        assert w.keys() == g.keys()
        for k in w:
            assert w[k] is not None and g[k] is not None, (step, k)
            assert torch.equal(dropin._bits(w[k]), dropin._bits(g[k])), (step, k)


def _engine_steps(make, step, steps=5, seed=3):
    """Outputs of ``steps`` engine steps on seeded gradients (odd steps heavy-tailed:
    the adaptation loop and the resample run)."""
    eng = make()
    gen = torch.Generator(device=DEV).manual_seed(seed)
    res = []
    for s in range(steps):
        res.append(step(eng, s, gen).clone())
        torch.cuda.synchronize()
    return eng, res


@pytest.mark.timeout(300)
@pytest.mark.parametrize("parts", [1, 2], ids=["one-collective", "split-2"])
@pytest.mark.parametrize("fill", ["inline", "sparse"])
def test_bucket_over_rccl(fill, parts, rccl_one_rank, monkeypatch):
    """DGCBucket's exchange through RCCL (one allgather, or the split exchange's two
    part collectives with the compute stream waiting on each in turn) equals the
    one-rank step without a collective."""
    from dgc.bucket import DGCBucket
    comm = rccl_one_rank
    N = 3_000_017

    def grad(s, gen):
        g = torch.randn(N, generator=gen, device=DEV)
        return g * torch.rand(N, generator=gen, device=DEV).pow(8) * 50 if s % 2 else g

    def run(collective):
        monkeypatch.setattr(comm, "ONE_RANK_SHORTCUT", not collective)
        out = torch.zeros(N, device=DEV)

        def step(b, s, gen):
            b.step(grad(s, gen), out)
            return out
        b, res = _engine_steps(lambda: DGCBucket(N, compress_ratio=0.001, momentum=0.9, nesterov=True, device=DEV,
                                                 world_size=1, seed=42, fill=fill,
                                                 exchange_parts=parts if collective else 1), step)
        assert b.exchanging == collective and b.parts == (parts if collective else 1)
        return res

    got = run(True)
    want = run(False)
    for s, (w, g) in enumerate(zip(want, got)):
        assert torch.equal(w.view(torch.int32), g.view(torch.int32)), s


@pytest.mark.timeout(300)
@pytest.mark.parametrize("parts", [1, 2], ids=["one-collective", "split-2"])
@pytest.mark.parametrize("fill", ["inline", "sparse"])
def test_batch_over_rccl(fill, parts, rccl_one_rank, monkeypatch):
    """DGCBatch likewise (every tensor's entries in one payload, one exchange)."""
    from dgc.batch import DGCBatch
    comm = rccl_one_rank
    shapes = [("a", (1000, 300)), ("b", (257, 3, 3, 64)), ("c", (70001,)), ("d", (2000, 500))]

    def step(b, s, gen):
        for n in b.names:
            g = torch.randn(b.shapes[n], generator=gen, device=DEV) * 1e-3
            if s % 2:
                g = g * torch.rand(b.shapes[n], generator=gen, device=DEV).pow(8) * 50
            b.grad(n).copy_(g)
        b.compress()
        b.exchange()
        return b.decompress()

    def run(collective):
        monkeypatch.setattr(comm, "ONE_RANK_SHORTCUT", not collective)
        b, res = _engine_steps(lambda: DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, nesterov=False,
                                                device=DEV, world_size=1, seed=7, fill=fill,
                                                exchange_parts=parts if collective else 1), step)
        assert b.exchanging == collective and b.parts == (parts if collective else 1)
        return res

    got = run(True)
    want = run(False)
    for s, (w, g) in enumerate(zip(want, got)):
        assert torch.equal(w.view(torch.int32), g.view(torch.int32)), s


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fp16", [False, True], ids=["wire-dtype", "wire-fp16"])
@pytest.mark.parametrize("batch", [True, "sparse"], ids=["batch", "batch-sparse"])
def test_batched_optimizer_over_rccl(batch, fp16, rccl_one_rank, monkeypatch):
    """DistributedOptimizer(batch=True): ONE RCCL collective per step — the grouped
    payload allgather, the dense tensors' wire values in its tail — equals the one-rank
    step without it."""
    modes = ["fresh", "fresh", "inplace", "fresh"]
    calls = {"all_gather_into_tensor": 0, "all_reduce": 0}

    def counted(name):
        fn = getattr(dist, name)

        def wrapper(*a, **kw):
            calls[name] += 1
            return fn(*a, **kw)
        return wrapper

    for name in calls:
        monkeypatch.setattr(rccl_one_rank.dist, name, counted(name))
    got = dropin._run(batch, fp16, modes, monkeypatch)
    assert calls == {"all_gather_into_tensor": len(modes), "all_reduce": 0}, calls
    monkeypatch.setattr(rccl_one_rank, "ONE_RANK_SHORTCUT", True)
    want = dropin._run(batch, fp16, modes, monkeypatch)
    for step, (w, g) in enumerate(zip(want, got)):
        assert w.keys() == g.keys()
        for k in w:
            assert torch.equal(dropin._bits(w[k]), dropin._bits(g[k])), (step, k)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("parts", [1, 2], ids=["payload-tail", "split-own-allgather"])
@pytest.mark.parametrize("fp16", [False, True], ids=["wire-dtype", "wire-fp16"])
def test_batched_optimizer_dense_wire_bytes_over_rccl(parts, fp16, rccl_one_rank, monkeypatch):
    """batch="sparse" through RCCL: the dense tensors' wire values (compress's cast,
    dgc/compression.py:175-177) arrive byte for byte as dgc_gather_cast wrote them — in
    the gathered payload's tail at ``extra_off`` of every rank's ``rank_stride`` (one
    collective), or, when the exchange splits (DGC_EXCHANGE_PARTS=2), in their own
    allgather (``dense_gathered``) — and the weights equal the one-rank step without
    collectives (the re-zero's alternating gather buffers included)."""
    monkeypatch.setenv("DGC_EXCHANGE_PARTS", str(parts))
    wire = torch.float16 if fp16 else torch.float32
    checked = []

    def on_step(opt, grads):
        plan = opt._batched._plan
        b = plan["batch"]
        assert b.parts == parts and (b.extra_off is None) == (parts > 1)
        if parts > 1:
            rows = plan["dense_gathered"].view(1, -1)
        else:
            rows = b.gathered.view(1, b.rank_stride)[:, b.extra_off:]
        for n, p, off, _ in plan["dense"]:
            nb = p.numel() * torch.empty(0, dtype=wire).element_size()
            ob = off * torch.empty(0, dtype=wire).element_size()
            want = grads[n].reshape(-1).to(wire).view(torch.uint8)
            assert torch.equal(rows[0, ob: ob + nb], want), n
        checked.append(len(plan["dense"]))

    modes = ["fresh", "fresh", "inplace", "fresh", "fresh"]
    got = dropin._run("sparse", fp16, modes, monkeypatch, on_step=on_step)
    assert len(checked) == len(modes) and checked[0] > 0
    monkeypatch.setattr(rccl_one_rank, "ONE_RANK_SHORTCUT", True)
    want = dropin._run("sparse", fp16, modes, monkeypatch)
    for step, (w, g) in enumerate(zip(want, got)):
        for k in w:
            assert torch.equal(dropin._bits(w[k]), dropin._bits(g[k])), (step, k)
