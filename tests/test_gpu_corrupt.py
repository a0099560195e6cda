"""A foreign or corrupted payload raises, as the reference does.

The reference decompresses with ``grad.zero_().index_put_([indices], values,
accumulate=True)`` (/root/reference/dgc/compression.py:191) and masks with
``index_fill_`` (/root/reference/dgc/memory.py:76-77): an index outside the tensor
raises there. Its authors saw NCCL's allgather hand over "random data once in a while"
(/root/reference/README.md:132), so a gathered payload can be corrupted in transit. The
kernels here drop such an entry (and clamp a header count outside [0, capacity]) and
store a flag into the caller's pinned status words (``dgc_decompress_bind_sink``,
``bad_flag``); every engine and drop-in entry point reads those words at its next call
— no host synchronisation — and raises ``RuntimeError``.

Each test corrupts one payload between the selection and the decompress (one rank's run
of a W-rank gather for the multi-run paths) with: an index >= n, a negative index, a
count above the capacity, a negative count. A healthy step before and after must not
raise (a reported error is cleared).
"""
import ctypes
import random

import numpy as np
import pytest
import torch

import test_gpu_split as S

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
KINDS = ["index-past-n", "index-negative", "count-past-capacity", "count-negative"]


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def corrupt(run, kind, n, cap, ioff, idtype):
    """One rank's packed payload (a uint8 tensor view): its first index or its count."""
    if kind.startswith("count"):
        run[:8].view(torch.int64).fill_(cap + 3 if kind == "count-past-capacity" else -2)
        return
    ib = 4 if idtype == torch.int32 else 8
    run[ioff: ioff + ib].view(idtype).fill_(n + 5 if kind == "index-past-n" else -3)


def _match(kind):
    return "outside the gradient" if kind.startswith("index") else "count outside"


def _grads(n, gen):
    g = torch.randn(n, generator=gen, device=DEV)
    return g * torch.rand(n, generator=gen, device=DEV).pow(4)


# ---------------------------------------------------------------- engines
@pytest.mark.timeout(120)
@pytest.mark.parametrize("fill", ["inline", "sparse"])
@pytest.mark.parametrize("kind", KINDS)
def test_bucket_raises_on_corrupt_payload(kind, fill):
    _need_gpu()
    from dgc.bucket import DGCBucket
    N = 2_000_003
    b = DGCBucket(N, compress_ratio=0.001, device=DEV, fill=fill, seed=5)
    out = torch.zeros(N, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(11)
    for _ in range(2):
        b.step(_grads(N, gen), out)
    b.status.check(sync=True)   # healthy: nothing raised
    real = b.exchange

    def bad_exchange():   # W = 1: the gathered buffer is the payload itself
        corrupt(b.gathered, kind, N, b.k, b.ioff, b.idtype)
        real()
    b.exchange = bad_exchange
    b.step(_grads(N, gen), out)
    b.exchange = real
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match=_match(kind)):
        b.step(_grads(N, gen), out)   # the next step's first check, before any launch
    for _ in range(2):   # reported once, then the engine runs on
        b.step(_grads(N, gen), out)
    b.status.check(sync=True)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
@pytest.mark.parametrize("kind", KINDS)
def test_batch_raises_on_corrupt_payload(kind, dtype):
    _need_gpu()
    from dgc.batch import DGCBatch
    shapes = [("conv", (256, 128, 3, 3)), ("fc", (1000, 512)), ("small", (64, 27))]
    b = DGCBatch(shapes, compress_ratio=0.001, device=DEV, seed=3, dtype=dtype)
    gen = torch.Generator(device=DEV).manual_seed(5)

    def step(bad=None):
        b.grad_flat.copy_(_grads(b.flat_numel, gen).to(dtype))
        b.compress()
        if bad:
            corrupt(b.payload, bad, b.flat_numel, b.capacity, b.ioff, b.idtype)
        b.exchange()
        b.decompress()

    step()
    b.infos()   # syncs and checks: healthy
    step(kind)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match=_match(kind)):
        step()
    step()
    b.infos()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind", ["index-past-n", "count-past-capacity"])
def test_batched_optimizer_raises_on_corrupt_payload(kind, monkeypatch):
    """DistributedOptimizer(batch=True) at W = 1 (HOROVOD_ELASTIC=1 registers the hooks,
    dgc/horovod/optimizer.py:79-80): the payload corrupted as it is sent; the next
    step() raises."""
    _need_gpu()
    from dgc.compression import DGCCompressor
    from dgc.horovod import DistributedOptimizer
    from dgc.memory import DGCSGDMemory
    monkeypatch.setenv("HOROVOD_ELASTIC", "1")
    torch.manual_seed(0)
    random.seed(0)
    model = torch.nn.Linear(2000, 1000).to(DEV)
    comp = DGCCompressor(0.01, memory=DGCSGDMemory(momentum=0.9))
    comp.memory.initialize(model.named_parameters())
    comp.initialize([(n, p) for n, p in model.named_parameters() if p.dim() > 1])
    opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1),
                               named_parameters=model.named_parameters(), compression=comp, batch=True)

    def step():
        opt.zero_grad()
        model.weight.grad = torch.randn(1000, 2000, device=DEV)
        model.bias.grad = torch.randn(1000, device=DEV)
        for _, hook in reversed(opt._hook_fns):
            hook()
        opt.step()

    step()
    b = opt._batched._plan["batch"]
    real = b.send

    def bad_send():
        corrupt(b.payload, kind, b.flat_numel, b.capacity, b.ioff, b.idtype)
        real()
    b.send = bad_send
    step()
    b.send = real
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match=_match(kind)):
        step()
    step()
    b.status.check(sync=True)


# ---------------------------------------------------------------- drop-in, per tensor
def _compressor(numel=400_000, dtype=torch.float32):
    from dgc.compression import DGCCompressor
    from dgc.memory import DGCSGDMemory
    p = torch.zeros(numel, device=DEV, dtype=dtype)
    comp = DGCCompressor(0.01, memory=DGCSGDMemory(momentum=0.9))
    comp.memory.initialize([("w", p)])
    comp.initialize([("w", p)])
    return comp


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind", KINDS)
def test_compressor_packed_path_raises(kind):
    """compress -> communicate -> synchronize -> decompress (the hook path): a count
    outside [0, capacity] raises in synchronize (it reads the headers on the host); a bad
    index raises at the next call after the decompress."""
    _need_gpu()
    from dgc.comm import Average
    comp = _compressor()
    g = torch.randn(400_000, device=DEV)
    (vals, idx), ctx = comp.compress(g, "w")
    payload, lay = comp._payloads["w"]
    corrupt(payload, kind, 400_000, lay[0], lay[5], lay[2])   # as if corrupted on the wire
    h = comp.communicate((vals, idx), "w", Average)
    if kind.startswith("count"):
        with pytest.raises(RuntimeError, match="outside"):
            comp.synchronize(h)
        return
    gathered = comp.synchronize(h)
    comp.decompress(gathered, ctx)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="outside the gradient"):
        comp.compress(torch.randn(400_000, device=DEV), "w")
    comp.compress(torch.randn(400_000, device=DEV), "w")   # reported once


@pytest.mark.timeout(120)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_compressor_list_path_wraps_negative_and_raises_past_n(dtype):
    """decompress((values, indices), ctx) in the reference's list form: index_put_ wraps
    an index in [-n, 0) (the result must equal torch's on CPU) and raises past n."""
    _need_gpu()
    n = 1000
    comp = _compressor(n, dtype)
    grad = torch.zeros(n, device=DEV, dtype=dtype)
    ctx = ("w", n, [n], dtype, torch.int64, grad)
    vals = torch.tensor([[1.5], [2.25], [-4.0]], device=DEV, dtype=dtype)
    idx = torch.tensor([[3], [-1], [-n]], device=DEV)
    out = comp.decompress([vals, idx], ctx)
    want = torch.zeros(n, dtype=dtype).index_put_([idx.cpu().view(-1)], vals.cpu().view(-1), accumulate=True)
    assert torch.equal(out.cpu().view(torch.int16 if dtype != torch.float32 else torch.int32),
                       want.view(torch.int16 if dtype != torch.float32 else torch.int32))
    comp.check(sync=True)
    comp.decompress([vals, torch.tensor([[3], [n], [5]], device=DEV)], ctx)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="outside the gradient"):
        comp.decompress([vals, idx], ctx)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16], ids=["fp32", "fp16"])
def test_memory_update_raises_past_n(dtype):
    """DGCSGDMemory.update: index_fill_ wraps [-n, 0) and raises outside [-n, n)."""
    _need_gpu()
    from dgc.memory import DGCSGDMemory
    n = 5000
    mem = DGCSGDMemory(momentum=0.9)
    mem.initialize([("w", torch.zeros(n, device=DEV, dtype=dtype))])
    mem.compensate(torch.ones(n, device=DEV, dtype=dtype), "w")
    mem.update("w", (torch.tensor([0, -1], device=DEV),))
    mem.check(sync=True)
    v = mem.velocities["w"].cpu()
    assert v[0] == 0 and v[n - 1] == 0 and v[1] != 0
    mem.update("w", (torch.tensor([7, n + 1], device=DEV),))
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="DGCSGDMemory.update"):
        mem.compensate(torch.ones(n, device=DEV, dtype=dtype), "w")
    mem.compensate(torch.ones(n, device=DEV, dtype=dtype), "w")


# ---------------------------------------------------------------- the C ABI, multi-run
@pytest.mark.timeout(120)
@pytest.mark.parametrize("form", ["dense", "over", "scatter"])
@pytest.mark.parametrize("kind", KINDS)
def test_packed_multi_rank_sink(kind, form):
    """dgc_decompress_packed / _over / dgc_scatter_packed over W = 3 ranks' payloads,
    rank 1's corrupted (the multi-run bounds path): the status word's bit and the bound
    sink's word are set; healthy payloads set neither."""
    _need_gpu()
    from dgc import _lib
    L = _lib.lib()
    N, W, cap = 1_000_003, 3, 2000
    rng = np.random.default_rng(7)
    runs = S._runs(rng, N, W, cap, 0.3, 0)
    vo, io = ctypes.c_int64(0), ctypes.c_int64(0)
    stride = L.dgc_payload_layout(cap, 0, 0, ctypes.byref(vo), ctypes.byref(io))
    pays = [S._rank_payload(L, v, i, cap, 0, 0) for v, i in runs]
    good = torch.cat(pays)
    bad = good.clone()
    corrupt(bad[stride: 2 * stride], kind, N, cap, io.value, torch.int64)
    wsz = L.dgc_decompress_packed_workspace(N, W, cap)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    sink = _lib.StatusSink("abi", DEV)
    sink.bind(ws)
    out = torch.zeros(N, device=DEV)

    def call(p):
        args = (W, stride, cap, 0, 0, S.P(out), N, 1.0 / W, S.P(ws), wsz, S.stream())
        if form == "dense":
            S.check(L, L.dgc_decompress_packed(S.P(p), *args))
        elif form == "scatter":
            S.check(L, L.dgc_fill_zero(S.P(out), N, S.stream()))
            S.check(L, L.dgc_scatter_packed(S.P(p), *args))
        else:
            S.check(L, L.dgc_decompress_packed(S.P(good), *args))
            S.check(L, L.dgc_decompress_packed_over(S.P(p), S.P(good.clone()), *args))
        st = ctypes.c_int32(-1)
        S.check(L, L.dgc_decompress_status(S.P(ws), ctypes.byref(st), S.stream()))
        return st.value

    assert call(good) & 5 == 0
    sink.check()
    st = call(bad)
    assert st & (1 if kind.startswith("index") else 4), st
    with pytest.raises(RuntimeError, match=_match(kind)):
        sink.check()
    assert call(good) & 5 == 0   # the status word is per call
    sink.check()
    S.check(L, L.dgc_decompress_bind_sink(S.P(ws), None))   # unbound: the words stay clear
    call(bad)
    sink.check()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind", KINDS)
def test_split_scatter_sink(kind):
    """The split exchange's phase scatters (dgc_scatter_split): rank 1's part-0 buffer
    corrupted as it landed."""
    _need_gpu()
    from dgc import _lib
    L = _lib.lib()
    N, W, parts, cap = 1_000_003, 2, 2, 3000
    runs = S._runs(np.random.default_rng(3), N, W, cap, 0.3, 0)
    sp = S.Split(L, N, W, parts, cap, 0, 0)
    g, _ = sp.gather(runs)
    sink = _lib.StatusSink("split", DEV)
    sink.bind(sp.ws)
    out = torch.zeros(N, device=DEV)
    sp.scatter(g, out, False)
    torch.cuda.synchronize()
    sink.check()
    io = ctypes.c_int64(0)
    L.dgc_payload_split_layout(cap, parts, 0, 0, None)
    vo = ctypes.c_int64(0)
    L.dgc_payload_layout(sp.pc, 0, 0, ctypes.byref(vo), ctypes.byref(io))
    corrupt(g[sp.pbytes: 2 * sp.pbytes], kind, N, sp.pc, io.value, torch.int64)   # part 0 of rank 1
    S.check(L, L.dgc_fill_zero(S.P(out), N, S.stream()))
    sp.scatter(g, out, False)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match=_match(kind)):
        sink.check()
