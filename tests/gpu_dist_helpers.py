"""Workers of the multi-rank GPU tests (tests/test_gpu_multirank.py): 2 processes on
cuda:0 over gloo, running the PRODUCT path — DGCSGDMemory / DGCCompressor /
DistributedOptimizer / DGCSGD / DGCBucket through libdgc_hip.so — with the exchange
staged through the host by ``dgc.comm`` (gloo moves host tensors). No oracle double
is involved: the oracle only checks.

The optimizer replays use the reference's own per-step gradients and hook order
(tests/golden/optimizer_trace.*, recorded from the reference run that produced
optimizer.npz / optimizer_resnet20.*): a chain of autograd nodes hands each parameter
its recorded gradient, in the recorded order, so the product DistributedOptimizer's
grad-accumulator hooks fire exactly as the reference's did (same compress order, same
``random.randint`` draws), then ``step()`` runs synchronize -> decompress -> DGCSGD.
"""
import contextlib
import hashlib
import io
import json
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (REPO, os.path.join(REPO, "adam-compression_amd"), HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

GOLDEN = os.path.join(HERE, "golden")


class _Feed(torch.autograd.Function):
    """x -> x; backward hands ``g`` to ``p``. Chained, the last one created runs first,
    and each parameter's AccumulateGrad (and so its DistributedOptimizer hook) runs as
    soon as its Feed has (AccumulateGrad nodes have the top scheduling priority)."""

    @staticmethod
    def forward(ctx, x, p, g):
        ctx.g = g
        return x.clone()

    @staticmethod
    def backward(ctx, gx):
        return gx, ctx.g, None


def replay_backward(params, order, grads, dev):
    x = torch.zeros((), device=dev)
    for name, g in reversed(list(zip(order, grads))):
        x = _Feed.apply(x, params[name], torch.from_numpy(np.ascontiguousarray(g)).to(dev))
    x.backward()


def _digest(model):
    h = hashlib.sha256()
    for _, p in model.named_parameters():
        h.update(p.detach().cpu().numpy().tobytes())
    return h.hexdigest()


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _load_cfg(label):
    if label == "tinynet":
        cfg = json.load(open(os.path.join(GOLDEN, "optimizer.json")))
        schedule = [(None, s) for s in range(cfg["steps"])]
    else:
        cfg = json.load(open(os.path.join(GOLDEN, "optimizer_resnet20.json")))
        spe = cfg["steps_per_epoch"]
        schedule = [(e if t == 0 else None, ei * spe + t) for ei, e in enumerate(cfg["epochs"]) for t in range(spe)]
    return cfg, schedule


def _setup(label, batch, dev, cfg, model_seed=None):
    """The reference's training objects for a replay: model, DGCSGD, DGCSGDMemory,
    DGCCompressor (initialised on the dim > 1 parameters, train.py:130-140) and the
    DistributedOptimizer around them, plus a spy on compress (the per-tensor calls)."""
    from dgc.comm import Average
    from dgc.compression import DGCCompressor
    from dgc.horovod import DistributedOptimizer
    from dgc.memory import DGCSGDMemory
    from dgc.optim import DGCSGD
    from models import ResNet20, TinyNet
    torch.manual_seed(cfg["model_seed"] if model_seed is None else model_seed)
    if label == "tinynet":
        model = TinyNet().to(dev)
        comp_kw = dict(fp16_values=False, int32_indices=False, warmup_epochs=-1)
    else:
        model = ResNet20().to(dev)
        comp_kw = dict(sample_ratio=cfg["sample_ratio"], fp16_values=cfg["fp16_values"],
                       int32_indices=cfg["int32_indices"], warmup_epochs=cfg["warmup_epochs"])
    opt = DGCSGD(model.parameters(), lr=cfg["lr"], momentum=cfg["momentum"],
                 weight_decay=cfg["weight_decay"], nesterov=cfg["nesterov_sgd"])
    mem = DGCSGDMemory(momentum=cfg["momentum"])
    with contextlib.redirect_stdout(io.StringIO()):
        comp = DGCCompressor(cfg["ratio"], memory=mem, **comp_kw)
        mem.initialize(model.named_parameters())
        comp.initialize([(n, p) for n, p in model.named_parameters() if p.dim() > 1])
    if batch == "default":   # no batch= argument: the drop-in default ("auto") must pick the batched step
        dopt = DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                    backward_passes_per_step=1, op=Average)
        assert dopt._batched is not None, "DistributedOptimizer's default did not take the batched step"
    else:
        dopt = DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                    backward_passes_per_step=1, op=Average, batch=batch)
    calls = []
    orig = comp.compress

    def spy(tensor, name):
        calls.append(name)
        return orig(tensor, name)

    comp.compress = spy
    return dict(model=model, opt=opt, mem=mem, comp=comp, dopt=dopt, params=dict(model.named_parameters()),
                calls=calls)


def _replay_step(run, label, batch, rank, epoch, s, meta, trace, dev, problems, zero_grad=None):
    """One training step of the reference's run: warmup ratio at an epoch start, the
    recorded backward (hooks fire in the recorded order), step, zero_grad."""
    if epoch is not None:
        with contextlib.redirect_stdout(io.StringIO()):
            run["comp"].warmup_compress_ratio(epoch)
    key = f"{label}/s{s}/r{rank}"
    order = meta[key]
    grads = [trace[f"{key}/{j}"] for j in range(len(order))]
    run["calls"].clear()
    replay_backward(run["params"], order, grads, dev)
    dopt = run["dopt"]
    if (list(dopt._order) if batch else run["calls"]) != order:
        problems.append(("hook order", s))
    if batch and run["calls"]:
        problems.append(("per-tensor compress in batch mode", s))
    dopt.step()
    if zero_grad is None:
        dopt.zero_grad()    # torch >= 2 default: set_to_none=True
    else:
        dopt.zero_grad(set_to_none=zero_grad)
    torch.cuda.synchronize()


def _check_weights(run, label, cfg, want, s, rank, problems, tag="weights"):
    model = run["model"]
    if label == "tinynet":
        for n, p in model.named_parameters():
            w = want[f"s{s}/r{rank}/{n}"]
            got = p.detach().cpu().numpy()
            if not np.array_equal(got.view(np.uint32), w.view(np.uint32)):
                problems.append((tag, s, n, float(np.abs(got - w).max())))
    elif _digest(model) != cfg["step_digests"][s][rank]:
        problems.append((tag + " digest", s))


def _check_final(run, label, want, problems):
    if label != "resnet20":
        return
    for n, p in run["model"].named_parameters():
        got = p.detach().cpu().numpy()
        w = want[f"final/{n}"]
        if not np.array_equal(got.view(np.uint32), w.view(np.uint32)):
            problems.append(("final", n, float(np.abs(got - w).max())))


def _want(label):
    return np.load(os.path.join(GOLDEN, "optimizer.npz" if label == "tinynet" else "optimizer_resnet20.npz"))


def optimizer_replay_worker(rank, world, port, label, batch, queue):
    """label "tinynet": optimizer.npz (3 steps, nesterov DGCSGD, fp32/int64, ratio 0.01);
    label "resnet20": BASELINE configs[0] (ResNet-20, ratio 0.001 with the 5-epoch warmup
    0.316 -> 0.1 -> 0.001 re-initialising mid-run, fp16 values, int32 indices).
    batch: DistributedOptimizer(batch=True) — one grouped exchange per step."""
    import torch.distributed as dist
    _init(rank, world, port)
    problems = []
    try:
        dev = torch.device("cuda:0")
        meta = json.load(open(os.path.join(GOLDEN, "optimizer_trace.json")))
        trace = np.load(os.path.join(GOLDEN, "optimizer_trace.npz"))
        cfg, schedule = _load_cfg(label)
        want = _want(label)
        run = _setup(label, batch, dev, cfg)
        if label == "resnet20" and _digest(run["model"]) != cfg["init_digest"]:
            problems.append(("init", "digest"))
        random.seed(cfg["random_seed"])
        for epoch, s in schedule:
            _replay_step(run, label, batch, rank, epoch, s, meta, trace, dev, problems)
            _check_weights(run, label, cfg, want, s, rank, problems)
        _check_final(run, label, want, problems)
        queue.put((rank, problems))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        queue.put((rank, [("error", repr(e), traceback.format_exc())]))
    finally:
        dist.destroy_process_group()


def _checkpoint(run):
    """train.py:244-253's checkpoint — model, optimizer and compression.memory state
    dicts — through torch.save into memory (a copy of every tensor, as on disk)."""
    buf = io.BytesIO()
    torch.save({"model": run["model"].state_dict(), "optimizer": run["dopt"].state_dict(),
                "compression": run["mem"].state_dict()}, buf)
    buf.seek(0)
    return buf


def _restore(run, buf, dev):
    """train.py:153-165's resume: load_state_dict of model, optimizer and memory."""
    ck = torch.load(buf, map_location=dev, weights_only=True)
    run["model"].load_state_dict(ck["model"])
    run["dopt"].load_state_dict(ck["optimizer"])
    run["mem"].load_state_dict(ck["compression"])


def resume_worker(rank, world, port, label, batch, mode, resume_at, queue):
    """Checkpoint / resume parity (train.py:153-165, 244-264;
    dgc/memory.py:79-88): run the reference's replay to the epoch boundary
    ``resume_at``, checkpoint model + optimizer + memory, then
      mode "fresh":   build NEW objects (another model init), load the checkpoint, go on;
      mode "inplace": run one more step (the state moves on), load the checkpoint into
                      the SAME objects — the memory's tensors are replaced, so the
                      batched step must copy them back into its flat layout — and go on.
    Python's ``random`` state is carried with the checkpoint (the sample starts of an
    uninterrupted run). The weights after every later step must equal the reference's
    (the goldens), which the uninterrupted run also reproduces. In batch mode every other
    step zeroes with set_to_none=False (the views stay bound), the rest with None."""
    import torch.distributed as dist
    _init(rank, world, port)
    problems = []
    try:
        dev = torch.device("cuda:0")
        meta = json.load(open(os.path.join(GOLDEN, "optimizer_trace.json")))
        trace = np.load(os.path.join(GOLDEN, "optimizer_trace.npz"))
        cfg, schedule = _load_cfg(label)
        want = _want(label)
        run = _setup(label, batch, dev, cfg)
        random.seed(cfg["random_seed"])
        zg = lambda s: (s % 2 == 1) if batch else None   # noqa: E731
        for epoch, s in schedule[:resume_at]:
            _replay_step(run, label, batch, rank, epoch, s, meta, trace, dev, problems, zero_grad=zg(s))
            _check_weights(run, label, cfg, want, s, rank, problems)
        buf = _checkpoint(run)
        rstate = random.getstate()
        if mode == "fresh":
            run = _setup(label, batch, dev, cfg, model_seed=cfg["model_seed"] + 1000)
        else:
            epoch, s = schedule[resume_at]
            _replay_step(run, label, batch, rank, epoch, s, meta, trace, dev, problems, zero_grad=zg(s))
        _restore(run, buf, dev)
        random.setstate(rstate)
        for epoch, s in schedule[resume_at:]:
            _replay_step(run, label, batch, rank, epoch, s, meta, trace, dev, problems, zero_grad=zg(s))
            _check_weights(run, label, cfg, want, s, rank, problems, tag="resumed weights")
        _check_final(run, label, want, problems)
        queue.put((rank, problems))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        queue.put((rank, [("error", repr(e), traceback.format_exc())]))
    finally:
        dist.destroy_process_group()


def bucket_worker(rank, world, port, fill, kind, *rest):   # rest: ([parts,] queue)
    """DGCBucket at W=2 (fixed-capacity packed payload, allgather, sparse or dense
    decompress) against the oracle over both ranks' payloads, step by step."""
    parts, queue = rest if len(rest) == 2 else ("auto",) + rest
    import torch.distributed as dist
    _init(rank, world, port)
    problems = []
    try:
        from dgc.bucket import DGCBucket
        from oracle import dgc_oracle as O
        from oracle import synth
        dev = torch.device("cuda:0")
        N, ratio = 3_000_017, 0.001
        b = DGCBucket(N, compress_ratio=ratio, momentum=0.9, nesterov=True, device=dev, world_size=world,
                      seed=42, fill=fill, exchange_parts=parts)
        if parts != "auto" and b.parts != parts:
            problems.append(("parts", b.parts))
        attrs = O.attributes(N, ratio)
        state = [(np.zeros(N, np.float32), np.zeros(N, np.float32)) for _ in range(world)]
        rng = random.Random(42)
        out = torch.full((N,), float("nan"), device=dev)
        branches = []
        for s in range(5):
            gs = [synth.gradient(100 * s + q, N, kind) for q in range(world)]
            start = rng.randint(0, attrs[4] - 1)
            b.step(torch.from_numpy(gs[rank]).to(dev), out)
            torch.cuda.synchronize()
            vals, idxs = [], []
            for q in range(world):
                m, v = state[q]
                ov, oi, info = O.compress_step(gs[q], m, v, attrs, start, nesterov=True)
                vals.append(ov)
                idxs.append(oi)
                if q == rank:
                    branches.append(info["branch"])
                    if s % 2 == 1 and not (   # reading flushes the deferred masking: odd steps only
                            np.array_equal(b.vec.cpu().numpy().view(np.uint32), v.view(np.uint32)) and
                            np.array_equal(b.mmt.cpu().numpy().view(np.uint32), m.view(np.uint32))):
                        problems.append(("state", s))
                    n = b.last_info()["count"]
                    pi = b.payload[b.ioff: b.ioff + 8 * n].view(torch.int64).cpu().numpy()
                    if not np.array_equal(pi, oi):
                        problems.append(("indices", s, info["branch"]))
            want = O.decompress(vals, idxs, N, world)
            if not np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32)):
                problems.append(("decompress", s, branches[-1]))
        queue.put((rank, problems + [("branches", branches)]))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        queue.put((rank, [("error", repr(e), traceback.format_exc())]))
    finally:
        dist.destroy_process_group()


def batch_worker(rank, world, port, fill, kind, *rest):   # rest: ([parts,] queue)
    """DGCBatch at W ranks (one packed payload of every tensor, allgather, decompress
    into the batch's persistent output — fill "sparse" re-zeroes only the previous
    step's gathered indices) against the oracle over all ranks' payloads, per tensor
    and step."""
    parts, queue = rest if len(rest) == 2 else ("auto",) + rest
    import torch.distributed as dist
    _init(rank, world, port)
    problems = []
    try:
        from dgc.batch import DGCBatch
        from oracle import dgc_oracle as O
        from oracle import synth
        dev = torch.device("cuda:0")
        shapes = [("a", (1000, 300)), ("b", (257, 3, 3, 64)), ("c", (70001,)), ("d", (2000, 500))]
        ratio = 0.001
        b = DGCBatch(shapes, compress_ratio=ratio, momentum=0.9, nesterov=False, device=dev, world_size=world,
                     seed=7, fill=fill, exchange_parts=parts)
        if parts != "auto" and b.parts != parts:
            problems.append(("parts", b.parts))
        state = {(q, n): (np.zeros(b.numels[i], np.float32), np.zeros(b.numels[i], np.float32))
                 for q in range(world) for i, n in enumerate(b.names)}
        branches = []
        for s in range(5):
            gs = {(q, n): synth.gradient(1000 * s + 10 * i + q, b.numels[i], kind, 1e-3)
                  for q in range(world) for i, n in enumerate(b.names)}
            for n in b.names:
                b.grad(n).copy_(torch.from_numpy(gs[(rank, n)]).view(b.shapes[n]))
            b.compress()
            b.exchange()
            b.decompress()
            torch.cuda.synchronize()
            for i, n in enumerate(b.names):
                attrs = O.attributes(b.numels[i], ratio)
                vals, idxs = [], []
                for q in range(world):
                    m, v = state[(q, n)]
                    ov, oi, info = O.compress_step(gs[(q, n)], m, v, attrs, b.starts[i])
                    vals.append(ov)
                    idxs.append(oi)
                    if q == rank:
                        branches.append(info["branch"])
                want = O.decompress(vals, idxs, b.numels[i], world)
                got = b.out(n).reshape(-1).cpu().numpy()
                if not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                    problems.append(("decompress", s, n, branches[-1]))
        queue.put((rank, problems + [("branches", branches)]))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        queue.put((rank, [("error", repr(e), traceback.format_exc())]))
    finally:
        dist.destroy_process_group()


def half_worker(rank, world, port, case_name, queue):
    """A 16-bit golden case (tests/golden/half.*) at its own world size over gloo: each
    rank compresses its own gradient (DGCSGDMemory / DGCCompressor on bf16 / fp16),
    communicate -> synchronize (the packed allgather) -> decompress; the payload, the
    16-bit state and the decompressed gradient must equal the reference's."""
    _init(rank, world, port)
    problems = []
    try:
        from dgc.compression import DGCCompressor
        from dgc.memory import DGCSGDMemory
        from dgc.comm import Average
        from oracle import synth
        with open(os.path.join(GOLDEN, "half.json")) as f:
            case = json.load(f)[case_name]
        arrays = np.load(os.path.join(GOLDEN, "half.npz"))
        assert case["W"] == world
        dt = getattr(torch, case["dtype"])
        dev = torch.device("cuda:0")
        N = case["N"]
        mem = DGCSGDMemory(momentum=0.9, nesterov=case["nesterov"], momentum_masking=case["masking"])
        with contextlib.redirect_stdout(io.StringIO()):
            comp = DGCCompressor(case["ratio"], memory=mem, fp16_values=case["fp16"], int32_indices=case["int32"],
                                 resample=case["resample"])
            prm = torch.zeros(N, dtype=dt, device=dev)
            mem.initialize([("w", prm)])
            comp.initialize([("w", prm)])
        random.seed(42)
        for s, step in enumerate(case["per_step"]):
            rk = step["ranks"][rank]
            g = torch.from_numpy(synth.gradient(rk["seed"], N, case["kind"], case["scale"]).copy()).to(dt).to(dev)
            (vals, idx), ctx = comp.compress(g, "w")
            key = f"{case_name}/s{s}/r{rank}"
            if not np.array_equal(idx.view(-1).cpu().numpy(), arrays[key + "/indices"]):
                problems.append((s, "indices"))
            if not np.array_equal(vals.view(-1).float().cpu().numpy().view(np.uint32),
                                  arrays[key + "/values"].view(np.uint32)):
                problems.append((s, "values"))
            h = comp.communicate((vals, idx), "w", Average)
            out = comp.decompress(comp.synchronize(h), ctx)
            want = np.zeros(N, np.float32)
            nz = arrays[f"{case_name}/s{s}/dec_nz_idx"]
            want[nz] = arrays[f"{case_name}/s{s}/dec_nz_val"]
            got = out.view(-1).float().cpu().numpy()
            if out.dtype != dt or not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                problems.append((s, "decompress"))
            if synth.digest(mem.velocities["w"].float().cpu().numpy()) != rk["vec_sha"]:
                problems.append((s, "vec"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        problems.append(("exception", traceback.format_exc()[-600:]))
    queue.put((rank, problems))


HALF_SHAPES = [("conv.weight", (64, 3, 7, 7)), ("bn.weight", (64,)), ("bn.bias", (64,)), ("odd.weight", (333, 7)),
               ("fc.weight", (1000, 512)), ("fc.bias", (1000,))]


def _half_run(batch, dtype, fp16, rank, dev, steps=4):
    from dgc.compression import DGCCompressor
    from dgc.horovod import DistributedOptimizer
    from dgc.memory import DGCSGDMemory
    named = [(n, torch.nn.Parameter(torch.zeros(s, device=dev, dtype=dtype))) for n, s in HALF_SHAPES]
    with contextlib.redirect_stdout(io.StringIO()):
        comp = DGCCompressor(0.01, memory=DGCSGDMemory(momentum=0.9), fp16_values=fp16, int32_indices=fp16)
        comp.memory.initialize(named)
        comp.initialize([(n, p) for n, p in named if p.dim() > 1])
    from dgc.optim import DGCSGD
    # the wrapped optimizer is DGCSGD: its 16-bit step is the fused K7-16 (dgc_sgd_step16)
    dopt = DistributedOptimizer(DGCSGD([p for _, p in named], lr=0.1, momentum=0.9, weight_decay=1e-4,
                                       nesterov=True), named_parameters=named, compression=comp, batch=batch)
    random.seed(5)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    out = []
    for s in range(steps):
        for i, (n, p) in enumerate(named):
            g = torch.randn(p.shape, generator=gen, device=dev) * (1e-3 * (1 + i))
            if s % 2:   # heavy-tailed: the adaptation loop and the resample run
                g = g * torch.rand(p.shape, generator=gen, device=dev).pow(8) * 50
            p.grad = g.to(dtype)
        for _, hook in reversed(dopt._hook_fns):
            hook()
        dopt.step()   # synchronize() (compress -> exchange -> decompress) + DGCSGD's fused 16-bit step
        torch.cuda.synchronize()
        st = comp.memory.state_dict()
        out.append({n: p.grad.clone() for n, p in named} | {f"m:{n}": t.clone() for n, t in st["momentums"].items()}
                   | {f"v:{n}": t.clone() for n, t in st["velocities"].items()}
                   | {f"p:{n}": p.detach().clone() for n, p in named})
        dopt.zero_grad()
    return out


def half_batch_worker(rank, world, port, dtype_name, fp16, q):
    """W ranks: DistributedOptimizer(batch=True) on bf16 / fp16 parameters (the 16-bit
    batch engine, one packed allgather, the 16-bit decompress and dense allreduce) equals
    the per-tensor path (pinned to the reference's 16-bit fixtures) bit for bit."""
    _init(rank, world, port)
    dev = torch.device("cuda:0")
    dtype = getattr(torch, dtype_name)
    want = _half_run(False, dtype, fp16, rank, dev)
    got = _half_run(True, dtype, fp16, rank, dev)
    problems = []
    for s, (w, g) in enumerate(zip(want, got)):
        for k in w:
            if not torch.equal(w[k].view(torch.int16), g[k].view(torch.int16)):
                problems.append((s, k))
    q.put((rank, problems))
    import torch.distributed as dist
    dist.destroy_process_group()


def multi_replay_worker(rank, world, port, label, batch, queue):
    """tests/golden/optimizer_multi.* case ``label`` at its own world size W (3, 4 or 8
    processes on cuda:0 over gloo): the reference's DistributedOptimizer + DGCSGD run on
    TinyNet, replayed from its recorded per-rank gradients and hook order through the
    product path — per tensor, or batch=True (dense wire values in the packed payload's
    tail, ONE allgather per step) — must reach the reference's weights bit for bit after
    every step. The dense tensors' Average is where W >= 3 can differ: the reference
    (restated) sums the ranks in rank order in the wire dtype (fp16 for fp16_values)."""
    import torch.distributed as dist
    _init(rank, world, port)
    problems = []
    try:
        from dgc.comm import Average
        from dgc.compression import DGCCompressor
        from dgc.horovod import DistributedOptimizer
        from dgc.memory import DGCSGDMemory
        from dgc.optim import DGCSGD
        from models import TinyNet
        meta = json.load(open(os.path.join(GOLDEN, "optimizer_multi.json")))
        arrays = np.load(os.path.join(GOLDEN, "optimizer_multi.npz"))
        cfg = meta[label]
        assert cfg["W"] == world, (cfg["W"], world)
        dev = torch.device("cuda:0")
        torch.manual_seed(cfg["model_seed"])
        model = TinyNet().to(dev)
        opt = DGCSGD(model.parameters(), lr=cfg["lr"], momentum=cfg["momentum"], weight_decay=cfg["weight_decay"],
                     nesterov=cfg["nesterov_sgd"])
        mem = DGCSGDMemory(momentum=cfg["momentum"])
        with contextlib.redirect_stdout(io.StringIO()):
            comp = DGCCompressor(cfg["ratio"], memory=mem, fp16_values=cfg["fp16_values"],
                                 int32_indices=cfg["int32_indices"], **cfg["warmup"])
            mem.initialize(model.named_parameters())
            comp.initialize([(n, p) for n, p in model.named_parameters() if p.dim() > 1])
        dopt = DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                    backward_passes_per_step=1, op=Average, batch=batch)
        params = dict(model.named_parameters())
        spe = cfg["steps_per_epoch"]
        schedule = [(e if t == 0 else None, ei * spe + t) for ei, e in enumerate(cfg["epochs"]) for t in range(spe)]
        random.seed(cfg["random_seed"])
        for epoch, s in schedule:
            if epoch is not None:
                with contextlib.redirect_stdout(io.StringIO()):
                    comp.warmup_compress_ratio(epoch)
            key = f"{label}/s{s}/r{rank}"
            order = meta[key]
            grads = [arrays[f"{key}/{j}"] for j in range(len(order))]
            replay_backward(params, order, grads, dev)
            dopt.step()
            dopt.zero_grad()
            torch.cuda.synchronize()
            for n, p in model.named_parameters():
                w = arrays[f"{label}/s{s}/{n}"]
                got = p.detach().cpu().numpy()
                if not np.array_equal(got.view(np.uint32), w.view(np.uint32)):
                    problems.append(("weights", s, n, int((got != w).sum()), float(np.abs(got - w).max())))
        queue.put((rank, problems))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        queue.put((rank, [("error", repr(e), traceback.format_exc())]))
    finally:
        dist.destroy_process_group()
