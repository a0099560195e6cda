#!/usr/bin/env python3
"""Generate the golden fixtures in ``tests/golden/`` from the REFERENCE itself.

Runs ONLY in the build container, where the reference is mounted read-only at
``/root/reference``. It imports the reference's own ``dgc.memory``,
``dgc.compression``, ``dgc.horovod`` and ``dgc.optim`` modules on CPU PyTorch with
an in-file stub for ``horovod.torch`` (Horovod is not installed; its allgather is
restated as "concatenate along dim 0 in rank order", its allreduce Average as
"sum in rank order, then divide by the size"), and records inputs/outputs as
small ``.npz``/``.json`` fixtures. Nothing from the reference is copied into the
fixtures except computed values. ``torch.set_num_threads(1)`` makes the CPU
``index_put_(accumulate=True)`` order sequential (multi-threaded CPU
``index_put_`` is run-to-run nondeterministic).

Inputs are not stored: they are regenerated from ``oracle/synth.py`` seeds, and
the fixture stores each input's SHA-256 so that a generator drift is detected.

Usage:  python tests/golden/make_goldens.py
"""
import json
import math
import os
import random
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))
from oracle import synth  # noqa: E402
from models import ResNet20, TinyNet  # noqa: E402


# ------------------------------------------------------------------ horovod stub
class _World:
    size = 1
    rank = 0
    registry = {}     # name -> {rank: tensor}
    reduced = {}      # name -> reduced tensor (allreduce)


def _install_horovod_stub():
    hvd = types.ModuleType("horovod")
    hvd.__path__ = []
    ht = types.ModuleType("horovod.torch")
    ht.__path__ = []
    mo = types.ModuleType("horovod.torch.mpi_ops")
    Average, Sum, Adasum = "Average", "Sum", "Adasum"

    class Handle:  # not a tuple: DGCCompressor.synchronize maps over tuples/lists
        def __init__(self, *fields):
            self.fields = fields

    def size():
        return _World.size

    def rank():
        return _World.rank

    def allgather_async(tensor, name=None):
        _World.registry.setdefault(name, {})[_World.rank] = tensor.detach().clone()
        return Handle("allgather", name)

    def allreduce_async_(tensor, name=None, op=Average):
        _World.registry.setdefault(name, {})[_World.rank] = tensor
        return Handle("allreduce", name, _World.rank, op)

    def synchronize(handle):
        handle = handle.fields
        kind, name = handle[0], handle[1]
        parts = _World.registry[name]
        if kind == "allgather":
            return torch.cat([parts[r] for r in range(_World.size)], dim=0)
        _, _, r, op = handle
        if name not in _World.reduced:
            acc = parts[0].detach().clone()
            for q in range(1, _World.size):
                acc.add_(parts[q])
            if op == Average:
                acc.div_(_World.size)
            _World.reduced[name] = acc
        parts[r].copy_(_World.reduced[name])
        return parts[r]

    def allreduce_(tensor, name=None, op=Average):
        return tensor

    for m in (ht, mo):
        m.size, m.rank, m.local_rank = size, rank, rank
    ht.allreduce_ = allreduce_
    mo.Average, mo.Sum, mo.Adasum = Average, Sum, Adasum
    mo.allreduce_async_, mo.allgather_async, mo.synchronize = allreduce_async_, allgather_async, synchronize
    ht.Average, ht.Sum, ht.Adasum = Average, Sum, Adasum
    ht.mpi_ops = mo
    hvd.torch = ht
    sys.modules.update({"horovod": hvd, "horovod.torch": ht, "horovod.torch.mpi_ops": mo})


def _import_reference():
    if not os.path.isdir(os.path.join(REF, "dgc")):
        raise SystemExit(f"reference not found at {REF}: goldens can only be regenerated in the build container")
    _install_horovod_stub()
    sys.path.insert(0, REF)
    import dgc.compression as C
    import dgc.memory as M
    import dgc.horovod as H
    import dgc.optim as O
    return C, M, H, O


# ------------------------------------------------------------------ recorders
class _Recorder:
    """Wraps torch.ge / torch.topk to record the threshold sequence, counts and
    whether the resample topk ran, without changing what the reference computes."""

    def __init__(self):
        self.ge, self.topk = torch.ge, torch.topk
        self.reset()

    def reset(self):
        self.thresholds, self.counts, self.topk_calls = [], [], 0

    def __enter__(self):
        rec = self

        def ge(a, b, *args, **kw):
            out = rec.ge(a, b, *args, **kw)
            if torch.is_tensor(b) and b.dim() == 0:
                rec.thresholds.append(np.float32(b.item()))
                rec.counts.append(int(out.sum().item()))
            return out

        def topk(*args, **kw):
            rec.topk_calls += 1
            return rec.topk(*args, **kw)

        torch.ge, torch.topk = ge, topk
        return self

    def __exit__(self, *exc):
        torch.ge, torch.topk = self.ge, self.topk


def _quiet(fn, *a, **kw):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **kw)


# ------------------------------------------------------------------ fixtures
def gen_attributes(C):
    numels = [1, 2, 7, 100, 999, 1000, 1001, 1999, 2000, 2001, 2002, 2500, 4096, 4097, 10000,
              65537, 100000, 147456, 1000000, 2359296, 25557032, 102760448, 1000000000, 7000000000]
    ratios = [1e-4, 1e-3, 0.00316, 0.01, 0.0316, 0.1, 0.316, 0.5, 1.0]
    samples = [0.001, 0.01, 0.05, 0.5, 1.0, 2.0]
    rows = []
    for sr in samples:
        comp = _quiet(C.DGCCompressor, 0.001, sample_ratio=sr)
        for r in ratios:
            comp.compress_ratio = r
            named = [(f"t{n}", (n, [n])) for n in numels]
            _quiet(comp.initialize, named)
            for n in numels:
                numel, shape, k, S, ks, stride = comp.attributes[f"t{n}"]
                rows.append(dict(numel=n, ratio=r, sample_ratio=sr, clamped_sample_ratio=comp.sample_ratio,
                                 attrs=[numel, k, S, ks, stride]))
    sched = {}
    for label, kw in {"wm5": dict(warmup_epochs=5), "wm5o": dict(warmup_epochs=5, warmup_coeff=[1, 1, 1, 1, 1]),
                      "wm0": dict(warmup_epochs=0), "wm3c": dict(warmup_epochs=3, warmup_coeff=0.5),
                      "ratio1000": dict(warmup_epochs=-1)}.items():
        ratio = 1000 if label == "ratio1000" else 0.001
        comp = _quiet(C.DGCCompressor, ratio, **kw)
        _quiet(comp.initialize, [("w", (1000000, [1000, 1000]))])
        seq = []
        for e in range(8):
            _quiet(comp.warmup_compress_ratio, e)
            seq.append([comp.compress_ratio, list(comp.attributes["w"][2:])])
        sched[label] = dict(kwargs=kw, base_ratio=ratio, per_epoch=seq)
    with open(os.path.join(HERE, "attributes.json"), "w") as f:
        json.dump(dict(rows=rows, schedules=sched), f, indent=0)
    print(f"attributes.json: {len(rows)} rows")


# compress cases: (name, N, ratio, kind, scale, nesterov, masking, fp16, int32, resample, steps, extra)
CASES = [
    ("n1m_r1e-3_nest", 1000000, 0.001, "normal", 1.0, True, True, False, False, True, 3, {}),
    ("n1m_r1e-3_plain_fp16_int32", 1000000, 0.001, "normal", 1.0, False, True, True, True, True, 3, {}),
    ("n200k_r1e-2_nest_nm", 200000, 0.01, "normal", 1.0, True, False, False, False, True, 3, {}),
    ("n147456_r1e-3_layered", 147456, 0.001, "layered", 1.0, True, True, False, False, True, 3, {}),
    ("n100k_bf16_ties", 100000, 0.001, "bf16", 1.0, True, True, False, False, True, 3, {}),
    ("n50k_r1e-2_noresample", 50000, 0.01, "normal", 1.0, False, True, False, False, False, 4, {}),
    ("n50k_r1e-2_noresample_layered", 50000, 0.01, "layered", 1.0, True, True, False, False, False, 4, {}),
    ("n2359296_r1e-3_nest", 2359296, 0.001, "normal", 1.0, True, True, False, False, True, 2, {}),
    ("n1500_small_direct", 1500, 0.001, "normal", 1.0, True, True, False, False, True, 3, {}),
    ("n2001_stride1", 2001, 0.001, "normal", 1.0, False, True, False, False, True, 3, {}),
    ("n4096_r1e-1", 4096, 0.1, "normal", 1.0, True, True, True, True, True, 3, {}),
    ("n30000_sparse_zeros", 30000, 0.01, "sparse", 1.0, True, True, False, False, True, 3, {}),
    ("n20000_ties_int", 20000, 0.01, "ties", 1.0, False, True, False, False, True, 3, {}),
    ("n65537_r1e-2_fp16_overflow", 65537, 0.01, "normal", 30000.0, False, True, True, False, True, 2, {}),
    ("n300k_iters3", 300000, 0.001, "layered", 1.0, True, True, False, False, True, 3, dict(max_adaptation_iters=3)),
]
FULL_STATE_MAX = 50000   # store full mmt/vec after each step up to this N


def gen_compress(C, M, rec):
    torch.set_num_threads(1)
    meta = {}
    arrays = {}
    for (name, N, r, kind, scale, nest, mask, fp16, i32, resample, steps, extra) in CASES:
        _World.size, _World.rank = 1, 0
        mem = M.DGCSGDMemory(momentum=0.9, nesterov=nest, momentum_masking=mask)
        comp = _quiet(C.DGCCompressor, r, memory=mem, fp16_values=fp16, int32_indices=i32,
                      resample=resample, **extra)
        param = torch.zeros(N)
        _quiet(mem.initialize, [("w", param)])
        _quiet(comp.initialize, [("w", param)])
        random.seed(42)
        case = dict(N=N, ratio=r, kind=kind, scale=scale, nesterov=nest, masking=mask, fp16=fp16,
                    int32=i32, resample=resample, steps=steps, extra=extra,
                    attrs=[comp.attributes["w"][i] for i in (0, 2, 3, 4, 5)], per_step=[])
        for s in range(steps):
            seed = 1000 * len(meta) + s
            g_np = synth.gradient(seed, N, kind, scale)
            grad = torch.from_numpy(g_np.copy())
            rstate = random.getstate()
            rec.reset()
            with rec:
                (vals, idx), ctx = comp.compress(grad, "w")
            start = None
            numel, shape, k, S, ks, stride = comp.attributes["w"]
            if numel != S:
                st = random.getstate()
                random.setstate(rstate)
                start = random.randint(0, stride - 1)
                random.setstate(st)
            step = dict(seed=seed, input_sha=synth.digest(g_np), start=start,
                        thresholds=[float(t) for t in rec.thresholds],
                        threshold_bits=[int(np.float32(t).view(np.uint32)) for t in rec.thresholds],
                        counts=rec.counts, topk_calls=rec.topk_calls, n=int(idx.numel()),
                        mmt_sha=synth.digest(mem.momentums["w"].numpy()),
                        vec_sha=synth.digest(mem.velocities["w"].numpy()))
            key = f"{name}/s{s}"
            arrays[key + "/indices"] = idx.view(-1).numpy().copy()
            arrays[key + "/values"] = vals.view(-1).numpy().copy()
            if N <= FULL_STATE_MAX:
                arrays[key + "/mmt"] = mem.momentums["w"].numpy().copy()
                arrays[key + "/vec"] = mem.velocities["w"].numpy().copy()
            # decompress at world size 1: result lands in the gradient buffer (ctx[5])
            out = comp.decompress((vals, idx), ctx)
            nz = np.flatnonzero(out.view(-1).numpy().view(np.uint32))
            arrays[key + "/dec_nz_idx"] = nz.astype(np.int64)
            arrays[key + "/dec_nz_val"] = out.view(-1).numpy()[nz].copy()
            case["per_step"].append(step)
        meta[name] = case
        print(f"compress {name}: branches " + ", ".join(f"{len(p['counts'])}c/{p['topk_calls']}t" for p in case["per_step"]))
    np.savez_compressed(os.path.join(HERE, "compress.npz"), **arrays)
    with open(os.path.join(HERE, "compress.json"), "w") as f:
        json.dump(meta, f, indent=1)


DEC_CASES = [
    # name, N, ratio, W, fp16, int32, kind
    ("w1", 20000, 0.01, 1, False, False, "normal"),
    ("w2", 20000, 0.01, 2, False, False, "normal"),
    ("w4_fp16_int32", 20000, 0.01, 4, True, True, "normal"),
    ("w8", 50000, 0.01, 8, False, False, "normal"),
    ("w8_fp16", 50000, 0.02, 8, True, False, "layered"),
    ("w3", 30000, 0.01, 3, False, False, "normal"),
]


def gen_decompress(C, M, rec):
    """W ranks emulated in one process: every rank seeds ``random`` identically
    (configs/__init__.py:9 + train.py seeding), compresses its own gradient with its
    own memory, and rank 0 decompresses the rank-order concatenation."""
    torch.set_num_threads(1)
    meta, arrays = {}, {}
    for ci, (name, N, r, W, fp16, i32, kind) in enumerate(DEC_CASES):
        _World.size = W
        comps = []
        for q in range(W):
            _World.rank = q
            mem = M.DGCSGDMemory(momentum=0.9, nesterov=True)
            comp = _quiet(C.DGCCompressor, r, memory=mem, fp16_values=fp16, int32_indices=i32)
            p = torch.zeros(N)
            _quiet(mem.initialize, [("w", p)])
            _quiet(comp.initialize, [("w", p)])
            comps.append(comp)
        random.seed(42)
        case = dict(N=N, ratio=r, W=W, fp16=fp16, int32=i32, kind=kind, steps=2, per_step=[])
        for s in range(2):
            rstate = random.getstate()
            payloads, ctxs, seeds = [], [], []
            for q in range(W):
                random.setstate(rstate)
                _World.rank = q
                seed = 50000 + 100 * ci + 10 * s + q
                g = synth.gradient(seed, N, kind)
                seeds.append(seed)
                (v, i), ctx = comps[q].compress(torch.from_numpy(g.copy()), "w")
                payloads.append((v, i))
                ctxs.append(ctx)
                arrays[f"{name}/s{s}/r{q}/values"] = v.view(-1).numpy().copy()
                arrays[f"{name}/s{s}/r{q}/indices"] = i.view(-1).numpy().copy()
            _World.rank = 0
            cat_v = torch.cat([p[0] for p in payloads])
            cat_i = torch.cat([p[1] for p in payloads])
            out = comps[0].decompress((cat_v, cat_i), ctxs[0])
            flat = out.view(-1).numpy()
            nz = np.flatnonzero(flat.view(np.uint32))
            arrays[f"{name}/s{s}/dec_nz_idx"] = nz.astype(np.int64)
            arrays[f"{name}/s{s}/dec_nz_val"] = flat[nz].copy()
            case["per_step"].append(dict(seeds=seeds, dense_sha=synth.digest(flat)))
        meta[name] = case
        print(f"decompress {name}: W={W}")
    np.savez_compressed(os.path.join(HERE, "decompress.npz"), **arrays)
    with open(os.path.join(HERE, "decompress.json"), "w") as f:
        json.dump(meta, f, indent=1)


def _trace_compress(comp, rank, trace, step):
    """Record every compress(p.grad, name) call of one rank: the order the reference's
    hooks fire in and the gradient each call sees (the GPU test replays both)."""
    orig = comp.compress

    def compress(tensor, name):
        trace.setdefault((step[0], rank), []).append((name, tensor.detach().clone().numpy()))
        return orig(tensor, name)

    comp.compress = compress


def _save_trace(label, trace, arrays, meta):
    for (s, q), calls in sorted(trace.items()):
        meta[f"{label}/s{s}/r{q}"] = [name for name, _ in calls]
        for j, (name, g) in enumerate(calls):
            arrays[f"{label}/s{s}/r{q}/{j}"] = g


def gen_optimizer(C, M, H, O, trace=None):
    """The reference's DistributedOptimizer + DGCSGD + DGCCompressor, 2 ranks emulated
    in one process. Records the weights after every step."""
    torch.set_num_threads(1)
    W, steps = 2, 3
    _World.size = W
    ranks = []
    for q in range(W):
        _World.rank = q
        torch.manual_seed(7)
        model = TinyNet()
        opt = O.DGCSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
        mem = M.DGCSGDMemory(momentum=0.9)
        comp = _quiet(C.DGCCompressor, 0.01, memory=mem, fp16_values=False, int32_indices=False,
                      warmup_epochs=-1)
        _quiet(mem.initialize, model.named_parameters())
        _quiet(comp.initialize, [(n, p) for n, p in model.named_parameters() if p.dim() > 1])
        dopt = H.DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                      backward_passes_per_step=1, op="Average")
        ranks.append((model, dopt, comp))
    step_ref = [0]
    if trace is not None:
        for q, (_, _, comp) in enumerate(ranks):
            _trace_compress(comp, q, trace, step_ref)
    random.seed(42)
    arrays = {}
    for s in range(steps):
        step_ref[0] = s
        _World.registry.clear()
        _World.reduced.clear()
        rstate = random.getstate()
        for q, (model, dopt, comp) in enumerate(ranks):
            _World.rank = q
            random.setstate(rstate)
            gen = torch.Generator().manual_seed(900 + 10 * s + q)
            x = torch.randn(32, 64, generator=gen)
            y = torch.randint(0, 10, (32,), generator=gen)
            loss = torch.nn.functional.cross_entropy(model(x), y)
            loss.backward()
        for q, (model, dopt, comp) in enumerate(ranks):
            _World.rank = q
            dopt.step()
            dopt.zero_grad()
            for n, p in model.named_parameters():
                arrays[f"s{s}/r{q}/{n}"] = p.detach().numpy().copy()
    torch.manual_seed(7)
    init = TinyNet()
    for n, p in init.named_parameters():
        arrays[f"init/{n}"] = p.detach().numpy().copy()
    np.savez_compressed(os.path.join(HERE, "optimizer.npz"), **arrays)
    with open(os.path.join(HERE, "optimizer.json"), "w") as f:
        json.dump(dict(W=W, steps=steps, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov_sgd=True,
                       memory_nesterov=False, ratio=0.01, batch=32, data_seed="900 + 10*step + rank",
                       model_seed=7, random_seed=42), f, indent=1)
    same = all(np.array_equal(arrays[f"s{s}/r0/{n}"], arrays[f"s{s}/r1/{n}"])
               for s in range(steps) for n, _ in ranks[0][0].named_parameters())
    print(f"optimizer: {steps} steps, replicas bit-identical: {same}")


def _digest(model):
    import hashlib
    h = hashlib.sha256()
    for _, p in model.named_parameters():
        h.update(p.detach().numpy().tobytes())
    return h.hexdigest()


def gen_optimizer_resnet20(C, M, H, O, trace=None):
    """BASELINE.json configs[0]: ResNet-20 / CIFAR-shaped batches with the reference's
    configs/cifar + configs/dgc + wm5 + fp16 + int32 settings (SGD lr 0.1, momentum
    0.9, wd 1e-4, no Nesterov; DGC ratio 0.001, sample 0.01, warmup 5 epochs,
    fp16 values, int32 indices), 2 ranks emulated in one process, 2 steps in each of
    epochs 0, 1 and 5 (ratios 0.316, 0.1, 0.001) with warmup_compress_ratio(epoch)
    called at each epoch start as train.py:203-208 does. Stores per-step SHA-256 digests of every rank's parameters and the final
    weights (replicas are bit-identical)."""
    torch.set_num_threads(1)
    W, epochs, spe, batch = 2, (0, 1, 5), 2, 8
    _World.size = W
    ranks = []
    for q in range(W):
        _World.rank = q
        torch.manual_seed(11)
        model = ResNet20()
        opt = O.DGCSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=False)
        mem = M.DGCSGDMemory(momentum=0.9)
        comp = _quiet(C.DGCCompressor, 0.001, memory=mem, sample_ratio=0.01, fp16_values=True,
                      int32_indices=True, warmup_epochs=5)
        _quiet(mem.initialize, model.named_parameters())
        _quiet(comp.initialize, [(n, p) for n, p in model.named_parameters() if p.dim() > 1])
        dopt = H.DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                      backward_passes_per_step=1, op="Average")
        ranks.append((model, dopt, comp))
    step_ref = [0]
    if trace is not None:
        for q, (_, _, comp) in enumerate(ranks):
            _trace_compress(comp, q, trace, step_ref)
    random.seed(42)
    digests, ratios = [], []
    for ei, e in enumerate(epochs):
        for q, (_, _, comp) in enumerate(ranks):
            _World.rank = q
            _quiet(comp.warmup_compress_ratio, e)
        ratios.append(ranks[0][2].compress_ratio)
        for t in range(spe):
            s = ei * spe + t
            step_ref[0] = s
            _World.registry.clear()
            _World.reduced.clear()
            rstate = random.getstate()
            for q, (model, dopt, comp) in enumerate(ranks):
                _World.rank = q
                random.setstate(rstate)
                gen = torch.Generator().manual_seed(1900 + 10 * s + q)
                x = torch.randn(batch, 3, 32, 32, generator=gen)
                y = torch.randint(0, 10, (batch,), generator=gen)
                loss = torch.nn.functional.cross_entropy(model(x), y)
                loss.backward()
            for q, (model, dopt, comp) in enumerate(ranks):
                _World.rank = q
                dopt.step()
                dopt.zero_grad()
            digests.append([_digest(m) for m, _, _ in ranks])
    arrays = {f"final/{n}": p.detach().numpy().copy() for n, p in ranks[0][0].named_parameters()}
    torch.manual_seed(11)
    init_digest = _digest(ResNet20())
    np.savez_compressed(os.path.join(HERE, "optimizer_resnet20.npz"), **arrays)
    with open(os.path.join(HERE, "optimizer_resnet20.json"), "w") as f:
        json.dump(dict(W=W, epochs=epochs, steps_per_epoch=spe, batch=batch, lr=0.1, momentum=0.9,
                       weight_decay=1e-4, nesterov_sgd=False, ratio=0.001, sample_ratio=0.01, warmup_epochs=5,
                       fp16_values=True, int32_indices=True, model_seed=11, random_seed=42,
                       data_seed="1900 + 10*step + rank", epoch_ratios=ratios, init_digest=init_digest,
                       step_digests=digests), f, indent=1)
    same = all(a == b for a, b in digests)
    print(f"optimizer_resnet20: {len(epochs) * spe} steps, ratios {ratios}, replicas bit-identical: {same}")


def gen_optimizer_trace(C, M, H, O):
    """The two DistributedOptimizer runs again, recording per step and rank the
    compress-call order and gradients (tests/golden/optimizer_trace.*): the GPU
    multi-rank test replays them through the product path on cuda:0 and must reach the
    reference's weights (optimizer.npz, optimizer_resnet20.*) bit for bit."""
    arrays, meta = {}, {}
    t1, t2 = {}, {}
    gen_optimizer(C, M, H, O, trace=t1)
    gen_optimizer_resnet20(C, M, H, O, trace=t2)
    _save_trace("tinynet", t1, arrays, meta)
    _save_trace("resnet20", t2, arrays, meta)
    np.savez_compressed(os.path.join(HERE, "optimizer_trace.npz"), **arrays)
    with open(os.path.join(HERE, "optimizer_trace.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"optimizer_trace: {len(meta)} (step, rank) call sequences")


# The dense Average beyond W = 2: the reference's DistributedOptimizer + DGCSGD on TinyNet
# at W = 3 / 4 / 8 (fp32 and fp16 wire values): its dense tensors (the biases; every
# tensor during a ratio-1 warmup epoch) are Average-allreduced (dgc/compression.py:205-206)
# — restated by the stub as the rank-order sum / W in the wire dtype, where the order
# decides the last bits. (label, W, fp16_values, int32_indices, epochs, steps_per_epoch,
# warmup kwargs)
MULTI_CASES = [
    ("w3_fp32", 3, False, False, (None,), 3, dict(warmup_epochs=-1)),
    ("w3_fp16", 3, True, True, (None,), 3, dict(warmup_epochs=-1)),
    ("w4_fp16", 4, True, False, (None,), 3, dict(warmup_epochs=-1)),
    ("w8_fp32", 8, False, False, (None,), 3, dict(warmup_epochs=-1)),
    ("w8_fp16", 8, True, True, (None,), 3, dict(warmup_epochs=-1)),
    # wm5o (configs/dgc/wm5o.py): ratio 1 for epochs 0-4 (every tensor dense), then 0.01
    ("w4_fp16_wm5o", 4, True, True, (0, 5), 2, dict(warmup_epochs=5, warmup_coeff=[1, 1, 1, 1, 1])),
]


def gen_optimizer_multi(C, M, H, O):
    """MULTI_CASES: W ranks emulated in one process (as gen_optimizer); per case the
    weights after every step (rank 0's; the replicas must be bit-identical, which is
    checked here) and every rank's compress-call order and gradients (the GPU tests
    replay them through the product path)."""
    torch.set_num_threads(1)
    arrays, meta = {}, {}
    for label, W, fp16, i32, epochs, spe, wkw in MULTI_CASES:
        _World.size = W
        ranks = []
        for q in range(W):
            _World.rank = q
            torch.manual_seed(7)
            model = TinyNet()
            opt = O.DGCSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
            mem = M.DGCSGDMemory(momentum=0.9)
            comp = _quiet(C.DGCCompressor, 0.01, memory=mem, fp16_values=fp16, int32_indices=i32, **wkw)
            _quiet(mem.initialize, model.named_parameters())
            _quiet(comp.initialize, [(n, p) for n, p in model.named_parameters() if p.dim() > 1])
            dopt = H.DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                          backward_passes_per_step=1, op="Average")
            ranks.append((model, dopt, comp))
        trace, step_ref = {}, [0]
        for q, (_, _, comp) in enumerate(ranks):
            _trace_compress(comp, q, trace, step_ref)
        random.seed(42)
        schedule = [(e if t == 0 else None, ei * spe + t) for ei, e in enumerate(epochs) for t in range(spe)]
        same = True
        for epoch, s in schedule:
            if epoch is not None:
                for q, (_, _, comp) in enumerate(ranks):
                    _World.rank = q
                    _quiet(comp.warmup_compress_ratio, epoch)
            step_ref[0] = s
            _World.registry.clear()
            _World.reduced.clear()
            rstate = random.getstate()
            for q, (model, dopt, comp) in enumerate(ranks):
                _World.rank = q
                random.setstate(rstate)
                gen = torch.Generator().manual_seed(3000 + 100 * W + 10 * s + q)
                x = torch.randn(32, 64, generator=gen)
                y = torch.randint(0, 10, (32,), generator=gen)
                torch.nn.functional.cross_entropy(model(x), y).backward()
            for q, (model, dopt, comp) in enumerate(ranks):
                _World.rank = q
                dopt.step()
                dopt.zero_grad()
            for n, p in ranks[0][0].named_parameters():
                arrays[f"{label}/s{s}/{n}"] = p.detach().numpy().copy()
                same &= all(np.array_equal(p.detach().numpy(), dict(m.named_parameters())[n].detach().numpy())
                            for m, _, _ in ranks[1:])
        if not same:
            raise SystemExit(f"optimizer_multi {label}: the reference's replicas diverged")
        _save_trace(label, trace, arrays, meta)
        meta[label] = dict(W=W, fp16_values=fp16, int32_indices=i32, epochs=list(epochs), steps_per_epoch=spe,
                           warmup=wkw, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov_sgd=True,
                           memory_nesterov=False, ratio=0.01, batch=32, data_seed="3000 + 100*W + 10*step + rank",
                           model_seed=7, random_seed=42, steps=len(schedule))
        print(f"optimizer_multi {label}: W={W}, {len(schedule)} steps, replicas bit-identical")
    np.savez_compressed(os.path.join(HERE, "optimizer_multi.npz"), **arrays)
    with open(os.path.join(HERE, "optimizer_multi.json"), "w") as f:
        json.dump(meta, f, indent=1)


# 16-bit parameters: the reference's memory + compressor on bf16 / fp16 tensors (every
# ATen op rounds to the dtype). (name, N, ratio, dtype, kind, scale, nesterov, masking,
# fp16_values, int32, resample, steps, W)
HALF_CASES = [
    ("bf16_n200k_nest", 200000, 0.001, "bfloat16", "normal", 1.0, True, True, False, False, True, 3, 1),
    ("bf16_n100k_plain_fp16v_i32", 100000, 0.01, "bfloat16", "normal", 1.0, False, True, True, True, True, 3, 1),
    ("bf16_n30000_ties_nm", 30000, 0.01, "bfloat16", "ties", 1.0, True, False, False, False, True, 3, 1),
    ("bf16_n50k_noresample", 50000, 0.01, "bfloat16", "layered", 1.0, True, True, False, False, False, 4, 1),
    ("fp16_n200k_nest", 200000, 0.001, "float16", "normal", 1e-2, True, True, False, False, True, 3, 1),
    ("fp16_n100k_plain_fp16v", 100000, 0.01, "float16", "layered", 1.0, False, True, True, False, True, 3, 1),
    ("fp16_n65537_overflow", 65537, 0.01, "float16", "normal", 3000.0, False, True, False, False, True, 2, 1),
    ("bf16_n2001_stride1", 2001, 0.001, "bfloat16", "normal", 1.0, False, True, False, False, True, 3, 1),
    ("bf16_w3", 20000, 0.01, "bfloat16", "normal", 1.0, True, True, False, False, True, 2, 3),
    ("fp16_w2_fp16v_i32", 20000, 0.01, "float16", "normal", 1e-2, True, True, True, True, True, 2, 2),
    ("bf16_w4_fp16v", 30000, 0.01, "bfloat16", "layered", 1.0, True, True, True, False, True, 2, 4),
]
HALF_FULL_STATE_MAX = 50000


def gen_half(C, M, rec):
    """Per step and rank: the indices and values the reference transmits, its
    thresholds / counts, the 16-bit state (N <= HALF_FULL_STATE_MAX) and the
    decompressed gradient of the rank-order concatenation (W ranks emulated as in
    gen_decompress: identical ``random`` state per rank)."""
    torch.set_num_threads(1)
    meta, arrays = {}, {}
    for ci, (name, N, r, dts, kind, scale, nest, mask, fp16, i32, resample, steps, W) in enumerate(HALF_CASES):
        dt = getattr(torch, dts)
        _World.size = W
        comps, mems = [], []
        for q in range(W):
            _World.rank = q
            mem = M.DGCSGDMemory(momentum=0.9, nesterov=nest, momentum_masking=mask)
            comp = _quiet(C.DGCCompressor, r, memory=mem, fp16_values=fp16, int32_indices=i32, resample=resample)
            prm = torch.zeros(N, dtype=dt)
            _quiet(mem.initialize, [("w", prm)])
            _quiet(comp.initialize, [("w", prm)])
            comps.append(comp)
            mems.append(mem)
        random.seed(42)
        case = dict(N=N, ratio=r, dtype=dts, kind=kind, scale=scale, nesterov=nest, masking=mask, fp16=fp16,
                    int32=i32, resample=resample, steps=steps, W=W,
                    attrs=[comps[0].attributes["w"][i] for i in (0, 2, 3, 4, 5)], per_step=[])
        for s in range(steps):
            rstate = random.getstate()
            payloads, ctxs, ranks = [], [], []
            for q in range(W):
                random.setstate(rstate)
                _World.rank = q
                seed = 70000 + 100 * ci + 10 * s + q
                g = torch.from_numpy(synth.gradient(seed, N, kind, scale).copy()).to(dt)
                rec.reset()
                with rec:
                    (v, i), ctx = comps[q].compress(g, "w")
                payloads.append((v, i))
                ctxs.append(ctx)
                key = f"{name}/s{s}/r{q}"
                arrays[key + "/indices"] = i.view(-1).numpy().copy()
                arrays[key + "/values"] = v.view(-1).float().numpy().copy()
                if N <= HALF_FULL_STATE_MAX:
                    arrays[key + "/mmt"] = mems[q].momentums["w"].float().numpy().copy()
                    arrays[key + "/vec"] = mems[q].velocities["w"].float().numpy().copy()
                ranks.append(dict(seed=seed, thresholds=[float(t) for t in rec.thresholds], counts=rec.counts,
                                  topk_calls=rec.topk_calls, n=int(i.numel()), values_dtype=str(v.dtype),
                                  mmt_sha=synth.digest(mems[q].momentums["w"].float().numpy()),
                                  vec_sha=synth.digest(mems[q].velocities["w"].float().numpy())))
            _World.rank = 0
            cat_v = torch.cat([p[0] for p in payloads])
            cat_i = torch.cat([p[1] for p in payloads])
            out = comps[0].decompress((cat_v, cat_i), ctxs[0])
            flat = out.view(-1).float().numpy()
            nz = np.flatnonzero(flat.view(np.uint32))
            arrays[f"{name}/s{s}/dec_nz_idx"] = nz.astype(np.int64)
            arrays[f"{name}/s{s}/dec_nz_val"] = flat[nz].copy()
            case["per_step"].append(dict(ranks=ranks, out_dtype=str(out.dtype), dense_sha=synth.digest(flat)))
        meta[name] = case
        print(f"half {name}: " + ", ".join(f"{len(p['ranks'][0]['counts'])}c/{p['ranks'][0]['topk_calls']}t"
                                           for p in case["per_step"]))
    np.savez_compressed(os.path.join(HERE, "half.npz"), **arrays)
    with open(os.path.join(HERE, "half.json"), "w") as f:
        json.dump(meta, f, indent=1)


# DGCSGD.step on bf16 / fp16 parameters (dgc/optim/sgd.py:42-68 on 16-bit tensors; CPU,
# one thread): (label, dtype, lr, momentum, dampening, weight_decay, nesterov). The shapes
# give every length class of the CPU kernels' 32-element vector body and scalar tail.
SGD16_CASES = [
    ("bf16_nest_wd", "bfloat16", 0.1, 0.9, 0.0, 1e-4, True),
    ("bf16_plain_wd_damp", "bfloat16", 0.05, 0.9, 0.1, 5e-4, False),
    ("bf16_nowd", "bfloat16", 0.1, 0.9, 0.0, 0.0, False),
    ("fp16_nest_wd", "float16", 0.1, 0.9, 0.0, 1e-4, True),
    ("fp16_plain_wd_damp", "float16", 0.05, 0.9, 0.1, 5e-4, False),
    ("fp16_wd_nomom", "float16", 0.1, 0.0, 0.0, 1e-4, False),
]
SGD16_SHAPES = [("a", (37,)), ("b", (64, 3, 7, 7)), ("c", (1000,)), ("d", (333, 7)), ("e", (16,)), ("f", (1024, 33))]


def sgd16_inputs(gen, dt, steps=3):
    """The seeded inputs of an SGD16 case (the test regenerates them the same way): the
    initial parameters, then each step's gradients, drawn in this order."""
    init = [(torch.randn(s, generator=gen) * 0.5).to(dt) for _, s in SGD16_SHAPES]
    grads = [[(torch.randn(s, generator=gen) * 0.01).to(dt) for _, s in SGD16_SHAPES] for _ in range(steps)]
    return init, grads


def gen_sgd16(O):
    """Per case: the parameters after each of 3 DGCSGD steps on 16-bit parameters, and
    the momentum buffers after the last (16-bit patterns), from the seeded inputs of
    ``sgd16_inputs`` (torch.Generator(4000 + case) normal draws; the test regenerates them)."""
    torch.set_num_threads(1)
    arrays, meta = {}, {}
    bits = lambda t: t.detach().contiguous().view(torch.int16).numpy().copy()   # noqa: E731
    for ci, (label, dts, lr, mom, damp, wd, nest) in enumerate(SGD16_CASES):
        dt = getattr(torch, dts)
        init, grads = sgd16_inputs(torch.Generator().manual_seed(4000 + ci), dt)
        params = [torch.nn.Parameter(t) for t in init]
        opt = O.DGCSGD(params, lr=lr, momentum=mom, dampening=damp, weight_decay=wd, nesterov=nest)
        for s in range(3):
            for p, g in zip(params, grads[s]):
                p.grad = g
            opt.step()
            for (n, _), p in zip(SGD16_SHAPES, params):
                arrays[f"{label}/s{s}/p/{n}"] = bits(p)
                buf = opt.state[p].get("momentum_buffer")
                if buf is not None and s == 2:
                    arrays[f"{label}/buf/{n}"] = bits(buf)
        meta[label] = dict(dtype=dts, lr=lr, momentum=mom, dampening=damp, weight_decay=wd, nesterov=nest, steps=3,
                           shapes=SGD16_SHAPES)
        print(f"sgd16 {label}")
    np.savez_compressed(os.path.join(HERE, "sgd16.npz"), **arrays)
    with open(os.path.join(HERE, "sgd16.json"), "w") as f:
        json.dump(meta, f, indent=1)


GENERATORS = ("attributes", "compress", "decompress", "optimizer", "optimizer_resnet20", "optimizer_trace", "half",
              "optimizer_multi", "sgd16")


def main(which=GENERATORS):
    C, M, H, O = _import_reference()
    rec = _Recorder()
    if "attributes" in which:
        gen_attributes(C)
    if "compress" in which:
        gen_compress(C, M, rec)
    if "decompress" in which:
        gen_decompress(C, M, rec)
    if "optimizer" in which:
        gen_optimizer(C, M, H, O)
    if "optimizer_resnet20" in which:
        gen_optimizer_resnet20(C, M, H, O)
    if "optimizer_trace" in which:
        gen_optimizer_trace(C, M, H, O)
    if "half" in which:
        gen_half(C, M, rec)
    if "optimizer_multi" in which:
        gen_optimizer_multi(C, M, H, O)
    if "sgd16" in which:
        gen_sgd16(O)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or GENERATORS)
