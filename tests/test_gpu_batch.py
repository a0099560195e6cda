"""The batched step: every compressed tensor of a model in one
set of launches (dgc.batch.DGCBatch -> dgc_batch_compress), checked tensor by tensor
against the oracle — the reference's per-hook compress (dgc/horovod/optimizer.py:116-155,
dgc/compression.py:155-177) with one random.randint per tensor in the tensors' order."""
import random

import numpy as np
import pytest
import torch

from oracle import dgc_oracle as O
from oracle import synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({4: np.uint32, 2: np.uint16, 8: np.uint64}[a.dtype.itemsize])


def _same_or_nan(a, b):
    """Bitwise equal, except that NaN matches NaN (numpy and the GPU may carry different
    NaN payloads through the momentum arithmetic)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return bool(np.all((np.isnan(a) & np.isnan(b)) | (bits(a) == bits(b))))


def _assert_sent(gi, gv, oi, wv, info, key):
    """The transmitted (indices, wire values) against the oracle's: in order, or — a
    resample whose k-th key was untied under resample_order="index" (tie rule "set") —
    torch.topk's set in ascending index order."""
    gi, gv = gi.cpu().numpy(), gv.cpu().numpy()
    if info.get("tie_rule") == "set":
        o = np.argsort(oi, kind="stable")
        oi, wv = oi[o], wv[o]
    assert np.array_equal(gi, oi), (key, info)
    assert np.array_equal(bits(gv), bits(wv)), (key, info)


def _sets():
    from dgc import workloads
    r50, _ = workloads.split(workloads.resnet50())
    vgg, _ = workloads.split(workloads.vgg16_bn())
    mixed = [("tiny_direct", (1500,)), ("stride1", (2001,)), ("a", (64, 3, 7, 7)), ("odd", (1000003,)),
             ("b", (300, 1000)), ("ties", (4099,)), ("c", (2048, 1024))]
    return {"resnet50": (r50, False, False), "vgg16_bn": (vgg, True, True), "mixed": (mixed, False, False)}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("label,shape", [("mixed", None), ("resnet50", None), ("vgg16_bn", None),
                                         ("mixed", "quarter"), ("resnet50", "quarter"), ("mixed+naninf", None),
                                         ("mixed", "k5multi"), ("resnet50", "k5multi"), ("mixed", "k5abort"),
                                         ("resnet50", "k5abort"), ("mixed", "topk"), ("resnet50", "topk")])
def test_batch_matches_per_tensor_oracle(label, shape, monkeypatch):
    """shape: the emit kernel (None: the library's choice — k_emit_wide for these few
    groups; "quarter": k_emit, the flat buckets' kernel, forced), or "k5multi": the
    resample replay's global phase over several workgroups per tensor (k_nth_global);
    "topk": resample_order="topk" (every resample replays torch's order; the K5 shapes
    too) — otherwise DGCBatch's default "index" (an untied resample: the set). "+naninf": tensor "b"
    gets a NaN at one of its samples on step 1 (its threshold turns NaN, nothing of it
    is selected), "odd" a NaN that is never sampled and "c" +-inf — the other tensors'
    selections must not notice."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if shape == "k5multi":   # K5's global phase over several workgroups per tensor, whatever the capacity
        monkeypatch.setenv("DGC_K5_GLOBAL", "multi")
    elif shape == "k5abort":   # ... whose residency consensus times out: the one-workgroup fallback
        monkeypatch.setenv("DGC_K5_GLOBAL", "abort")
    elif shape and shape != "topk":
        monkeypatch.setenv("DGC_EMIT_SHAPE", shape)
    order = "topk" if shape in ("k5multi", "k5abort", "topk") else "index"
    from dgc.batch import DGCBatch
    naninf = label.endswith("+naninf")
    label = label.split("+")[0]
    shapes, fp16, int32 = _sets()[label]
    nest = label == "mixed"
    b = DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, nesterov=nest, fp16_values=fp16,
                 int32_indices=int32, device=DEV, seed=42, resample_order=order)
    ref_rng = random.Random(42)
    state = {n: (np.zeros(b.numels[i], np.float32), np.zeros(b.numels[i], np.float32))
             for i, n in enumerate(b.names)}
    branches = set()
    fallbacks = replays = sets = 0
    steps = 3 if label != "vgg16_bn" else 2
    for s in range(steps):
        # state read on odd and last steps only: reading flushes the deferred masking, so the
        # other steps leave it to the next K1 (the bench's path)
        check_state = s % 2 == 1 or s == steps - 1
        grads = {}
        starts = b.draw_starts()
        for t, name in enumerate(b.names):
            kind = "ties" if name == "ties" else ("layered" if t % 3 == 0 else "normal")
            g = synth.gradient(1000 * s + t, b.numels[t], kind, 1e-3 * (1 + t % 7))
            if naninf:
                stride = b.attrs[t][3]
                if name == "b" and s == 1:
                    g[7 * stride + starts[t]] = np.nan                       # sampled this step
                if name == "odd" and s == 0:
                    g[5 * stride + (starts[t] + 1) % stride] = np.nan      # a residue not sampled at s=0
                if name == "c":
                    g[[11 + s, 5000 + s]] = [np.inf, -np.inf]
            grads[name] = g
            b.grad(name).copy_(torch.from_numpy(g).view(b.shapes[name]))
        b.compress(starts)
        out = b.decompress()
        torch.cuda.synchronize()
        sent = b.transmitted()
        infos = b.infos()
        for t, name in enumerate(b.names):
            N = b.numels[t]
            attrs = O.attributes(N, 0.001)
            start = ref_rng.randint(0, attrs[4] - 1) if attrs[0] != attrs[2] else 0
            assert start == starts[t], (name, s)
            m_o, v_o = state[name]
            ov, oi, info = O.compress_step(grads[name], m_o, v_o, attrs, start, nesterov=nest)
            wv, wi = O.wire_cast(ov, oi, fp16, int32)
            key = f"{label}/s{s}/{name}"
            branches.add(info["branch"])
            assert infos[t]["branch"] == info["branch"], key
            replays += infos[t]["branch"] == "resample" and infos[t]["tie_rule"] == "exact"
            sets += infos[t]["tie_rule"] == "set"
            assert order == "index" or infos[t]["tie_rule"] != "set", key
            fallbacks += infos[t]["k5_fallback"]
            if shape != "k5abort":
                assert not infos[t]["k5_fallback"], (key, infos[t])
            gv, gi = sent[name]
            _assert_sent(gi, gv, oi, wv, infos[t], key)
            if check_state:
                assert _same_or_nan(b.momentum_of(name).reshape(-1).cpu().numpy(), m_o), key
                assert _same_or_nan(b.velocity_of(name).reshape(-1).cpu().numpy(), v_o), key
            if naninf and name == "b" and s == 1:
                assert np.isnan(infos[t]["threshold0"]) and infos[t]["count"] == 0, (key, infos[t])
            dense = O.decompress([wv], [oi], N, 1)
            assert np.array_equal(bits(b.out(name).reshape(-1).cpu().numpy()), bits(dense)), key
        # padding between tensors stays zero (no tensor writes outside itself)
        pad = torch.ones(b.flat_numel, dtype=torch.bool, device=DEV)
        for off, n in zip(b.offsets, b.numels):
            pad[off: off + n] = False
        assert not bool(out[pad].any())
        if check_state:
            assert not bool(b.vec_flat[pad].any())
    if label == "mixed":
        assert {"direct", "resample"} <= branches, branches
        if order == "index":   # the untied resamples took the set path, the "ties" tensor the replay
            assert sets > 0, (sets, replays)
    if shape == "k5abort":   # every replay that reached the consensus fell back, exactly
        assert replays > 0 and fallbacks > 0, (replays, fallbacks)


def test_batch_warmup_ratio_change():
    """warmup_compress_ratio re-initialises the attributes mid-run (dgc/compression.py:91-107)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dgc import workloads
    from dgc.batch import DGCBatch
    shapes, _ = workloads.split(workloads.resnet20())
    b = DGCBatch(shapes, compress_ratio=0.316, momentum=0.9, fp16_values=True, int32_indices=True, device=DEV,
                 seed=7)
    ref_rng = random.Random(7)
    state = {n: (np.zeros(b.numels[i], np.float32), np.zeros(b.numels[i], np.float32))
             for i, n in enumerate(b.names)}
    for s, ratio in enumerate([0.316, 0.316, 0.1, 0.001, 0.001]):
        if ratio != b.ratio:
            b.set_ratio(ratio)
        grads = {}
        for t, name in enumerate(b.names):
            grads[name] = synth.gradient(77 * s + t, b.numels[t], "normal", 0.01)
            b.grad(name).copy_(torch.from_numpy(grads[name]).view(b.shapes[name]))
        b.compress()
        if s == 4:
            b.out_flat.add_(1.0)   # an in-place write (version bump): the next decompress fills densely
        out = b.decompress()   # persistent output: sparse re-zero except after a ratio change
        torch.cuda.synchronize()
        sent = b.transmitted()
        infos = b.infos()
        for t, name in enumerate(b.names):
            attrs = O.attributes(b.numels[t], ratio)
            start = ref_rng.randint(0, attrs[4] - 1) if attrs[0] != attrs[2] else 0
            m_o, v_o = state[name]
            ov, oi, _ = O.compress_step(grads[name], m_o, v_o, attrs, start)
            wv, wi = O.wire_cast(ov, oi, True, True)
            _assert_sent(sent[name][1], sent[name][0], oi, wv, infos[t], (s, name))
            dense = O.decompress([wv], [oi], b.numels[t], 1)
            assert np.array_equal(bits(b.out(name).reshape(-1).cpu().numpy()), bits(dense)), (s, name)
        pad = torch.ones(b.flat_numel, dtype=torch.bool, device=DEV)
        for off, n in zip(b.offsets, b.numels):
            pad[off: off + n] = False
        assert not bool(out[pad].any()), s


def test_batch_sparse_rezero_matches_dense_fill():
    """fill="sparse" (the persistent output's re-zero of the previous step's entries)
    against fill="inline" (the dense zero_() every step): identical outputs, step by
    step, on the ResNet-50 set with the bench's synthetic gradients."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dgc import workloads
    from dgc.batch import DGCBatch
    shapes, _ = workloads.split(workloads.resnet50())
    bs = [DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, device=DEV, seed=3, fill=f)
          for f in ("sparse", "inline")]
    gen = torch.Generator(device=DEV)
    for s in range(6):
        gen.manual_seed(100 + s % 2)
        g = torch.zeros(bs[0].flat_numel, device=DEV)
        for off, n in zip(bs[0].offsets, bs[0].numels):
            g[off: off + n] = torch.randn(n, generator=gen, device=DEV) * 1e-3
        outs = []
        for b in bs:
            b.grad_flat.copy_(g)
            b.compress()
            outs.append(b.decompress())
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)), s


@pytest.mark.timeout(600)
def test_batch_index_order_equals_topk_order():
    """resample_order="index" (the set of an untied resample in index order, K5s) against
    "topk" (torch's order, the exact replay) on the ResNet-50 set with the bench's
    alternating gradients, whose bimodal velocities resample every other step: the same
    sets, the same dense outputs and the same memory state, bit for bit, every step."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dgc import workloads
    from dgc.batch import DGCBatch
    shapes, _ = workloads.split(workloads.resnet50())
    bs = [DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, device=DEV, seed=5, resample_order=o)
          for o in ("index", "topk")]
    gen = torch.Generator(device=DEV)
    sets = 0
    for s in range(8):
        gen.manual_seed(0xD6C + s % 2)
        g = torch.zeros(bs[0].flat_numel, device=DEV)
        for off, n in zip(bs[0].offsets, bs[0].numels):
            g[off: off + n] = torch.randn(n, generator=gen, device=DEV) * 1e-3
        outs = []
        for b in bs:
            b.grad_flat.copy_(g)
            b.compress()
            outs.append(b.decompress().clone())
        torch.cuda.synchronize()
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)), s
        ia, it = bs[0].infos(), bs[1].infos()
        sa, st = bs[0].transmitted(), bs[1].transmitted()
        for t, name in enumerate(bs[0].names):
            assert ia[t]["branch"] == it[t]["branch"] and ia[t]["count"] == it[t]["count"], (s, name)
            if ia[t]["tie_rule"] == "set":
                sets += 1
                assert it[t]["tie_rule"] == "exact", (s, name)
                oi = st[name][1].cpu().numpy()
                o = np.argsort(oi, kind="stable")
                assert np.array_equal(sa[name][1].cpu().numpy(), oi[o]), (s, name)
                assert np.array_equal(bits(sa[name][0].cpu().numpy()), bits(st[name][0].cpu().numpy()[o])), (s, name)
            else:
                assert torch.equal(sa[name][1], st[name][1]), (s, name)
    for name in bs[0].names:
        assert torch.equal(bs[0].velocity_of(name).view(torch.int32), bs[1].velocity_of(name).view(torch.int32))
        assert torch.equal(bs[0].momentum_of(name).view(torch.int32), bs[1].momentum_of(name).view(torch.int32))
    assert sets > 0


def biased_sample_gradient(n, stride, start):
    """A gradient whose resample set's sampled positions hold its LARGEST keys: 60000
    magnitudes 3.1 - i * 1e-6 (decreasing with the index) at the first positions the
    strided sample (start, stride) misses, then 200000 magnitudes 2 + i * 4.5e-6 (the
    sample's share sets the threshold near their top), N(0, 1e-3) elsewhere."""
    g = torch.randn(n, generator=torch.Generator().manual_seed(3)) * 1e-3
    idx = torch.arange(n)
    free = idx[(idx - start) % stride != 0][:60000]
    g[free] = 3.1 - torch.arange(60000, dtype=torch.float64).mul(1e-6).float()
    b0 = int(free[-1]) + 1
    g[b0: b0 + 200000] = 2.0 + torch.arange(200000, dtype=torch.float64).mul(4.5e-6).float()
    return g


def test_batch_index_order_biased_samples():
    """K5s bounds its radix passes from 4096 samples taken at fixed candidate positions
    (rounds 0, 4, 8, 12 in index order) once a set passes 16384 candidates. Here those
    positions hold the set's largest keys (``biased_sample_gradient``), so the sampled
    bound sits above the k-th key and the count check must drop it: the set (a resample
    over ~70k candidates, k = 10000, untied) still equals torch's top-k."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import random
    from dgc.batch import DGCBatch
    n = 10_000_000
    shapes = [("a", (n,)), ("small", (300, 1000))]
    bs = [DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, device=DEV, seed=11, resample_order=o)
          for o in ("index", "topk")]
    stride = bs[0].attrs[0][3]
    start = random.Random(11).randint(0, stride - 1)   # the batch's first draw: tensor 0's sample start
    flat = torch.zeros(bs[0].flat_numel)
    flat[:n] = biased_sample_gradient(n, stride, start)
    off, m = bs[0].offsets[1], bs[0].numels[1]
    flat[off: off + m] = torch.randn(m, generator=torch.Generator().manual_seed(4)) * 1e-3
    outs = []
    for b in bs:
        b.grad_flat.copy_(flat.to(DEV))
        b.compress()
        outs.append(b.decompress().clone())
    torch.cuda.synchronize()
    ia = bs[0].infos()[0]
    assert ia["branch"] == "resample" and ia["candidates"] > 16384 and ia["tie_rule"] == "set", ia
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    sa, st = bs[0].transmitted()["a"], bs[1].transmitted()["a"]
    o = np.argsort(st[1].cpu().numpy(), kind="stable")
    assert np.array_equal(sa[1].cpu().numpy(), st[1].cpu().numpy()[o])
    assert np.array_equal(bits(sa[0].cpu().numpy()), bits(st[0].cpu().numpy()[o]))
    assert torch.equal(bs[0].velocity_of("a").view(torch.int32), bs[1].velocity_of("a").view(torch.int32))


def designed_big_gradient(n, k, stride, start, seed, top=1.2):
    """A gradient whose resample has more candidates than one workgroup's set path, its
    k-th largest magnitude untied and `top` / 1 above the threshold (within an octave by
    default): k distinct magnitudes top + i * 2e-7 at positions the strided sample
    (start, stride) misses, a plateau of 500k magnitudes exactly 1.0, N(0, 1e-3)
    elsewhere, random signs. The samples see only the plateau, so the threshold is 1.0
    and its count (~520k) passes 1.3k: resample over ~520k candidates, whose top k are
    the distinct ones."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g) * 1e-3
    off = (start + stride // 2) % stride                      # a residue the samples never hit
    slots = torch.arange(off, n, stride)
    big = slots[torch.randperm(slots.numel(), generator=g)[:k]]
    x[big] = (top + torch.arange(k, dtype=torch.float64).mul(2e-7)).float()
    rest = torch.ones(n, dtype=torch.bool)
    rest[big] = False
    cand = rest.nonzero().view(-1)
    x[cand[torch.randperm(cand.numel(), generator=g)[:500_000]]] = 1.0
    sign = torch.randint(0, 2, (n,), generator=g).float().mul(2).sub(1)
    return x * sign


@pytest.mark.timeout(600)
def test_batch_index_order_big_resample():
    """The set path past 16 x 16384 = 262144 candidates (a tensor whose capacity exceeds
    it gets up to 128 co-resident workgroups in k_resample_set) against the exact replay: a
    20M-element tensor (k = 20000, up to 64k = 1.28M candidates) whose first gradient
    (``designed_big_gradient``) resamples over ~520k candidates (32 workgroups), then
    random steps — the same sets, outputs and state as resample_order="topk"."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import random
    from dgc.batch import DGCBatch
    shapes = [("big", (20_000_000,)), ("small", (300, 1000))]
    bs = [DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, device=DEV, seed=5, resample_order=o)
          for o in ("index", "topk")]
    k, _, _, stride = bs[0].attrs[0]
    start = random.Random(5).randint(0, stride - 1)   # the batch's first draw: tensor 0's sample start
    gen = torch.Generator(device=DEV)
    big_sets = 0
    for s in range(3):
        gen.manual_seed(77 + s)
        g = torch.randn(bs[0].flat_numel, generator=gen, device=DEV) * 1e-3
        if s == 0:
            g[bs[0].offsets[0]: bs[0].offsets[0] + bs[0].numels[0]] = \
                designed_big_gradient(bs[0].numels[0], k, stride, start, 100).to(DEV)
        outs = []
        for b in bs:
            b.grad_flat.copy_(g)
            b.compress()
            outs.append(b.decompress().clone())
        torch.cuda.synchronize()
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)), s
        ia, it = bs[0].infos(), bs[1].infos()
        sa, st = bs[0].transmitted(), bs[1].transmitted()
        for t, name in enumerate(bs[0].names):
            assert ia[t]["branch"] == it[t]["branch"] and ia[t]["candidates"] == it[t]["candidates"], (s, name)
            if ia[t]["tie_rule"] == "set":
                big_sets += ia[t]["candidates"] > 262144
                oi = st[name][1].cpu().numpy()
                o = np.argsort(oi, kind="stable")
                assert np.array_equal(sa[name][1].cpu().numpy(), oi[o]), (s, name)
                assert np.array_equal(bits(sa[name][0].cpu().numpy()), bits(st[name][0].cpu().numpy()[o])), (s, name)
            else:
                assert torch.equal(sa[name][1], st[name][1]), (s, name)
        if s == 0:   # the designed step: a resample of ~520k candidates through the set path
            assert ia[0]["branch"] == "resample" and ia[0]["candidates"] > 262144, ia[0]
            assert ia[0]["tie_rule"] == "set", ia[0]
    for name in bs[0].names:
        assert torch.equal(bs[0].velocity_of(name).view(torch.int32), bs[1].velocity_of(name).view(torch.int32))
        assert torch.equal(bs[0].momentum_of(name).view(torch.int32), bs[1].momentum_of(name).view(torch.int32))
    assert big_sets > 0


@pytest.mark.timeout(600)
def test_batch_index_order_wide_span_resample():
    """A resample whose k-th largest is more than four octaves above the threshold (the
    designed gradient with its k distinct magnitudes at 40, the plateau at 1.0): past
    the set path's 25-bit key span above key(t_cur), so the exact replay takes the
    tensor — the payload, velocity and momentum of resample_order="index" equal
    resample_order="topk"'s bit for bit, in topk's order."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import random
    from dgc.batch import DGCBatch
    shapes = [("big", (20_000_000,)), ("small", (300, 1000))]
    bs = [DGCBatch(shapes, compress_ratio=0.001, momentum=0.9, device=DEV, seed=5, resample_order=o)
          for o in ("index", "topk")]
    k, _, _, stride = bs[0].attrs[0]
    start = random.Random(5).randint(0, stride - 1)
    g = torch.randn(bs[0].flat_numel, generator=torch.Generator(device=DEV).manual_seed(78), device=DEV) * 1e-3
    g[bs[0].offsets[0]: bs[0].offsets[0] + bs[0].numels[0]] = \
        designed_big_gradient(bs[0].numels[0], k, stride, start, 100, top=40.0).to(DEV)
    outs = []
    for b in bs:
        b.grad_flat.copy_(g)
        b.compress()
        outs.append(b.decompress().clone())
    torch.cuda.synchronize()
    ia, it = bs[0].infos(), bs[1].infos()
    assert ia[0]["branch"] == "resample" and ia[0]["candidates"] > 262144, ia[0]
    assert ia[0]["tie_rule"] != "set" and ia[0]["tie_rule"] == it[0]["tie_rule"], (ia[0], it[0])
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    sa, st = bs[0].transmitted()["big"], bs[1].transmitted()["big"]
    assert torch.equal(sa[1], st[1])
    assert np.array_equal(bits(sa[0].cpu().numpy()), bits(st[0].cpu().numpy()))
    for name in bs[0].names:
        assert torch.equal(bs[0].velocity_of(name).view(torch.int32), bs[1].velocity_of(name).view(torch.int32))
        assert torch.equal(bs[0].momentum_of(name).view(torch.int32), bs[1].momentum_of(name).view(torch.int32))
