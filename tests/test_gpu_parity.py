"""GPU parity: every kernel of libdgc_hip.so against the numpy oracle (bit-exact for
indices, counts, thresholds, state and wire bytes), and the drop-in classes against
the reference-generated golden fixtures. Runs through the C ABI on cuda:0."""
import ctypes
import math
import zlib
import random

import numpy as np
import pytest
import torch

from oracle import dgc_oracle as O
from oracle import synth

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dgc import _lib
    return _lib.lib()


def stream():
    from dgc import _lib
    return _lib.stream_of(DEV)


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({4: np.uint32, 2: np.uint16, 8: np.uint64}[a.dtype.itemsize])


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def check(L, rc):
    assert rc == 0, L.dgc_last_error().decode()


# ----------------------------------------------------------------------------- K1
@pytest.mark.parametrize("nesterov", [True, False])
@pytest.mark.parametrize("n", [1, 3, 4, 1000, 4099, (1 << 20) + 3])
def test_compensate_accumulate_bitexact(L, nesterov, n):
    g0, m0, v0 = synth.gradient(1, n), synth.gradient(2, n), synth.gradient(3, n)
    m, v = m0.copy(), v0.copy()
    tg, tm, tv = to_dev(g0), to_dev(m0), to_dev(v0)
    for step in range(3):
        O.compensate(g0, m, v, 0.9, nesterov, True)
        check(L, L.dgc_compensate(P(tg), P(tm), P(tv), None, n, 0.9, int(nesterov), 1, None, 0, 1, 0, stream()))
    torch.cuda.synchronize()
    assert np.array_equal(bits(tm.cpu().numpy()), bits(m))
    assert np.array_equal(bits(tv.cpu().numpy()), bits(v))


@pytest.mark.parametrize("nesterov", [True, False])
def test_compensate_dense_branch_and_unaligned(L, nesterov):
    n = 100003
    g0, m0 = synth.gradient(4, n + 1), synth.gradient(5, n + 1)
    m = m0[1:].copy()
    want = O.compensate(g0[1:], m, None, 0.9, nesterov, accumulate=False)
    tg, tm = to_dev(g0), to_dev(m0)
    out = torch.empty(n + 1, device=DEV)
    # element offset 1: 4-B aligned only -> scalar path
    check(L, L.dgc_compensate(tg.data_ptr() + 4, tm.data_ptr() + 4, None, out.data_ptr() + 4, n, 0.9,
                              int(nesterov), 0, None, 0, 1, 0, stream()))
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()[1:]), bits(want))
    assert np.array_equal(bits(tm.cpu().numpy()[1:]), bits(m))


@pytest.mark.parametrize("stride,start", [(97, 0), (97, 5), (97, 96), (9, 3), (33, 32), (2, 1), (3, 0)])
@pytest.mark.parametrize("n", [1000003, 4096 * 3 + 1])
def test_compensate_fused_sample(L, n, stride, start):
    g0, m0, v0 = synth.gradient(6, n), synth.gradient(7, n), synth.gradient(8, n)
    m, v = m0.copy(), v0.copy()
    O.compensate(g0, m, v, 0.9, True, True)
    want = O.strided_samples(v, start, stride)
    tg, tm, tv = to_dev(g0), to_dev(m0), to_dev(v0)
    cnt = (n - start + stride - 1) // stride
    samples = torch.full((cnt + 1,), -1.0, device=DEV)
    check(L, L.dgc_compensate(P(tg), P(tm), P(tv), None, n, 0.9, 1, 1, P(samples), start, stride, cnt, stream()))
    torch.cuda.synchronize()
    got = samples.cpu().numpy()
    assert np.array_equal(bits(got[:cnt]), bits(want)) and got[cnt] == -1.0
    assert np.array_equal(bits(tv.cpu().numpy()), bits(v))
    # standalone K2 over the same velocity gives the same samples
    s2 = torch.empty(cnt, device=DEV)
    check(L, L.dgc_sample_strided(P(tv), n, start, stride, P(s2), cnt, stream()))
    torch.cuda.synchronize()
    assert np.array_equal(bits(s2.cpu().numpy()), bits(want))


def test_sample_gather(L):
    n = 50000
    v = synth.gradient(9, n)
    idx = np.random.default_rng(0).integers(0, n, 777)
    out = torch.empty(777, device=DEV)
    tv, ti = to_dev(v), to_dev(idx)
    check(L, L.dgc_sample_gather(P(tv), P(ti), 777, P(out), stream()))
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(np.abs(v[idx])))


# ----------------------------------------------------------------------------- K3
def kth_dev(L, x_np, k):
    x = to_dev(x_np)
    out = torch.empty(1, device=DEV)
    wsz = L.dgc_kth_largest_workspace(x_np.size)
    ws = torch.empty(max(wsz, 256), dtype=torch.uint8, device=DEV)
    check(L, L.dgc_kth_largest(P(x), x_np.size, k, P(out), P(ws), wsz, stream()))
    torch.cuda.synchronize()
    return out.cpu().numpy()[0]


@pytest.mark.parametrize("n", [1, 100, 32768, 32769, 1000000, 10309279])
def test_kth_largest_matches_topk_min(L, n):
    x = synth.gradient(10 + n % 7, n)
    for k in sorted({1, max(1, n // 1000), max(1, n // 97), n}):
        want = O.kth_largest(np.abs(x), k)
        got = kth_dev(L, x, k)
        assert bits(np.float32(got)) == bits(want), (n, k)


@pytest.mark.parametrize("kind", ["ties", "sparse", "bf16"])
def test_kth_largest_ties(L, kind):
    x = synth.gradient(11, 200000, kind)
    for k in (1, 7, 2000, 150000, 200000):
        assert bits(np.float32(kth_dev(L, x, k))) == bits(O.kth_largest(np.abs(x), k)), (kind, k)


def test_kth_largest_specials(L):
    x = synth.gradient(12, 50000)
    x[[5, 77]] = np.inf
    x[100] = -np.inf
    assert kth_dev(L, x, 3) == np.inf and kth_dev(L, x, 4) == O.kth_largest(np.abs(x), 4)
    x[9] = np.nan
    assert np.isnan(kth_dev(L, x, 1000))          # topk ranks NaN first, min propagates it
    small = x[:1000].copy()
    assert np.isnan(kth_dev(L, small, 10))
    z = np.zeros(5000, np.float32)
    z[::2] = -0.0
    assert bits(np.float32(kth_dev(L, z, 17))) == 0   # |-0| == +0


# ----------------------------------------------------------------------------- K4
def select_dev(L, vec_np, mmt_np, thr, attrs, *, upper=1.3, lower=0.8, max_iters=10, resample=True,
               masking=True, fp16=False, int32=False, update_memory=True, sync=1):
    from dgc import _lib
    numel, k, S, ks, stride = attrs
    p = _lib.SelectParams()
    p.numel, p.num_selects, p.num_samples = numel, k, S
    p.upper_count, p.lower_count = O.adapt_bounds(k, upper, lower)
    p.upper, p.lower = upper, lower
    p.max_iters, p.resample, p.masking = max_iters, int(resample), int(masking)
    p.vdtype, p.idtype, p.update_memory = int(fp16), int(int32), int(update_memory)
    tv, tm = to_dev(vec_np), to_dev(mmt_np)
    t0 = torch.tensor([thr], dtype=torch.float32, device=DEV)
    vals = torch.empty(k, dtype=torch.float16 if fp16 else torch.float32, device=DEV)
    idx = torch.empty(k, dtype=torch.int32 if int32 else torch.int64, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    info = torch.zeros(_lib.INFO_BYTES, dtype=torch.uint8, device=DEV)
    wsz = L.dgc_select_workspace(numel, k)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    check(L, L.dgc_select(P(tv), P(tm), P(t0), ctypes.byref(p), P(vals), P(idx), P(cnt), P(info), P(ws), wsz,
                          sync, stream()))
    torch.cuda.synchronize()
    n = int(cnt.item())
    inf = _lib.SelectInfo.from_buffer_copy(info.cpu().numpy().tobytes())
    return (vals.cpu().numpy()[:n], idx.cpu().numpy()[:n], tv.cpu().numpy(), tm.cpu().numpy(),
            _lib.BRANCHES[inf.branch], inf)


SELECT_CASES = [
    # name, n, ratio, kind, scale, extra oracle kwargs
    ("normal_1m", 1000000, 0.001, "normal", 1.0, {}),
    ("normal_2m_r1e-2", 2000003, 0.01, "normal", 1.0, {}),
    ("layered_resample", 300000, 0.001, "layered", 1.0, {}),
    ("layered_overflow", 200000, 0.05, "layered", 1.0, {}),   # dense local candidates: list spill
    ("ties_int", 100000, 0.01, "ties", 1.0, {}),
    ("sparse_zeros", 100000, 0.01, "sparse", 1.0, {}),
    ("bf16", 500000, 0.001, "bf16", 1.0, {}),
    ("noresample", 50000, 0.01, "layered", 1.0, dict(resample=False)),
    ("iters2", 300000, 0.001, "layered", 1.0, dict(max_iters=2)),
    ("iters0", 300000, 0.001, "normal", 1.0, dict(max_iters=0)),
    ("iters20_iterative", 300000, 0.001, "layered", 1.0, dict(max_iters=20)),   # > 16: one recount per step
    ("direct_small", 1500, 0.001, "normal", 1.0, {}),
    ("tail_odd", 4096 * 5 + 3, 0.01, "normal", 1.0, {}),
]


@pytest.mark.parametrize("case", SELECT_CASES, ids=[c[0] for c in SELECT_CASES])
@pytest.mark.parametrize("thr_scale", [1.0, 1.25, 0.85, 3.0])
def test_select_matches_oracle(L, case, thr_scale):
    name, n, ratio, kind, scale, kw = case
    attrs = O.attributes(n, ratio)
    vec = synth.gradient(zlib.crc32(name.encode()) % 1000, n, kind, scale)
    mmt = synth.gradient(zlib.crc32(name.encode()) % 1000 + 1, n)
    start = 3 % attrs[4]
    samples = np.abs(vec[start::attrs[4]]) if attrs[0] != attrs[2] else np.abs(vec)
    t0 = np.float32(O.kth_largest(samples, attrs[3]) * np.float32(thr_scale))
    okw = dict(upper=1.3, lower=0.8, max_iters=kw.get("max_iters", 10), resample=kw.get("resample", True))
    ov, oi, info = O.sparsify(vec, attrs, threshold=t0, **okw)
    for sync in (1, 0):
        gv, gi, gvec, gmmt, branch, inf = select_dev(L, vec, mmt, t0, attrs, sync=sync, **okw)
        assert branch == info["branch"], (name, sync)
        assert inf.recounts == len(info["counts"]) - 1
        assert np.array_equal(gi, oi), (name, sync, branch)
        assert np.array_equal(bits(gv), bits(ov))
        assert bits(np.float32(inf.threshold)) == bits(info["threshold"])
        ev, em = vec.copy(), mmt.copy()
        O.update(em, ev, oi, True)
        assert np.array_equal(bits(gvec), bits(ev)) and np.array_equal(bits(gmmt), bits(em))
    if name == "layered_overflow" and thr_scale == 1.0:
        assert inf.overflow_segments > 0      # the spill path really ran


RESAMPLE_CASES = [
    # name, N, ratio, kind, candidates targeted at the given threshold
    ("lds_only", 400_000, 0.001, "normal", 3_000),          # <= 12288 candidates: LDS phase only
    ("global_phase", 2_000_003, 0.001, "normal", 60_000),   # global-memory partitions first
    ("bf16_ties", 1_000_000, 0.001, "bf16", 20_000),        # dense boundary ties
    ("int_ties", 300_000, 0.002, "ties", 30_000),           # every key tied many times
    ("near_64k", 100_000, 0.001, "normal", 6_390),          # k * 64 > n just barely (nth path)
    ("big", 20_000_000, 0.001, "normal", 1_000_000),        # 1M candidates: many global steps
]


@pytest.mark.parametrize("k5", ["multi", "wg"])
@pytest.mark.parametrize("case", RESAMPLE_CASES, ids=[c[0] for c in RESAMPLE_CASES])
def test_resample_replays_torch_topk(L, case, k5, monkeypatch):
    """K5: the resample's indices are torch.topk(importance[indices], k, sorted=False)'s,
    IN ORDER (dgc/compression.py:134-137), so the payload bytes equal the reference's.
    k5: the global-memory phase (> 12288 candidates) over several co-resident
    workgroups (k_nth_global; by default only for candidate capacities > 262144) or
    inside the one-workgroup kernel."""
    monkeypatch.setenv("DGC_K5_GLOBAL", k5)
    name, n, ratio, kind, target = case
    attrs = O.attributes(n, ratio)
    k = attrs[1]
    vec = synth.gradient(zlib.crc32(name.encode()) % 997, n, kind)
    mmt = synth.gradient(5, n)
    imp = np.abs(vec)
    t0 = np.float32(np.partition(imp, n - target)[n - target])
    ov, oi, info = O.sparsify(vec, attrs, threshold=t0)
    assert info["branch"] == "resample" and info["counts"][0] < 64 * k, info["counts"]
    cand = np.flatnonzero(imp >= t0)
    want = cand[torch.topk(torch.from_numpy(imp[cand]), k, 0, largest=True, sorted=False)[1].numpy()]
    assert np.array_equal(oi, want)                       # the oracle is torch's topk
    for sync in (1, 0):
        gv, gi, gvec, gmmt, branch, inf = select_dev(L, vec, mmt, t0, attrs, sync=sync)
        assert branch == "resample" and inf.tie_rule == 1, (name, sync)
        assert np.array_equal(gi, want), (name, sync)
        assert np.array_equal(bits(gv), bits(vec[want])), (name, sync)
        ev, em = vec.copy(), mmt.copy()
        O.update(em, ev, want, True)
        assert np.array_equal(bits(gvec), bits(ev)) and np.array_equal(bits(gmmt), bits(em))


PARTIAL_SORT_CASES = [
    # name, N, ratio, kind, candidates (>= 64k: torch's topk takes its partial_sort path)
    ("normal", 300_000, 0.001, "normal", 40_000),
    ("bf16_ties", 300_000, 0.001, "bf16", 40_000),          # boundary + inner ties: heap layout decides
    ("int_ties", 400_000, 0.002, "ties", 120_000),
    ("k4096_bf16", 4_096_000, 0.001, "bf16", 300_000),
    ("k5000_normal", 5_000_000, 0.001, "normal", 400_000),  # k > 4096 (round 2's LDS heap limit)
    ("k5000_bf16", 5_000_000, 0.001, "bf16", 400_000),
    ("k16383_bf16", 16_383_000, 0.001, "bf16", 1_100_000),  # the heap's last all-LDS size
    ("k20000_ties", 20_000_000, 0.001, "ties", 1_400_000),  # nodes past the LDS levels: global memory
    ("vgg_fc6_bf16", 102_760_448, 0.001, "bf16", 7_000_000),  # VGG-16-BN fc6: k = 102,761
]


def _torch_topk_order(imp, cand, k):
    """indices[topk(importance[indices], k, sorted=False)[1]] with torch's own CPU topk —
    the reference's op (dgc/compression.py:134-137), order included."""
    return cand[torch.topk(torch.from_numpy(imp[cand]), k, 0, largest=True, sorted=False)[1].numpy()]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", PARTIAL_SORT_CASES, ids=[c[0] for c in PARTIAL_SORT_CASES])
def test_resample_partial_sort_path(L, case):
    """candidates >= 64k (a sampled threshold >= 64x too low): torch's CPU topk runs
    partial_sort — heap select + sort_heap — and emits the top k in descending value
    order, equal keys (and which boundary ties survive) as the heap's exact layout
    decides. K5b replays it for every k (heap nodes past the 14 LDS levels in global
    memory): the same indices in the same order as torch.topk itself, tied keys included."""
    name, n, ratio, kind, target = case
    attrs = O.attributes(n, ratio)
    k = attrs[1]
    vec = synth.gradient(zlib.crc32(name.encode()) % 991, n, kind)
    mmt = synth.gradient(78, n)
    imp = np.abs(vec)
    t0 = np.float32(np.partition(imp, n - target)[n - target])
    cand = np.flatnonzero(imp >= t0)
    assert cand.size >= 64 * k and cand.size > math.floor(1.3 * k), (cand.size, k)
    want = _torch_topk_order(imp, cand, k)
    if n <= 5_000_000:   # the oracle's restatement (pure Python heap) agrees with torch, order included
        ov, oi, info = O.sparsify(vec, attrs, threshold=t0)
        assert info["branch"] == "resample" and np.array_equal(oi, want)
    if kind != "normal":   # the case exercises ties among the transmitted keys
        assert np.unique(imp[want]).size < k, name
    for sync in (1, 0):
        gv, gi, gvec, gmmt, branch, inf = select_dev(L, vec, mmt, t0, attrs, sync=sync)
        assert branch == "resample" and inf.tie_rule == 1, (name, sync)
        assert np.array_equal(gi, want), (name, sync)
        assert np.array_equal(bits(gv), bits(vec[want])), (name, sync)
        ev, em = vec.copy(), mmt.copy()
        O.update(em, ev, want, True)
        assert np.array_equal(bits(gvec), bits(ev)) and np.array_equal(bits(gmmt), bits(em))


@pytest.mark.timeout(600)
def test_resample_partial_sort_path_past_2_32():
    """The partial_sort replay on a tensor of N > 2^32 elements: heap entries carry
    33-bit element indices. A sparse velocity (200k nonzeros, bf16-rounded: dense ties,
    a quarter of them past index 2^32), k = 3,000, every nonzero a candidate (>= 64k):
    the payload's indices equal torch.topk's over the candidates, in order, and exactly
    those slots of vec / mmt are zeroed."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    if free < 60 * 2 ** 30:
        pytest.skip("needs ~60 GiB of free HBM")
    from dgc import _lib
    L = _lib.lib()
    N, k, M = (1 << 32) + (1 << 28), 3000, 200_000
    gen = torch.Generator(device=DEV)
    gen.manual_seed(4242)
    # M distinct positions: 3/4 below 2^32, 1/4 above
    lo = torch.randint(0, 1 << 32, (M * 3 // 4 + 1000,), generator=gen, device=DEV).unique()[: M * 3 // 4]
    hi = torch.randint(1 << 32, N, (M // 4 + 1000,), generator=gen, device=DEV).unique()[: M - lo.numel()]
    pos = torch.cat([lo, hi]).sort().values
    vals = torch.randn(pos.numel(), generator=gen, device=DEV).to(torch.bfloat16).float()
    vals[vals == 0] = 1.0
    vec = torch.zeros(N, device=DEV)
    mmt = torch.zeros(N, device=DEV)
    vec[pos] = vals
    mmt[pos] = torch.randn(pos.numel(), generator=gen, device=DEV) + 3.0
    p = _lib.SelectParams()
    p.numel, p.num_selects, p.num_samples = N, k, N // 100
    p.upper_count, p.lower_count = O.adapt_bounds(k)
    p.upper, p.lower, p.max_iters, p.resample, p.masking = 1.3, 0.8, 10, 1, 1
    p.vdtype, p.idtype, p.update_memory = 0, 0, 1
    t0 = torch.tensor([float(vals.abs().min())], device=DEV)
    out_v = torch.empty(k, device=DEV)
    out_i = torch.empty(k, dtype=torch.int64, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    info = torch.zeros(_lib.INFO_BYTES, dtype=torch.uint8, device=DEV)
    wsz = L.dgc_select_workspace(N, k)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    check(L, L.dgc_select(P(vec), P(mmt), P(t0), ctypes.byref(p), P(out_v), P(out_i), P(cnt), P(info), P(ws),
                          wsz, 0, stream()))
    torch.cuda.synchronize()
    inf = _lib.SelectInfo.from_buffer_copy(info.cpu().numpy().tobytes())
    assert _lib.BRANCHES[inf.branch] == "resample" and inf.tie_rule == 1 and inf.candidates == pos.numel(), inf
    imp = vals.abs().cpu()
    want = pos.cpu()[torch.topk(imp, k, 0, largest=True, sorted=False)[1]]
    assert int(cnt.item()) == k
    got = out_i.cpu()
    assert torch.equal(got, want)
    assert int(want.max()) >= 1 << 32 and np.unique(imp.numpy()[np.isin(pos.cpu().numpy(), want.numpy())]).size < k
    wv = torch.zeros(N, device=DEV)
    wv[pos] = vals
    assert torch.equal(out_v.cpu().view(torch.int32), wv[want.to(DEV)].cpu().view(torch.int32))
    assert int(torch.count_nonzero(vec[want.to(DEV)])) == 0 and int(torch.count_nonzero(mmt[want.to(DEV)])) == 0
    assert int(torch.count_nonzero(vec)) == pos.numel() - k and int(torch.count_nonzero(mmt)) == pos.numel() - k


@pytest.mark.timeout(900)
def test_resample_partial_sort_path_past_2_33():
    """The partial_sort replay on a tensor of N = 2^33 + 2^28 elements, past the 33-bit
    element index a heap entry can carry: entries then carry one of k slots, recycled as
    entries replace the root, and the slot -> element index map beside them. 200k bf16-
    rounded nonzeros (dense ties), a quarter past 2^33, k = 3,000, every nonzero a
    candidate (>= 64k): the payload equals torch.topk's over the candidates, in order,
    and exactly those slots of vec / mmt are zeroed (the reference takes any N:
    dgc/compression.py:124-137)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    if free < 100 * 2 ** 30:
        pytest.skip("needs ~100 GiB of free HBM")
    from dgc import _lib
    L = _lib.lib()
    N, k, M = (1 << 33) + (1 << 28), 3000, 200_000
    gen = torch.Generator(device=DEV)
    gen.manual_seed(4343)
    lo = torch.randint(0, 1 << 33, (M * 3 // 4 + 1000,), generator=gen, device=DEV).unique()[: M * 3 // 4]
    hi = torch.randint(1 << 33, N, (M // 4 + 1000,), generator=gen, device=DEV).unique()[: M - lo.numel()]
    pos = torch.cat([lo, hi]).sort().values
    vals = torch.randn(pos.numel(), generator=gen, device=DEV).to(torch.bfloat16).float()
    vals[vals == 0] = 1.0
    vec = torch.zeros(N, device=DEV)
    mmt = torch.zeros(N, device=DEV)
    vec[pos] = vals
    mmt[pos] = torch.randn(pos.numel(), generator=gen, device=DEV) + 3.0
    p = _lib.SelectParams()
    p.numel, p.num_selects, p.num_samples = N, k, N // 100
    p.upper_count, p.lower_count = O.adapt_bounds(k)
    p.upper, p.lower, p.max_iters, p.resample, p.masking = 1.3, 0.8, 10, 1, 1
    p.vdtype, p.idtype, p.update_memory = 0, 0, 1
    t0 = torch.tensor([float(vals.abs().min())], device=DEV)
    out_v = torch.empty(k, device=DEV)
    out_i = torch.empty(k, dtype=torch.int64, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    info = torch.zeros(_lib.INFO_BYTES, dtype=torch.uint8, device=DEV)
    wsz = L.dgc_select_workspace(N, k)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    check(L, L.dgc_select(P(vec), P(mmt), P(t0), ctypes.byref(p), P(out_v), P(out_i), P(cnt), P(info), P(ws),
                          wsz, 0, stream()))
    torch.cuda.synchronize()
    inf = _lib.SelectInfo.from_buffer_copy(info.cpu().numpy().tobytes())
    assert _lib.BRANCHES[inf.branch] == "resample" and inf.tie_rule == 1 and inf.candidates == pos.numel(), inf
    imp = vals.abs().cpu()
    want = pos.cpu()[torch.topk(imp, k, 0, largest=True, sorted=False)[1]]
    assert int(cnt.item()) == k
    assert torch.equal(out_i.cpu(), want)
    assert int(want.max()) >= 1 << 33 and np.unique(imp.numpy()[np.isin(pos.cpu().numpy(), want.numpy())]).size < k
    assert torch.equal(out_v.cpu().view(torch.int32), vals.cpu()[torch.searchsorted(pos.cpu(), want)].view(torch.int32))
    assert int(torch.count_nonzero(vec[want.to(DEV)])) == 0 and int(torch.count_nonzero(mmt[want.to(DEV)])) == 0
    assert int(torch.count_nonzero(vec)) == pos.numel() - k and int(torch.count_nonzero(mmt)) == pos.numel() - k
    del vec, mmt, ws
    torch.cuda.empty_cache()


@pytest.mark.parametrize("fp16,int32,masking,update", [(True, True, True, True), (False, True, False, True),
                                                        (True, False, True, False)])
def test_select_wire_and_memory_flags(L, fp16, int32, masking, update):
    n, ratio = 65537, 0.01
    attrs = O.attributes(n, ratio)
    vec = synth.gradient(31, n, "normal", 30000.0)      # fp16 overflow -> inf, like torch
    mmt = synth.gradient(32, n)
    t0 = O.kth_largest(np.abs(vec[::attrs[4]]), attrs[3])
    ov, oi, info = O.sparsify(vec, attrs, threshold=t0)
    wv, wi = O.wire_cast(ov, oi, fp16, int32)
    gv, gi, gvec, gmmt, branch, _ = select_dev(L, vec, mmt, t0, attrs, fp16=fp16, int32=int32, masking=masking,
                                               update_memory=update)
    assert gi.dtype == wi.dtype and np.array_equal(gi, wi)
    assert np.array_equal(bits(gv), bits(wv))
    ev, em = vec.copy(), mmt.copy()
    if update:
        O.update(em, ev, oi, masking)
    assert np.array_equal(bits(gvec), bits(ev)) and np.array_equal(bits(gmmt), bits(em))


# ----------------------------------------------------------------------------- drop-in
def quiet(fn, *a, **kw):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **kw)


def test_dropin_compress_against_goldens(L, golden_compress):
    from dgc.compression import DGCCompressor
    from dgc.memory import DGCSGDMemory
    meta, arrays = golden_compress
    for name, case in meta.items():
        N = case["N"]
        extra = case["extra"]
        mem = DGCSGDMemory(momentum=0.9, nesterov=case["nesterov"], momentum_masking=case["masking"])
        comp = quiet(DGCCompressor, case["ratio"], memory=mem, fp16_values=case["fp16"],
                     int32_indices=case["int32"], resample=case["resample"], **extra)
        param = torch.zeros(N, device=DEV)
        quiet(mem.initialize, [("w", param)])
        quiet(comp.initialize, [("w", param)])
        attrs = tuple(case["attrs"])
        m_o, v_o = np.zeros(N, np.float32), np.zeros(N, np.float32)
        random.seed(42)
        okw = dict(resample=case["resample"], max_iters=extra.get("max_adaptation_iters", 10))
        for s, step in enumerate(case["per_step"]):
            g = synth.gradient(step["seed"], N, case["kind"], case["scale"])
            state = random.getstate()
            start = random.randint(0, attrs[4] - 1) if attrs[0] != attrs[2] else 0
            random.setstate(state)
            (vals, idx), ctx = comp.compress(to_dev(g), "w")
            ov, oi, info = O.compress_step(g, m_o, v_o, attrs, start, nesterov=case["nesterov"],
                                           momentum_masking=case["masking"], **okw)
            wv, wi = O.wire_cast(ov, oi, case["fp16"], case["int32"])
            gi = idx.view(-1).cpu().numpy()
            gv = vals.view(-1).cpu().numpy()
            key = f"{name}/s{s}"
            assert comp.last_info()["branch"] == info["branch"], key
            assert np.array_equal(gi, wi), key
            assert np.array_equal(bits(gv), bits(wv)), key
            assert np.array_equal(bits(mem.momentums["w"].cpu().numpy()), bits(m_o)), key
            assert np.array_equal(bits(mem.velocities["w"].cpu().numpy()), bits(v_o)), key
            # the reference's own payload, in its order (resample included: K5), and state
            assert np.array_equal(gi, arrays[key + "/indices"]), key
            assert np.array_equal(bits(gv), bits(arrays[key + "/values"])), key
            assert synth.digest(mem.velocities["w"].cpu().numpy()) == step["vec_sha"], key
            assert synth.digest(mem.momentums["w"].cpu().numpy()) == step["mmt_sha"], key
            # decompress at W = 1 back into the gradient buffer
            out = comp.decompress(comp.synchronize(comp.communicate((vals, idx), "w", "Average")), ctx)
            dense = out.view(-1).cpu().numpy()
            want = O.decompress([wv], [wi], N, 1)
            assert np.array_equal(bits(dense), bits(want)), key


def test_dropin_decompress_against_goldens(L, golden_decompress):
    from dgc.compression import DGCCompressor
    meta, arrays = golden_decompress
    for name, case in meta.items():
        N, W = case["N"], case["W"]
        for s in range(case["steps"]):
            vals = [arrays[f"{name}/s{s}/r{q}/values"] for q in range(W)]
            idxs = [arrays[f"{name}/s{s}/r{q}/indices"] for q in range(W)]
            want = np.zeros(N, np.float32)
            nz = arrays[f"{name}/s{s}/dec_nz_idx"]
            want[nz] = arrays[f"{name}/s{s}/dec_nz_val"]
            comp = quiet(DGCCompressor, case["ratio"], fp16_values=case["fp16"], int32_indices=case["int32"])
            comp.world_size = W
            quiet(comp.initialize, [("w", (N, [N]))])
            grad = torch.full((N,), 7.0, device=DEV)
            ctx = ("w", N, [N], torch.float32, torch.int64, grad)
            cat_v, cat_i = to_dev(np.concatenate(vals)), to_dev(np.concatenate(idxs))
            # (a) runs detected on device (reference-format input, resample order included)
            out = comp.decompress([cat_v, cat_i], ctx)
            assert np.array_equal(bits(out.cpu().numpy()), bits(want)), (name, s, "detect")
            assert synth.digest(out.cpu().numpy()) == case["per_step"][s]["dense_sha"]
            # (b) host-known run offsets, as our synchronize provides: each rank's run
            #     ascending, as our compress emits it (resample payloads of the reference
            #     come in topk order; indices are unique per rank, so sorting is exact)
            from dgc.compression import _Gathered
            order = [np.argsort(i, kind="stable") for i in idxs]
            cat_v = to_dev(np.concatenate([v[o] for v, o in zip(vals, order)]))
            cat_i = to_dev(np.concatenate([i[o] for i, o in zip(idxs, order)]))
            g = _Gathered([cat_v.view(-1, 1), cat_i.view(-1, 1)])
            g.run_offsets = list(np.cumsum([0] + [len(v) for v in vals]))
            grad.fill_(3.0)
            out = comp.decompress(g, ctx)
            assert np.array_equal(bits(out.cpu().numpy()), bits(want)), (name, s, "offsets")


def test_decompress_packed_and_repeats(L):
    from dgc import _lib
    N, W, cap = 100000, 4, 3000
    rng = np.random.default_rng(5)
    stride = L.dgc_payload_layout(cap, 0, 0, None, None)
    voff, ioff = 16, 16 + 4 * cap
    payload = np.zeros(W * stride, np.uint8)
    vals, idxs = [], []
    for r in range(W):
        c = int(rng.integers(0, cap))
        i = np.sort(rng.choice(N, c, replace=False)).astype(np.int64)
        v = rng.standard_normal(c).astype(np.float32)
        base = r * stride
        payload[base: base + 8] = np.frombuffer(np.int64(c).tobytes(), np.uint8)
        payload[base + voff: base + voff + 4 * c] = np.frombuffer(v.tobytes(), np.uint8)
        payload[base + ioff: base + ioff + 8 * c] = np.frombuffer(i.tobytes(), np.uint8)
        vals.append(v)
        idxs.append(i)
    want = O.decompress(vals, idxs, N, W)
    grad = torch.empty(N, device=DEV)
    wsz = L.dgc_decompress_packed_workspace(N, W, cap)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    tp = to_dev(payload)
    check(L, L.dgc_decompress_packed(P(tp), W, stride, cap, 0, 0, P(grad), N, 1.0 / W, P(ws), wsz,
                                     stream()))
    torch.cuda.synchronize()
    assert np.array_equal(bits(grad.cpu().numpy()), bits(want))
    # one non-decreasing run with repeated indices: sequential order within the repeats
    i = np.sort(rng.integers(0, 5000, 20000)).astype(np.int64)
    v = rng.standard_normal(20000).astype(np.float32)
    want = O.decompress([v], [i], 5000, 1)
    grad = torch.empty(5000, device=DEV)
    offs = (ctypes.c_int64 * 2)(0, 20000)
    wsz = L.dgc_decompress_workspace(5000, 1)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    tv, ti = to_dev(v), to_dev(i)
    check(L, L.dgc_decompress(P(tv), 0, P(ti), 0, 20000, offs, 1, P(grad), 5000, 1.0, P(ws), wsz,
                              stream()))
    torch.cuda.synchronize()
    assert np.array_equal(bits(grad.cpu().numpy()), bits(want))
    # out-of-range indices are ignored and flagged
    bad = np.array([-1, 3, 5000], np.int64)
    offs = (ctypes.c_int64 * 2)(0, 3)
    tv, tb = to_dev(np.ones(3, np.float32)), to_dev(bad)
    check(L, L.dgc_decompress(P(tv), 0, P(tb), 0, 3, offs, 1, P(grad), 5000,
                              1.0, P(ws), wsz, stream()))
    st = ctypes.c_int32(0)
    check(L, L.dgc_decompress_status(P(ws), ctypes.byref(st), stream()))
    assert st.value == 1 and grad[3].item() == 1.0 and grad.sum().item() == 1.0


def _packed(L, runs, cap, fp16, int32):
    """Pack per-rank (values, indices) runs into the padded allgather layout."""
    vd, idt = (1 if fp16 else 0), (1 if int32 else 0)
    vo, io = ctypes.c_int64(0), ctypes.c_int64(0)
    stride = L.dgc_payload_layout(cap, vd, idt, ctypes.byref(vo), ctypes.byref(io))
    payload = np.zeros(len(runs) * stride, np.uint8)
    for r, (v, i) in enumerate(runs):
        base = r * stride
        v = v.astype(np.float16 if fp16 else np.float32)
        i = i.astype(np.int32 if int32 else np.int64)
        payload[base: base + 8] = np.frombuffer(np.int64(len(i)).tobytes(), np.uint8)
        payload[base + vo.value: base + vo.value + v.nbytes] = np.frombuffer(v.tobytes(), np.uint8)
        payload[base + io.value: base + io.value + i.nbytes] = np.frombuffer(i.tobytes(), np.uint8)
    return payload, stride, vd, idt


@pytest.mark.parametrize("N,W,cap,overlap,fp16,int32,shuffled", [
    (1_000_003, 1, 1000, 0.0, False, False, 0),     # single run: thread per entry
    (1_000_003, 1, 1000, 0.0, True, True, 0),
    (1_000_003, 2, 1000, 0.5, False, False, 0),     # wave per super-chunk, cross-rank duplicates
    (1_000_003, 8, 1000, 0.3, True, False, 0),
    (1_000_000, 4, 10000, 0.2, False, False, 0),    # ~160 per chunk: overflow to the staged workgroup path
    (300_000, 8, 30000, 0.3, False, True, 0),       # denser: the workgroup path's LDS accumulate
    (50_000, 5, 20000, 0.9, False, False, 0),       # > kStage entries per chunk: LDS accumulate
    # runs in a resample's topk order (not ascending): regrouped by chunk, same sums
    (1_000_003, 1, 1000, 0.0, False, False, 1),
    (1_000_003, 2, 1000, 0.5, False, False, 1),     # rank 0 shuffled only
    (1_000_003, 8, 1000, 0.3, True, True, 2),       # every rank shuffled
    (300_000, 8, 30000, 0.3, False, False, 2),      # crowded chunks after regrouping
])
def test_sparse_scatter_matches_dense_decompress(L, N, W, cap, overlap, fp16, int32, shuffled):
    """dgc_fill_zero + dgc_scatter_packed == dgc_decompress_packed == the oracle, bit for bit."""
    rng = np.random.default_rng(N + W)
    shared = np.sort(rng.choice(N, cap, replace=False))
    runs = []
    for r in range(W):
        c = int(rng.integers(cap // 2, cap + 1))
        own = rng.choice(N, c, replace=False)
        pick = rng.random(c) < overlap
        idx = np.unique(np.where(pick, shared[:c], own))[:c]
        v = rng.standard_normal(idx.size).astype(np.float32)
        if shuffled == 2 or (shuffled == 1 and r == 0):
            o = rng.permutation(idx.size)
            v, idx = v[o], idx[o]
        runs.append((v, idx.astype(np.int64)))
    payload, stride, vd, idt = _packed(L, runs, cap, fp16, int32)
    wv = [v.astype(np.float16).astype(np.float32) if fp16 else v for v, _ in runs]
    want = O.decompress(wv, [i for _, i in runs], N, W)
    tp = to_dev(payload)
    wsz = L.dgc_decompress_packed_workspace(N, W, cap)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    dense = torch.full((N,), float("nan"), device=DEV)
    check(L, L.dgc_decompress_packed(P(tp), W, stride, cap, vd, idt, P(dense), N, 1.0 / W, P(ws), wsz, stream()))
    sparse = torch.full((N,), float("nan"), device=DEV)
    check(L, L.dgc_fill_zero(P(sparse), N, stream()))
    check(L, L.dgc_scatter_packed(P(tp), W, stride, cap, vd, idt, P(sparse), N, 1.0 / W, P(ws), wsz, stream()))
    st = ctypes.c_int32(-1)
    check(L, L.dgc_decompress_status(P(ws), ctypes.byref(st), stream()))
    torch.cuda.synchronize()
    assert st.value == (2 if shuffled else 0)
    assert np.array_equal(bits(dense.cpu().numpy()), bits(want))
    assert np.array_equal(bits(sparse.cpu().numpy()), bits(want))


@pytest.mark.parametrize("N,W,cap,fp16,int32,shuffled", [
    (1_000_003, 1, 1000, False, False, 0),
    (500_000, 4, 3000, True, True, 1),
    (300_000, 8, 30000, False, False, 2),
])
def test_decompress_over_previous_output(L, N, W, cap, fp16, int32, shuffled):
    """dgc_decompress_packed_over (and its two halves, dgc_clear_packed +
    dgc_scatter_packed_cleared): a persistent output that holds the previous payload's
    decompress is re-zeroed at those indices only; the result equals the dense
    decompress of the new payload bit for bit, over overlapping / disjoint / shuffled
    runs and three steps."""
    rng = np.random.default_rng(N + 7 * W)
    wsz = L.dgc_decompress_packed_workspace(N, W, cap)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    out = torch.full((N,), float("nan"), device=DEV)
    prev = None
    for step in range(3):
        runs = []
        for r in range(W):
            c = int(rng.integers(cap // 2, cap + 1))
            idx = np.sort(rng.choice(N if step != 1 else N // 3, c, replace=False))   # step 1: a crowded prefix
            v = rng.standard_normal(idx.size).astype(np.float32)
            if shuffled == 2 or (shuffled == 1 and r == 0):
                o = rng.permutation(idx.size)
                v, idx = v[o], idx[o]
            runs.append((v, idx.astype(np.int64)))
        payload, stride, vd, idt = _packed(L, runs, cap, fp16, int32)
        tp = to_dev(payload)
        wv = [v.astype(np.float16).astype(np.float32) if fp16 else v for v, _ in runs]
        want = O.decompress(wv, [i for _, i in runs], N, W)
        if prev is None:
            check(L, L.dgc_decompress_packed(P(tp), W, stride, cap, vd, idt, P(out), N, 1.0 / W, P(ws), wsz,
                                             stream()))
        elif step == 1:
            check(L, L.dgc_decompress_packed_over(P(tp), P(prev), W, stride, cap, vd, idt, P(out), N, 1.0 / W,
                                                  P(ws), wsz, stream()))
        else:   # the same in two calls (the engine issues the clear on a side stream)
            check(L, L.dgc_clear_packed(P(prev), W, stride, cap, vd, idt, P(out), N, P(ws), wsz, stream()))
            check(L, L.dgc_scatter_packed_cleared(P(tp), W, stride, cap, vd, idt, P(out), N, 1.0 / W, P(ws), wsz,
                                                  stream()))
        st = ctypes.c_int32(-1)
        check(L, L.dgc_decompress_status(P(ws), ctypes.byref(st), stream()))
        torch.cuda.synchronize()
        assert st.value == (2 if shuffled else 0), step
        assert np.array_equal(bits(out.cpu().numpy()), bits(want)), step
        prev = tp
    assert L.dgc_decompress_packed_over(P(prev), P(prev), W, stride, cap, vd, idt, P(out), N, 1.0, P(ws), wsz,
                                        stream()) != 0


@pytest.mark.parametrize("lead", [0, 1, 3])
def test_multi_run_decompress_into_offset_view(L, lead):
    """W = 4 runs decompressed into grad = buf[lead:]: with lead != 0 the 64-B granules
    straddle the 4096-element chunks, so lone entries must fall back to word stores at
    chunk edges (k_scatter_waves writes whole granules only inside its super-chunk)."""
    N, W, cap = 600_000, 4, 1500   # ~40 entries per 4096-element chunk: the wave path, granule stores on
    rng = np.random.default_rng(lead + 40)
    runs = []
    for r in range(W):
        idx = np.sort(rng.choice(N, cap, replace=False))
        idx[:8] = np.arange(4090, 4106)[r::2][:8] if r < 2 else idx[:8]   # entries around a chunk edge
        idx = np.unique(idx)
        runs.append((rng.standard_normal(idx.size).astype(np.float32), idx.astype(np.int64)))
    payload, stride, vd, idt = _packed(L, runs, cap, False, False)
    want = O.decompress([v for v, _ in runs], [i for _, i in runs], N, W)
    tp = to_dev(payload)
    wsz = L.dgc_decompress_packed_workspace(N, W, cap)
    ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
    buf = torch.full((N + lead,), float("nan"), device=DEV)
    out = buf[lead:]
    check(L, L.dgc_decompress_packed(P(tp), W, stride, cap, vd, idt, P(out), N, 1.0 / W, P(ws), wsz, stream()))
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(want))
    if lead:
        assert bool(torch.isnan(buf[:lead]).all())   # nothing written before the view


def test_sparse_scatter_flags_out_of_range(L):
    N, cap = 10_000, 8
    for W in (1, 3):
        runs = [(np.ones(3, np.float32), np.array([-1, 3, N], np.int64))] + \
               [(np.ones(2, np.float32), np.array([3, 7], np.int64))] * (W - 1)
        payload, stride, vd, idt = _packed(L, runs, cap, False, False)
        tp = to_dev(payload)
        wsz = L.dgc_decompress_packed_workspace(N, W, cap)
        ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)
        out = torch.empty(N, device=DEV)
        check(L, L.dgc_fill_zero(P(out), N, stream()))
        check(L, L.dgc_scatter_packed(P(tp), W, stride, cap, vd, idt, P(out), N, 1.0, P(ws), wsz, stream()))
        st = ctypes.c_int32(-1)
        check(L, L.dgc_decompress_status(P(ws), ctypes.byref(st), stream()))
        assert st.value & 1, W
        assert out[3].item() == float(W) and out.sum().item() == float(W + (W - 1))


def test_decompress_unsorted_falls_back_to_stable_order(L):
    from dgc.compression import DGCCompressor
    N = 3000
    rng = np.random.default_rng(6)
    i = rng.integers(0, N, 5000).astype(np.int64)          # thousands of descents, repeats
    v = rng.standard_normal(5000).astype(np.float32)
    want = O.decompress([v], [i], N, 2)
    comp = quiet(DGCCompressor, 0.01)
    comp.world_size = 2
    quiet(comp.initialize, [("w", (N, [N]))])
    grad = torch.zeros(N, device=DEV)
    out = comp.decompress([to_dev(v), to_dev(i)], ("w", N, [N], torch.float32, torch.int64, grad))
    assert np.array_equal(bits(out.cpu().numpy()), bits(want))


def test_memory_update_and_dense_branch(L):
    from dgc.compression import DGCCompressor
    from dgc.memory import DGCSGDMemory
    mem = DGCSGDMemory(momentum=0.9, nesterov=True)
    comp = quiet(DGCCompressor, 0.01, memory=mem, fp16_values=True)
    b = torch.zeros(1000, device=DEV)
    quiet(mem.initialize, [("b", b)])
    g = synth.gradient(40, 1000)
    t, ctx = comp.compress(to_dev(g), "b")                  # dense: fp16 cast only
    assert t.dtype == torch.float16
    out = comp.decompress(t, ctx)                           # upcast + compensate(accumulate=False)
    m = np.zeros(1000, np.float32)
    want = O.compensate(g.astype(np.float16).astype(np.float32), m, None, 0.9, True, accumulate=False)
    assert np.array_equal(bits(out.cpu().numpy()), bits(want))
    mem.update("b", (torch.tensor([1, 5, -1], device=DEV),))
    mm = mem.momentums["b"].cpu().numpy()
    assert mm[1] == 0 and mm[5] == 0 and mm[-1] == 0 and mm[2] != 0


def test_generic_path_uniform_sampling_and_plain_memory(L):
    """strided_sample=False and the no-op Memory go through compensate -> _sparsify -> update."""
    from dgc.compression import DGCCompressor
    from dgc.memory import Memory
    N = 200000
    comp = quiet(DGCCompressor, 0.001, memory=Memory)
    quiet(comp.initialize, [("w", (N, [N]))])
    g = synth.gradient(41, N)
    tg = to_dev(g)
    (vals, idx), ctx = comp.compress(tg, "w")
    attrs = O.attributes(N, 0.001)
    random.seed(0)
    info = comp.last_info()
    ov, oi, oinfo = O.sparsify(g, attrs, threshold=info["threshold0"])
    assert np.array_equal(idx.view(-1).cpu().numpy(), oi) and np.array_equal(tg.cpu().numpy(), g)
    torch.manual_seed(3)
    comp2 = quiet(DGCCompressor, 0.001, memory=Memory, strided_sample=False)
    quiet(comp2.initialize, [("w", (N, [N]))])
    (v2, i2), _ = comp2.compress(tg, "w")
    t0 = comp2.last_info()["threshold0"]
    torch.manual_seed(3)
    sidx = torch.randint(0, N, (attrs[2],), device=DEV).cpu().numpy()
    assert np.float32(t0) == O.kth_largest(np.abs(g[sidx]), attrs[3])
    ov, oi, _ = O.sparsify(g, attrs, threshold=t0)
    assert np.array_equal(i2.view(-1).cpu().numpy(), oi)


# ----------------------------------------------------------------------------- full size
@pytest.mark.parametrize("N", [100_000_000])
def test_large_bucket_properties(L, N):
    """Size-independent properties at a large flat bucket, plus bit-exact state vs numpy."""
    from dgc.compression import DGCCompressor
    from dgc.memory import DGCSGDMemory
    mem = DGCSGDMemory(momentum=0.9, nesterov=True)
    comp = quiet(DGCCompressor, 0.001, memory=mem)
    p = torch.zeros(N, device=DEV)
    quiet(mem.initialize, [("w", p)])
    quiet(comp.initialize, [("w", p)])
    g = torch.randn(N, generator=torch.Generator(device=DEV).manual_seed(5), device=DEV)
    random.seed(42)
    (vals, idx), ctx = comp.compress(g, "w")
    info = comp.last_info()
    k = comp.attributes["w"][2]
    i = idx.view(-1)
    assert info["count"] == i.numel() <= k and i.numel() >= 0.8 * k
    assert bool((i[1:] > i[:-1]).all())                            # ascending, unique
    vec = mem.velocities["w"]
    assert bool((vec[i] == 0).all()) and bool((mem.momentums["w"][i] == 0).all())
    # reconstruct the pre-masking velocity (nesterov, first step: vec = g*0.9 + g)
    v_np = g.cpu().numpy()
    m_np = np.zeros(N, np.float32)
    vv = np.zeros(N, np.float32)
    O.compensate(v_np, m_np, vv, 0.9, True)
    ii = i.cpu().numpy()
    assert np.array_equal(bits(vals.view(-1).cpu().numpy()), bits(vv[ii]))
    start = random.Random(42).randint(0, comp.attributes["w"][5] - 1)
    t0 = O.kth_largest(np.abs(vv[start::comp.attributes["w"][5]]), comp.attributes["w"][4])
    assert bits(np.float32(info["threshold0"])) == bits(t0)
    ov, oi, _ = O.sparsify(vv, O.attributes(N, 0.001), threshold=t0)
    assert np.array_equal(ii, oi)
    O.update(m_np, vv, oi)
    assert np.array_equal(bits(vec.cpu().numpy()), bits(vv))
    out = comp.decompress(comp.synchronize(comp.communicate((vals, idx), "w", "Average")), ctx)
    dense = out.view(-1)
    assert int((dense != 0).sum()) == int((vals != 0).sum()) and bool((dense[i] == vals.view(-1)).all())


# ----------------------------------------------------------------------------- bucket engine
@pytest.mark.parametrize("N,ratio,kind,scales,fill", [
    (3_000_003, 0.001, "normal", [1, 1, 1, 1, 1], "inline"),  # lists serve steps 2+ (tail segment spills)
    (3_000_003, 0.001, "normal", [1, 1, 1], "allgather"),
    (2_000_000, 0.001, "normal", [1, 1, 0.1, 0.1, 3], "inline"),   # scale drop: speculation fails
    (1_048_576, 0.05, "layered", [1, 1, 1], "inline"),         # dense candidates: lists spill, re-reads
    (500_000, 0.01, "bf16", [1, 1, 1, 1], "inline"),
    (1_000_000, 0.001, "normal", [1, 3, 9, 27], "inline"),     # fast growth: K1 lists overflow -> dropped
    (3_000_003, 0.001, "normal", [1, 1, 1, 1, 1], "sparse"),  # persistent output: sparse re-zero
    (1_048_576, 0.05, "layered", [1, 1, 1, 0.1], "sparse"),
    (1_000_000, 0.001, "normal", [1, 3, 9, 27, 1], "sparse+poke"),   # out written in place: dense fallback
    (1_000_000, 0.001, "normal", [1, 1, 1, 1], "sparse+alias"),      # out is the gradient buffer itself
    (5_000_000, 0.001, "normal", [1, 1, 1, 1, 1], "sparse"),   # > 32K samples: K3 reads K1's window list
    (5_000_000, 0.001, "normal", [1, 1, 0.1, 0.1, 3], "inline"),   # the window misses after the drop
])
@pytest.mark.parametrize("shape", [None, "quarter"])
def test_bucket_steps_match_oracle(L, N, ratio, kind, scales, fill, shape, monkeypatch):
    """DGCBucket (speculative K1 lists, DGC_SYNC_DEVICE, side-stream zero fill + sparse
    scatter, the dense decompress, or the sparse re-zero of a persistent output) vs the
    oracle, step by step."""
    if shape:   # the emit kernel of >= 256 groups (k_emit), forced at these sizes
        monkeypatch.setenv("DGC_EMIT_SHAPE", shape)
    poke = fill.endswith("+poke")
    alias = fill.endswith("+alias")
    fill = fill.split("+")[0]
    from dgc.bucket import DGCBucket
    b = DGCBucket(N, compress_ratio=ratio, momentum=0.9, nesterov=True, device=DEV, seed=7, fill=fill)
    attrs = O.attributes(N, ratio)
    m_o, v_o = np.zeros(N, np.float32), np.zeros(N, np.float32)
    rng = random.Random(7)
    out = torch.full((N,), float("nan"), device=DEV)   # the fill must clear it
    served_by_lists = windowed = 0
    for s, sc in enumerate(scales):
        g = synth.gradient(300 + s, N, kind, float(sc))
        start = rng.randint(0, attrs[4] - 1) if attrs[0] != attrs[2] else 0
        if alias:   # the reference's in-place layout: decompress into the gradient compressed;
            # written through .data, which leaves out's version counter alone, so only the
            # storage-aliasing guard keeps the sparse re-zero off
            out.data.copy_(to_dev(g))
            b.step(out, out)
        else:
            b.step(to_dev(g), out)
        torch.cuda.synchronize()
        info = b.last_info()
        ov, oi, oinfo = O.compress_step(g, m_o, v_o, attrs, start, nesterov=True)
        n = int(b.payload[:8].view(torch.int64).item())
        gi = b.payload[b.ioff: b.ioff + 8 * n].view(torch.int64).cpu().numpy()
        gv = b.payload[b.voff: b.voff + 4 * n].view(torch.float32).cpu().numpy()
        assert info["branch"] == oinfo["branch"], (s, info)
        assert np.array_equal(gi, oi), (s, info)
        assert np.array_equal(bits(gv), bits(ov)), s
        if s % 2 == 1 or s == len(scales) - 1:   # reading flushes the deferred masking: not every step
            assert np.array_equal(bits(b.vec.cpu().numpy()), bits(v_o)), s
            assert np.array_equal(bits(b.mmt.cpu().numpy()), bits(m_o)), s
        assert np.array_equal(bits(out.cpu().numpy()), bits(O.decompress([ov], [oi], N, 1))), s
        served_by_lists += info["full_passes"] == 0
        windowed += info["window_keys"] > 0
        assert info["window_keys"] == 0 or attrs[2] + 1 > 32768, info   # only multi-block thresholds
        assert bits(np.float32(info["threshold0"])) == bits(oinfo["thresholds"][0]), (s, info)
        if poke and s % 2 == 0:
            out[s:: 97].fill_(7.0)   # an in-place write the next step must not build on
    if scales == [1, 1, 1, 1, 1]:
        # the steady state skips the re-read of vec, and K3's pass over all samples
        assert served_by_lists >= (2 if N == 5_000_000 else 3), (served_by_lists, windowed)
        if N == 5_000_000:
            assert windowed >= 3, (served_by_lists, windowed)


@pytest.mark.parametrize("engine", ["bucket", "batch"])
def test_default_fill_survives_data_writes(L, engine):
    """The default fill ("auto" = the dense zero_()) stays right when the caller writes
    the output through ``.data`` between steps — the reference's own idiom, which
    leaves torch's version counter alone, so only the dense fill can be trusted then
    (the opt-in "sparse" re-zero cannot see such a write)."""
    from dgc.batch import DGCBatch
    from dgc.bucket import DGCBucket
    N, ratio = 1_000_000, 0.001
    attrs = O.attributes(N, ratio)
    m_o, v_o = np.zeros(N, np.float32), np.zeros(N, np.float32)
    rng = random.Random(9)
    if engine == "bucket":
        b = DGCBucket(N, compress_ratio=ratio, momentum=0.9, nesterov=True, device=DEV, seed=9)
        assert b.fill == "inline"
        out = torch.empty(N, device=DEV)
    else:
        b = DGCBatch([("w", (N,))], compress_ratio=ratio, momentum=0.9, nesterov=True, device=DEV, seed=9)
        assert b.fill == "inline"
    for s in range(4):
        g = synth.gradient(40 + s, N, "normal")
        start = rng.randint(0, attrs[4] - 1)
        if engine == "bucket":
            b.step(to_dev(g), out)
            got = out
        else:
            b.grad("w").copy_(to_dev(g))
            got = b.step()[:N]
        torch.cuda.synchronize()
        ov, oi, _ = O.compress_step(g, m_o, v_o, attrs, start, nesterov=True)
        assert np.array_equal(bits(got.cpu().numpy()), bits(O.decompress([ov], [oi], N, 1))), (engine, s)
        got.data.add_(3.0)   # no version bump: the next step must not build on this buffer's zeros


def _same_bits_or_nan(a, b):
    """Bitwise equal, except that any NaN matches any NaN (numpy and the GPU may carry
    different NaN payloads through the momentum arithmetic)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(both_nan | (bits(a) == bits(b))))


@pytest.mark.parametrize("N", [1_000_003, 5_000_000])
@pytest.mark.parametrize("case", ["nan_unsampled", "nan_sampled"])
def test_bucket_nan_inf_gradients_match_oracle(L, case, N):
    """NaN and +-inf gradients through DGCBucket against the oracle: an inf is selected
    like any large value; a NaN is never selected (|NaN| >= t is false) and stays in
    the velocity; a NaN among the strided samples makes the threshold NaN (topk ranks
    it first, min propagates it, dgc/compression.py:123) and nothing is selected,
    through the whole adaptation loop — also when K3 reads K1's sample window list
    (N = 5M: > 32K samples), which must then hold the NaN sample and the infs. (NaN
    inputs: parity against the oracle's restatement of torch's NaN ordering; the
    reference's goldens hold no NaN.)"""
    from dgc.bucket import DGCBucket
    ratio = 0.001
    attrs = O.attributes(N, ratio)
    stride = attrs[4]
    rng = random.Random(11)
    starts = [rng.randint(0, stride - 1) for _ in range(4)]
    free = [r for r in range(stride) if r not in starts]   # residues no step samples
    b = DGCBucket(N, compress_ratio=ratio, momentum=0.9, nesterov=True, device=DEV, seed=11)
    m_o, v_o = np.zeros(N, np.float32), np.zeros(N, np.float32)
    out = torch.empty(N, device=DEV)
    nan_thresholds, inf_sent = 0, 0
    for s, start in enumerate(starts):
        g = synth.gradient(700 + s, N, "normal")
        g[[(1000 + s) * stride + free[0], (2000 + s) * stride + free[1]]] = [np.inf, -np.inf]
        if case == "nan_unsampled":
            g[(500 + s) * stride + free[2]] = np.nan
        elif s in (1, 3):
            g[(300 + s) * stride + start] = np.nan                 # sampled at this step
        b.step(to_dev(g), out)
        torch.cuda.synchronize()
        info = b.last_info()
        ov, oi, oinfo = O.compress_step(g, m_o, v_o, attrs, start, nesterov=True)
        n = int(b.payload[:8].view(torch.int64).item())
        gi = b.payload[b.ioff: b.ioff + 8 * n].view(torch.int64).cpu().numpy()
        gv = b.payload[b.voff: b.voff + 4 * n].view(torch.float32).cpu().numpy()
        assert info["branch"] == oinfo["branch"], (s, info, oinfo)
        assert np.array_equal(gi, oi), (s, info)
        assert _same_bits_or_nan(gv, ov), s
        assert _same_bits_or_nan(np.float32(info["threshold0"]), oinfo["thresholds"][0]), (s, info)
        nan_thresholds += bool(np.isnan(info["threshold0"]))
        inf_sent += int(np.isinf(gv).sum())
        if np.isnan(info["threshold0"]):
            assert n == 0, info
        assert _same_bits_or_nan(b.vec.cpu().numpy(), v_o), s
        assert _same_bits_or_nan(b.mmt.cpu().numpy(), m_o), s
        assert np.array_equal(bits(out.cpu().numpy()), bits(O.decompress([ov], [oi], N, 1))), s
    assert inf_sent > 0
    assert nan_thresholds == (2 if case == "nan_sampled" else 0)


def test_bucket_deferred_masking_equals_immediate(L):
    """The deferred masking (first-k branches leave DGCSGDMemory.update's zeroing to the
    next K1) against the immediate one: identical payloads every step, identical
    momentum/velocity whenever read (a mid-run read flushes, the rest ride in K1)."""
    from dgc.bucket import DGCBucket
    N = 2_000_000
    kw = dict(compress_ratio=0.001, momentum=0.9, nesterov=True, device=DEV, seed=5)
    a = DGCBucket(N, deferred_masking=True, **kw)
    b = DGCBucket(N, deferred_masking=False, **kw)
    out_a, out_b = torch.empty(N, device=DEV), torch.empty(N, device=DEV)
    branches = set()
    for s, sc in enumerate([1, 1, 1, 0.1, 1, 5, 1, 1]):
        g = to_dev(synth.gradient(900 + s, N, "layered" if s % 3 == 0 else "normal", float(sc)))
        a.step(g, out_a)
        b.step(g, out_b)
        torch.cuda.synchronize()
        branches.add(a.last_info()["branch"])
        assert torch.equal(a.payload, b.payload), s
        assert torch.equal(out_a.view(torch.int32), out_b.view(torch.int32)), s
        if s in (3, 7):
            assert torch.equal(a.vec.view(torch.int32), b.vec.view(torch.int32)), s
            assert torch.equal(a.mmt.view(torch.int32), b.mmt.view(torch.int32)), s
    assert len(branches) >= 2, branches


# ----------------------------------------------------------------------------- model gradient sets
@pytest.mark.parametrize("model,fp16,int32,steps", [("resnet50", False, False, 2),    # BASELINE configs[1]
                                                    ("vgg16_bn", True, True, 2)])     # BASELINE configs[2]
def test_model_gradient_set_matches_oracle(L, model, fp16, int32, steps):
    """Every dim>1 tensor of the model's gradient set through the drop-in DGCCompressor
    (ratio 0.001, Nesterov-free memory as configs/dgc sets it), step by step vs the oracle:
    indices, values, branch, momentum and velocity bit-exact; decompress at W=1."""
    from dgc import workloads
    from dgc.compression import DGCCompressor
    from dgc.memory import DGCSGDMemory
    comp_set, _ = workloads.split(getattr(workloads, model)())
    mem = DGCSGDMemory(momentum=0.9)
    comp = quiet(DGCCompressor, 0.001, memory=mem, fp16_values=fp16, int32_indices=int32)
    params = [(n, torch.zeros(s, device=DEV)) for n, s in comp_set]
    quiet(mem.initialize, params)
    quiet(comp.initialize, params)
    state = {n: (np.zeros(p.numel(), np.float32), np.zeros(p.numel(), np.float32)) for n, p in params}
    random.seed(42)
    for s in range(steps):
        for t, (name, p) in enumerate(params):
            N = p.numel()
            attrs = O.attributes(N, 0.001)
            assert tuple(comp.attributes[name][i] for i in (0, 2, 3, 4, 5)) == attrs, name
            g = synth.gradient(1000 * s + t, N, "normal", 1e-3 * (1 + t % 7))
            rs = random.getstate()
            start = random.randint(0, attrs[4] - 1) if attrs[0] != attrs[2] else 0
            random.setstate(rs)
            (vals, idx), ctx = comp.compress(to_dev(g).view(p.shape), name)
            m_o, v_o = state[name]
            ov, oi, info = O.compress_step(g, m_o, v_o, attrs, start, nesterov=False)
            wv, wi = O.wire_cast(ov, oi, fp16, int32)
            key = f"{model}/s{s}/{name}"
            assert comp.last_info()["branch"] == info["branch"], key
            assert np.array_equal(idx.view(-1).cpu().numpy(), wi), key
            assert np.array_equal(bits(vals.view(-1).cpu().numpy()), bits(wv)), key
            assert np.array_equal(bits(mem.momentums[name].view(-1).cpu().numpy()), bits(m_o)), key
            assert np.array_equal(bits(mem.velocities[name].view(-1).cpu().numpy()), bits(v_o)), key
            out = comp.decompress(comp.synchronize(comp.communicate((vals, idx), name, "Average")), ctx)
            assert np.array_equal(bits(out.view(-1).cpu().numpy()), bits(O.decompress([wv], [wi], N, 1))), key
