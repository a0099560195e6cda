"""Parity at the bench's own size: the 1e9-element flat bucket (BASELINE configs[3])
stepped through dgc.bucket.DGCBucket exactly as bench.py steps it (the same fresh
gradient per step, seed 0xD6C + step, ratio 0.001, nesterov), compared with the numpy oracle
after EVERY step: the transmitted indices (in order) and values, momentum and
velocity, and the decompressed dense gradient, all bit for bit. The steady state the
bench times — K1's speculative candidate lists serving the selection, spilled lists,
the trunc branch — is reached and recorded."""
import random
import sys

import numpy as np
import pytest
import torch

from oracle import dgc_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CH = 1 << 27   # host comparisons in 512 MB chunks


def _equal_bits(gpu, host):
    n = host.size
    for c0 in range(0, n, CH):
        c1 = min(n, c0 + CH)
        if not np.array_equal(gpu[c0:c1].cpu().numpy().view(np.uint32), host[c0:c1].view(np.uint32)):
            return False
    return True


@pytest.mark.timeout(1200)
def test_flat_1b_bucket_steps_match_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.empty_cache()   # what earlier tests left cached
    free, _ = torch.cuda.mem_get_info()
    if free < 40 * 2 ** 30:
        pytest.skip("needs ~40 GiB of free HBM")
    from dgc.bucket import DGCBucket
    N, steps = 10 ** 9, 10
    b = DGCBucket(N, compress_ratio=1e-3, momentum=0.9, nesterov=True, device=DEV, seed=42, fill="sparse")
    attrs = O.attributes(N, 1e-3)
    rng = random.Random(42)
    g = torch.empty(N, device=DEV)
    out = torch.empty(N, device=DEV)
    m_o = np.zeros(N, np.float32)
    v_o = np.zeros(N, np.float32)
    seen = []
    for s in range(steps):
        _bench_gradient(g, N, 0xD6C + s, bf16=False)   # bench.py's FlatRun, rank 0, step s
        start = rng.randint(0, attrs[4] - 1)
        b.step(g, out)
        torch.cuda.synchronize()
        info = b.last_info()
        ov, oi, oinfo = O.compress_step(g.cpu().numpy(), m_o, v_o, attrs, start, nesterov=True)
        n = info["count"]
        gi = b.payload[b.ioff: b.ioff + 8 * n].view(torch.int64).cpu().numpy()
        gv = b.payload[b.voff: b.voff + 4 * n].view(torch.float32).cpu().numpy()
        assert info["branch"] == oinfo["branch"], (s, info)
        assert np.array_equal(gi, oi), (s, info)
        assert np.array_equal(gv.view(np.uint32), ov.view(np.uint32)), s
        if s % 3 == 2 or s == steps - 1:   # reading flushes the deferred masking: most steps leave it to K1
            assert _equal_bits(b.vec, v_o) and _equal_bits(b.mmt, m_o), s
        dense = np.zeros(N, np.float32)
        dense[oi] = ov    # W = 1: unique indices, scale 1
        assert _equal_bits(out, dense), s
        del dense
        seen.append((info["branch"], info["full_passes"], info["overflow_segments"]))
        print(f"step {s}: {info}", file=sys.stderr, flush=True)
    # the bench's steady state was exercised: selections served by the K1 lists
    assert any(fp == 0 for _, fp, _ in seen[1:]), seen


def _ref_compensate_(g, mmt, vec, chunk=1 << 28):
    """DGCSGDMemory.compensate, nesterov (dgc/memory.py:58-61), as the reference's own
    torch ops — separate add_/mul_ kernels, one rounding each — chunk by chunk."""
    for c0 in range(0, g.numel(), chunk):
        s = slice(c0, min(g.numel(), c0 + chunk))
        mmt[s].add_(g[s]).mul_(0.9)
        vec[s].add_(mmt[s]).add_(g[s])


def _count_ge(vec, t, chunk=1 << 28):
    return sum(int((vec[c0:c0 + chunk].abs() >= t).sum()) for c0 in range(0, vec.numel(), chunk))


def _first_ge(vec, t, limit, chunk=1 << 28):
    """nonzero(|vec| >= t)[:limit] in index order, chunk by chunk (int64)."""
    parts, got = [], 0
    for c0 in range(0, vec.numel(), chunk):
        idx = torch.nonzero(vec[c0:c0 + chunk].abs() >= t).view(-1) + c0
        parts.append(idx[: limit - got])
        got += parts[-1].numel()
        if got >= limit:
            break
    return torch.cat(parts)


def _bench_gradient(g, N, seed, bf16, chunk=1 << 30):
    """bench.py's FlatRun buffer ``seed``: one generator seeded once, randn in 2^30
    chunks, bf16-rounded for the bf16-origin workload — regenerated in place, so the
    test holds one gradient buffer instead of the bench's two."""
    gen = torch.Generator(device=DEV)
    gen.manual_seed(seed)
    for c0 in range(0, N, chunk):
        c1 = min(N, c0 + chunk)
        x = torch.randn(c1 - c0, generator=gen, device=DEV)
        g[c0:c1] = x.to(torch.bfloat16).float() if bf16 else x
        del x


def _equal_chunks(a, b, chunk=1 << 28):
    return all(torch.equal(a[c0:c0 + chunk].view(torch.int32), b[c0:c0 + chunk].view(torch.int32))
               for c0 in range(0, a.numel(), chunk))


@pytest.mark.timeout(1100)
def test_flat_7b_bf16_steps_match_reference_ops():
    """BASELINE configs[4] at full size and at the bench's steady state: N = 7e9 (> 2^32,
    so indices past 32 bits), bf16-origin gradients (dense ties), ratio 1e-4, nesterov,
    EIGHT steps through DGCBucket exactly as bench.py runs it — its two alternating
    gradient buffers (seeds 0xD6C, 0xD6C + 1), its persistent output with the sparse
    re-zero, its sample starts. Checked after every step against the reference's
    algorithm re-run with torch ops on the GPU, chunked (the numpy oracle is too slow at
    7e9): compensate (bit-exact momentum/velocity, compared raw — NOT flushed — so the
    deferred masking rides in the next K1 as in the bench), the sampled threshold (topk
    of the strided samples), the adaptation loop on exact counts, the transmitted
    indices in order and values, the masking, and the decompressed output. The run must
    reach the bench's steady state: selections served by K1's candidate lists
    (full_passes == 0) with K3 reading the sample window list (window_keys > 0)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.empty_cache()   # what earlier tests left cached
    free, _ = torch.cuda.mem_get_info()
    if free < 200 * 2 ** 30:
        pytest.skip("needs ~200 GiB of free HBM")
    from dgc.bucket import DGCBucket
    N, ratio, steps = 7 * 10 ** 9, 1e-4, 8
    b = DGCBucket(N, compress_ratio=ratio, momentum=0.9, nesterov=True, device=DEV, seed=42, fill="sparse")
    numel, k, S, ks, stride = O.attributes(N, ratio)
    assert (b.k, b.stride, b.top_k_samples) == (k, stride, ks)
    g = torch.empty(N, device=DEV)
    mmt_e = torch.zeros(N, device=DEV)
    vec_e = torch.zeros(N, device=DEV)
    out = torch.empty(N, device=DEV)
    rng = random.Random(42)
    U, Lc = O.adapt_bounds(k)
    seen = []
    for s in range(steps):
        _bench_gradient(g, N, 0xD6C + s % 2, bf16=True)
        start = rng.randint(0, stride - 1)
        b.step(g, out)
        torch.cuda.synchronize()
        info = b.last_info()
        _ref_compensate_(g, mmt_e, vec_e)
        samples = vec_e[start::stride].abs()
        t = torch.topk(samples, ks).values.min()
        assert t.view(torch.int32).item() == torch.tensor([info["threshold0"]]).view(torch.int32).item(), s
        del samples
        n = _count_ge(vec_e, t)
        branch = "exhausted"
        for _ in range(10):                                   # dgc/compression.py:128-149
            if n > k:
                branch = "resample" if n > U else "trunc"
                break
            if n < Lc:
                t = t * torch.tensor(0.8, device=DEV)
                n = _count_ge(vec_e, t)
            else:
                branch = "ok"
                break
        assert (branch, n) == (info["branch"], info["candidates"]), (s, info, branch, n)
        if branch == "resample":
            cand = _first_ge(vec_e, t, n)
            order = torch.topk(vec_e[cand].abs().cpu(), k, sorted=False)[1]   # the reference's CPU topk
            want = cand.cpu()[order]
        else:
            want = _first_ge(vec_e, t, min(n, k)).cpu()
        cnt = info["count"]
        gi = b.payload[b.ioff: b.ioff + 8 * cnt].view(torch.int64).cpu()
        gv = b.payload[b.voff: b.voff + 4 * cnt].view(torch.float32).cpu()
        assert torch.equal(gi, want), s
        assert int(gi.max()) >= 2 ** 32 or int(want.max()) < 2 ** 32
        wd = want.to(DEV)
        wv = vec_e[wd].cpu()
        assert torch.equal(gv.view(torch.int32), wv.view(torch.int32)), s
        deferred = branch != "resample"   # the first-k branches leave the zeroing to the next K1
        if deferred:   # raw state (no flush) = the state before DGCSGDMemory.update
            assert _equal_chunks(b._vec, vec_e) and _equal_chunks(b._mmt, mmt_e), s
        vec_e[wd] = 0.0                                       # DGCSGDMemory.update (dgc/memory.py:72-77)
        mmt_e[wd] = 0.0
        if not deferred:
            assert _equal_chunks(b._vec, vec_e) and _equal_chunks(b._mmt, mmt_e), s
        assert torch.equal(out[wd].cpu().view(torch.int32), wv.view(torch.int32))
        assert sum(int(torch.count_nonzero(out[c0:c0 + (1 << 28)])) for c0 in range(0, N, 1 << 28)) == \
            int(torch.count_nonzero(wv))
        seen.append((info["branch"], info["full_passes"], info["window_keys"]))
        print(f"7B step {s}: {info}, max index {int(gi.max())}", file=sys.stderr, flush=True)
    assert _equal_chunks(b.vec, vec_e) and _equal_chunks(b.mmt, mmt_e)   # flushed at the end
    # the bench's steady state: lists serve the selection and K3 reads the window list
    assert any(fp == 0 and wk > 0 for _, fp, wk in seen[2:]), seen
