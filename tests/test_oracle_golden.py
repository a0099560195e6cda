"""Pin the numpy oracle (oracle/dgc_oracle.py) to the golden fixtures generated from
the reference itself (tests/golden/make_goldens.py). CPU only."""
import random

import numpy as np
import pytest

from oracle import dgc_oracle as O
from oracle import synth


def f32bits(x):
    return int(np.float32(x).view(np.uint32))


def test_attributes_grid(golden_attributes):
    rows = golden_attributes["rows"]
    assert len(rows) > 1000
    for row in rows:
        got = O.attributes(row["numel"], row["ratio"], row["clamped_sample_ratio"])
        assert list(got) == row["attrs"], row


def test_warmup_schedules(golden_attributes):
    for label, sched in golden_attributes["schedules"].items():
        kw = sched["kwargs"]
        base = sched["base_ratio"]
        base = base if base <= 1.0 else 1.0 / base
        E = kw.get("warmup_epochs", -1)
        coeff = kw.get("warmup_coeff")
        if E > 0 and coeff is None:
            coeff = base ** (1.0 / (E + 1))
        for epoch, (ratio, attrs) in enumerate(sched["per_epoch"]):
            r = O.warmup_ratio(base, E, coeff, epoch)
            assert r == ratio, (label, epoch)
            numel, k, S, ks, stride = O.attributes(1000000, r, 0.01)
            assert [k, S, ks, stride] == attrs, (label, epoch)


def test_compress_cases(golden_compress):
    meta, arrays = golden_compress
    for name, case in meta.items():
        N = case["N"]
        attrs = tuple(case["attrs"])
        assert attrs == O.attributes(N, case["ratio"], 0.01)
        mmt = np.zeros(N, np.float32)
        vec = np.zeros(N, np.float32)
        random.seed(42)
        kw = dict(resample=case["resample"], max_iters=case["extra"].get("max_adaptation_iters", 10))
        for s, step in enumerate(case["per_step"]):
            g = synth.gradient(step["seed"], N, case["kind"], case["scale"])
            assert synth.digest(g) == step["input_sha"], "input generator drifted"
            start = random.randint(0, attrs[4] - 1) if attrs[0] != attrs[2] else 0
            if step["start"] is not None:
                assert start == step["start"]
            O.compensate(g, mmt, vec, 0.9, case["nesterov"])
            values, indices, info = O.sparsify(vec, attrs, start, **kw)
            key = f"{name}/s{s}"
            ref_idx = arrays[key + "/indices"].astype(np.int64)
            ref_val = arrays[key + "/values"]
            # threshold sequence and counts, bit-exact
            assert [f32bits(t) for t in info["thresholds"]] == step["threshold_bits"], key
            assert list(info["counts"]) == step["counts"], key
            assert (info["branch"] == "resample") == (step["topk_calls"] == 2), key
            wv, wi = O.wire_cast(values, indices, case["fp16"], case["int32"])
            assert wi.dtype == arrays[key + "/indices"].dtype, key
            # every branch, resample included: indices and values in the reference's order
            assert np.array_equal(wi, arrays[key + "/indices"]), key
            assert np.array_equal(wv.view(np.uint8), ref_val.view(np.uint8)), key
            O.update(mmt, vec, indices, case["masking"])
            assert synth.digest(mmt) == step["mmt_sha"], key
            assert synth.digest(vec) == step["vec_sha"], key
            if key + "/mmt" in arrays:
                assert np.array_equal(mmt.view(np.uint32), arrays[key + "/mmt"].view(np.uint32))
                assert np.array_equal(vec.view(np.uint32), arrays[key + "/vec"].view(np.uint32))
            dense = O.decompress([wv], [wi], N, 1)
            nz = np.flatnonzero(dense.view(np.uint32))
            assert np.array_equal(nz, arrays[key + "/dec_nz_idx"]), key
            assert np.array_equal(dense[nz].view(np.uint32), arrays[key + "/dec_nz_val"].view(np.uint32)), key


def test_decompress_cases(golden_decompress):
    meta, arrays = golden_decompress
    for name, case in meta.items():
        N, W = case["N"], case["W"]
        attrs = O.attributes(N, case["ratio"], 0.01)
        mmts = [np.zeros(N, np.float32) for _ in range(W)]
        vecs = [np.zeros(N, np.float32) for _ in range(W)]
        random.seed(42)
        for s, step in enumerate(case["per_step"]):
            start = random.randint(0, attrs[4] - 1)
            vals, idxs = [], []
            for q in range(W):
                g = synth.gradient(step["seeds"][q], N, case["kind"])
                v, i, info = O.compress_step(g, mmts[q], vecs[q], attrs, start, nesterov=True)
                v, i = O.wire_cast(v, i, case["fp16"], case["int32"])
                rv = arrays[f"{name}/s{s}/r{q}/values"]
                ri = arrays[f"{name}/s{s}/r{q}/indices"]
                assert np.array_equal(i, ri), (name, s, q)
                assert np.array_equal(v.view(np.uint8), rv.view(np.uint8)), (name, s, q)
                vals.append(arrays[f"{name}/s{s}/r{q}/values"])
                idxs.append(arrays[f"{name}/s{s}/r{q}/indices"])
            dense = O.decompress(vals, idxs, N, W)
            assert synth.digest(dense) == step["dense_sha"], (name, s)
            nz = np.flatnonzero(dense.view(np.uint32))
            assert np.array_equal(nz, arrays[f"{name}/s{s}/dec_nz_idx"])


@pytest.mark.parametrize("nesterov", [True, False])
@pytest.mark.parametrize("accumulate", [True, False])
def test_compensate_matches_torch_cpu(nesterov, accumulate):
    """The numpy restatement equals the torch-CPU op sequence of dgc/memory.py:50-70."""
    torch = pytest.importorskip("torch")
    from oracle import torch_cpu
    N = 100003
    g = synth.gradient(1, N)
    m0 = synth.gradient(2, N)
    v0 = synth.gradient(3, N)
    m, v = m0.copy(), v0.copy()
    out = O.compensate(g, m, v, 0.9, nesterov, accumulate)
    tm, tv = torch.from_numpy(m0.copy()), torch.from_numpy(v0.copy())
    tout = torch_cpu.compensate(torch.from_numpy(g), tm, tv, 0.9, nesterov, accumulate)
    assert np.array_equal(out.view(np.uint32), tout.numpy().view(np.uint32))
    assert np.array_equal(m.view(np.uint32), tm.numpy().view(np.uint32))
    assert np.array_equal(v.view(np.uint32), tv.numpy().view(np.uint32))


def test_kth_largest_edge_cases():
    s = np.array([3, 1, 2, 2, 5], np.float32)
    assert O.kth_largest(s, 1) == 5 and O.kth_largest(s, 3) == 2 and O.kth_largest(s, 5) == 1
    assert np.isnan(O.kth_largest(np.array([1, np.nan, 2], np.float32), 1))
    assert O.kth_largest(np.array([np.inf, 1], np.float32), 1) == np.inf
    assert O.adapt_bounds(1000) == (1300, 800)
    assert O.adapt_bounds(3) == (3, 3)       # 3*1.3 = 3.9 -> n > 3 ; 0.8*3 = 2.4 -> n < 3
