"""Parity at the steady state the bench times, for the two model-set workloads
(BASELINE configs[1] ResNet-50, configs[2] VGG-16-BN): ``bench.py``'s own ``ModelRun``
— the same ``DGCBatch`` settings, the same x1e-3 ``randn`` gradient set per step (seed
0xD6C + step), the same sample starts (``random.Random(42)``, one draw
per sampled tensor per step), the same persistent output with the sparse re-zero —
stepped 25 times and compared with the oracle after EVERY step, tensor by tensor:

* branch, count, transmitted indices (in order) and wire values (fp16/int32 casts) —
  a resample with an untied k-th key (``DGCBatch``'s default ``resample_order="index"``,
  tie rule "set") lists torch.topk's SET in index order, so there the indices must be
  the oracle's set, ascending, with each index's wire value;
* momentum and velocity as the bench leaves them, i.e. NOT flushed: the first-k
  branches defer ``DGCSGDMemory.update``'s zeroing to the next K1 (so the raw state
  must equal the pre-masking state there), the resample branch masks at once;
* the decompressed output (W = 1) and the dense tensors' ``compensate(accumulate=False)``.

Reference: dgc/compression.py:109-198, dgc/memory.py:50-77. The run must pass through
what the bench's ``selection`` record shows — resamples (the set path, and K5's exact
replay where the k-th key is tied) and full select passes — or the test fails."""
import importlib.util
import os
import random
import sys

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import dgc_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _bench():
    spec = importlib.util.spec_from_file_location("bench_steady", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({4: np.uint32, 2: np.uint16, 8: np.uint64}[a.dtype.itemsize])


@pytest.mark.timeout(1100)
@pytest.mark.parametrize("workload", ["resnet50", "vgg16_bn"])
def test_model_set_bench_steady_state_matches_oracle(workload):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    bench = _bench()
    wl = bench.WORKLOADS[workload]
    steps = 25
    run = bench.ModelRun(wl, 0, 1, DEV, "sparse", nsteps=steps)
    assert run.nbuf == steps
    b = run.b
    assert b.fill == "sparse"
    fp16, int32, nest, ratio = wl["fp16"], wl["int32"], wl["nesterov"], wl["ratio"]
    attrs = [O.attributes(n, ratio) for n in b.numels]
    state = [(np.zeros(n, np.float32), np.zeros(n, np.float32)) for n in b.numels]
    dense_m = np.zeros(run.n_dense, np.float32)
    ref_rng = random.Random(42)
    exact = as_set = full_pass_steps = resample_max = 0
    branches = {}
    for s in range(steps):
        g, gd = run.grad_of(s)
        host = [g[off: off + n].cpu().numpy() for off, n in zip(b.offsets, b.numels)]
        dense_host = gd.cpu().numpy()
        run.step(s)
        torch.cuda.synchronize()
        sent = b.transmitted()
        infos = b.infos()
        raw_m = b._mmt_flat.cpu().numpy()   # not b.mmt_flat: reading that would flush the deferred masking
        raw_v = b._vec_flat.cpu().numpy()
        out = b.out_flat.cpu().numpy()
        full_pass_steps += any(i["full_passes"] for i in infos)
        for t, name in enumerate(b.names):
            N, off, a = b.numels[t], b.offsets[t], attrs[t]
            start = ref_rng.randint(0, a[4] - 1) if a[0] != a[2] else 0
            key = f"{workload}/step{s}/{name}"
            assert start == b.starts[t], key
            m_o, v_o = state[t]
            O.compensate(host[t], m_o, v_o, 0.9, nest)
            ov, oi, oinfo = O.sparsify(v_o, a, start)
            info = infos[t]
            assert info["branch"] == oinfo["branch"], (key, info)
            assert info["count"] == oi.size, (key, info)
            wv, wi = O.wire_cast(ov, oi, fp16, int32)
            gv, gi = sent[name]
            gi, gv = gi.cpu().numpy(), gv.cpu().numpy()
            if info["tie_rule"] == "set":   # topk's set, ascending (the oracle lists topk's order)
                o = np.argsort(oi, kind="stable")
                assert np.array_equal(gi, oi[o]), (key, info)
                assert np.array_equal(bits(gv), bits(wv[o])), key
            else:
                assert np.array_equal(gi, oi), (key, info)
                assert np.array_equal(bits(gv), bits(wv)), key
            deferred = info["branch"] != "resample"   # k_sel_finish: first-k branches defer the masking
            if deferred:   # raw state = the pre-masking state
                assert np.array_equal(bits(raw_v[off: off + N]), bits(v_o)), key
                assert np.array_equal(bits(raw_m[off: off + N]), bits(m_o)), key
            O.update(m_o, v_o, oi)
            if not deferred:
                assert np.array_equal(bits(raw_v[off: off + N]), bits(v_o)), key
                assert np.array_equal(bits(raw_m[off: off + N]), bits(m_o)), key
            assert np.array_equal(bits(out[off: off + N]), bits(O.decompress([wv], [oi], N, 1))), key
            branches[info["branch"]] = branches.get(info["branch"], 0) + 1
            if info["branch"] == "resample":
                exact += info["tie_rule"] == "exact"
                as_set += info["tie_rule"] == "set"
                resample_max = max(resample_max, info["candidates"])
                assert info["tie_rule"] in ("exact", "set"), (key, info)
        # dense tensors: wire cast -> (W = 1 allreduce) -> compensate(accumulate=False)
        src = dense_host.astype(np.float16).astype(np.float32) if fp16 else dense_host
        want = O.compensate(src, dense_m, None, 0.9, nest, accumulate=False)
        assert np.array_equal(bits(run.dense_out.cpu().numpy()), bits(want)), (workload, s)
        print(f"{workload} step {s}: branches so far {branches}, resamples exact {exact} / set {as_set} "
              f"(max {resample_max} candidates), steps with full passes {full_pass_steps}", file=sys.stderr,
              flush=True)
    # the flushed state at the end equals the oracle's
    for t, name in enumerate(b.names):
        m_o, v_o = state[t]
        assert np.array_equal(bits(b.velocity_of(name).reshape(-1).cpu().numpy()), bits(v_o)), name
        assert np.array_equal(bits(b.momentum_of(name).reshape(-1).cpu().numpy()), bits(m_o)), name
    # the bench's dynamics were exercised: resamples (set path) and full select passes
    assert as_set > 0 and full_pass_steps > 0, (branches, exact, as_set, full_pass_steps)
