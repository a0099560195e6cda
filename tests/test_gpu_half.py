"""GPU parity for bf16 / fp16 parameters on the per-tensor drop-in path
(DGCSGDMemory + DGCCompressor, dgc_compensate16 / dgc_select / dgc_mask_indices16 /
dgc_decompress16) against the reference's own 16-bit fixtures (tests/golden/half.*,
generated from /root/reference by make_goldens.py gen_half; the torch-CPU port is
pinned to the same fixtures in test_half_port.py). Bit-exact: transmitted indices in
order, values, the 16-bit momentum / velocity, the decompressed gradient."""
import contextlib
import io
import random

import numpy as np
import pytest
import torch

from oracle import synth

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def quiet(fn, *a, **kw):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **kw)


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({4: np.uint32, 2: np.uint16, 8: np.uint64}[a.dtype.itemsize])


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dgc import _lib
    return _lib.lib()


def _ranks(case):
    from dgc.compression import DGCCompressor
    from dgc.memory import DGCSGDMemory
    dt = getattr(torch, case["dtype"])
    comps, mems = [], []
    for _ in range(case["W"]):
        mem = DGCSGDMemory(momentum=0.9, nesterov=case["nesterov"], momentum_masking=case["masking"])
        comp = quiet(DGCCompressor, case["ratio"], memory=mem, fp16_values=case["fp16"],
                     int32_indices=case["int32"], resample=case["resample"])
        comp.world_size = case["W"]
        prm = torch.zeros(case["N"], dtype=dt, device=DEV)
        quiet(mem.initialize, [("w", prm)])
        quiet(comp.initialize, [("w", prm)])
        comps.append(comp)
        mems.append(mem)
    return comps, mems


@pytest.mark.parametrize("decomp", ["offsets", "reference_format"])
def test_half_dropin_against_reference_goldens(L, golden_half, decomp):
    from dgc.compression import _Gathered
    meta, arrays = golden_half
    for name, case in meta.items():
        dt = getattr(torch, case["dtype"])
        N, W = case["N"], case["W"]
        comps, mems = _ranks(case)
        random.seed(42)
        for s, step in enumerate(case["per_step"]):
            rstate = random.getstate()
            payload, ctxs = [], []
            for q, rk in enumerate(step["ranks"]):
                random.setstate(rstate)
                g = torch.from_numpy(synth.gradient(rk["seed"], N, case["kind"], case["scale"]).copy()).to(dt)
                (vals, idx), ctx = comps[q].compress(g.to(DEV), "w")
                key = f"{name}/s{s}/r{q}"
                assert vals.dtype == getattr(torch, rk["values_dtype"].split(".")[1]), key
                assert np.array_equal(idx.view(-1).cpu().numpy(), arrays[key + "/indices"]), key
                assert np.array_equal(bits(vals.view(-1).float().cpu().numpy()), bits(arrays[key + "/values"])), key
                m = mems[q].momentums["w"].float().cpu().numpy()
                v = mems[q].velocities["w"].float().cpu().numpy()
                assert synth.digest(m) == rk["mmt_sha"], key
                assert synth.digest(v) == rk["vec_sha"], key
                assert mems[q].momentums["w"].dtype == dt and ctx[3] == dt, key
                payload.append((vals.clone(), idx.clone()))
                ctxs.append(ctx)
            want = np.zeros(N, np.float32)
            nz = arrays[f"{name}/s{s}/dec_nz_idx"]
            want[nz] = arrays[f"{name}/s{s}/dec_nz_val"]
            cat_v = torch.cat([p[0] for p in payload])
            cat_i = torch.cat([p[1] for p in payload])
            if decomp == "offsets":   # as our synchronize hands it over: one run per rank
                gath = _Gathered([cat_v, cat_i])
                gath.run_offsets = list(np.cumsum([0] + [p[0].numel() for p in payload]))
                gath.distinct_runs = True
            else:                     # the reference's list of two concatenations
                gath = [cat_v, cat_i]
            ctxs[0][5].fill_(7.0)     # decompress overwrites the gradient buffer
            out = comps[0].decompress(gath, ctxs[0])
            assert out.dtype == dt
            got = out.view(-1).float().cpu().numpy()
            assert np.array_equal(bits(got), bits(want)), (name, s, decomp)
            assert synth.digest(got) == step["dense_sha"], (name, s, decomp)


def test_half_dense_branch_and_state_dict(L):
    """compensate(accumulate=False) on 16-bit state (the dense tensors' branch,
    dgc/memory.py:64-70) against the torch op sequence; state_dict keeps the dtype."""
    from dgc.memory import DGCSGDMemory
    from oracle import torch_cpu as TC
    for dt in (torch.bfloat16, torch.float16):
        for nest in (True, False):
            N = 10007
            mem = DGCSGDMemory(momentum=0.9, nesterov=nest)
            quiet(mem.initialize, [("b", torch.zeros(N, dtype=dt, device=DEV))])
            m_ref = torch.zeros(N, dtype=dt)
            for s in range(3):
                g = torch.from_numpy(synth.gradient(900 + s, N).copy()).to(dt)
                out = mem.compensate(g.to(DEV), "b", accumulate=False)
                want = TC.compensate(g, m_ref, None, 0.9, nest, accumulate=False)
                assert out.dtype == dt
                assert torch.equal(out.cpu().view(torch.int16), want.view(torch.int16)), (dt, nest, s)
                assert torch.equal(mem.momentums["b"].cpu().view(torch.int16), m_ref.view(torch.int16))
            sd = mem.state_dict()
            assert sd["momentums"]["b"].dtype == dt


def test_half_batch_mixed_dtypes_refuse(L):
    import torch.nn as nn
    from dgc.compression import DGCCompressor
    from dgc.memory import DGCSGDMemory
    from dgc.horovod.optimizer import DistributedOptimizer
    model = nn.Sequential(nn.Linear(64, 64), nn.Linear(64, 64).to(torch.bfloat16)).to(DEV)
    mem = DGCSGDMemory(momentum=0.9)
    comp = quiet(DGCCompressor, 0.01, memory=mem)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    with pytest.raises(NotImplementedError, match="share one dtype"):
        DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp, batch=True)


def test_half_batch_against_reference_goldens(L, golden_half):
    """DGCBatch on a 16-bit tensor (the engine of DistributedOptimizer(batch=True) on
    bf16 / fp16 parameters): K1-16 over the flat 16-bit buffers, the selection on the
    fp32 image (dgc_batch_select), the 16-bit masking from the payload and the packed
    16-bit decompress, one DGCBatch per rank — against the reference's own fixtures, every
    case and step, W = 1 to 4: indices in order (an untied resample: the set, ascending),
    values, 16-bit state, dense output."""
    from dgc.batch import DGCBatch
    meta, arrays = golden_half
    for name, case in meta.items():
        dt = getattr(torch, case["dtype"])
        N, W = case["N"], case["W"]
        bs = [DGCBatch([("w", (N,))], compress_ratio=case["ratio"], momentum=0.9, nesterov=case["nesterov"],
                       momentum_masking=case["masking"], resample=case["resample"], fp16_values=case["fp16"],
                       int32_indices=case["int32"], device=DEV, world_size=W, dtype=dt) for _ in range(W)]
        assert tuple(bs[0].attrs[0]) == tuple(case["attrs"][1:]), name
        stride = bs[0].attrs[0][3]
        random.seed(42)
        for s, step in enumerate(case["per_step"]):
            rstate = random.getstate()
            for q, rk in enumerate(step["ranks"]):
                random.setstate(rstate)
                start = random.randint(0, stride - 1) if N != bs[q].attrs[0][1] else 0
                g = torch.from_numpy(synth.gradient(rk["seed"], N, case["kind"], case["scale"]).copy()).to(dt)
                bs[q].grad("w").copy_(g.to(DEV))
                bs[q].compress([start])
                key = f"{name}/s{s}/r{q}"
                vals, idx = bs[q].transmitted()["w"]
                assert vals.dtype == getattr(torch, rk["values_dtype"].split(".")[1]), key
                want_i, want_v = arrays[key + "/indices"], arrays[key + "/values"]
                if bs[q].infos()[0]["tie_rule"] == "set":   # an untied resample: topk's set, index order
                    o = np.argsort(want_i, kind="stable")
                    want_i, want_v = want_i[o], want_v[o]
                assert np.array_equal(idx.cpu().numpy(), want_i), key
                assert np.array_equal(bits(vals.float().cpu().numpy()), bits(want_v)), key
                assert synth.digest(bs[q].momentum_of("w").float().cpu().numpy()) == rk["mmt_sha"], key
                assert synth.digest(bs[q].velocity_of("w").float().cpu().numpy()) == rk["vec_sha"], key
            gathered = torch.cat([b.payload for b in bs])   # the allgather: rank order
            b0 = bs[0]
            b0._gathers = [gathered] * len(b0._gathers) if W > 1 else b0._gathers
            out = b0.decompress().view(-1)[:N]
            assert out.dtype == dt
            got = out.float().cpu().numpy()
            want = np.zeros(N, np.float32)
            want[arrays[f"{name}/s{s}/dec_nz_idx"]] = arrays[f"{name}/s{s}/dec_nz_val"]
            assert np.array_equal(bits(got), bits(want)), (name, s)
            assert synth.digest(got) == step["dense_sha"], (name, s)
