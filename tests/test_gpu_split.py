"""Split exchange (dgc_payload_split / dgc_scatter_split / dgc_clear_split): the
allgather of dgc/compression.py:200-212 in `parts` collectives, the decompress
(dgc/compression.py:179-194) of each part scattered as it lands.

Single process: W ranks' packed payloads are split on the device, assembled
part-major as the `parts` allgathers would leave them, and scattered phase by phase.
The dense result must be the oracle's sequential index_put_ sums bit for bit, and
after every phase each value already written must be final (a phase never writes an
index whose entries have not all landed).
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle.dgc_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def L():
    from dgc import _lib
    return _lib.lib()


def P(t):
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def check(L, rc):
    assert rc == 0, L.dgc_last_error().decode()


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _rank_payload(L, v, i, cap, vd, idt):
    vo, io = ctypes.c_int64(0), ctypes.c_int64(0)
    stride = L.dgc_payload_layout(cap, vd, idt, ctypes.byref(vo), ctypes.byref(io))
    p = np.zeros(stride, np.uint8)
    v = v.astype(np.float16 if vd else np.float32)
    i = i.astype(np.int32 if idt else np.int64)
    p[:8] = np.frombuffer(np.int64(len(i)).tobytes(), np.uint8)
    p[vo.value: vo.value + v.nbytes] = np.frombuffer(v.tobytes(), np.uint8)
    p[io.value: io.value + i.nbytes] = np.frombuffer(i.tobytes(), np.uint8)
    return torch.from_numpy(p).to(DEV)


def _runs(rng, N, W, cap, overlap, shuffled, full=False, prefix=None):
    shared = np.sort(rng.choice(N, cap, replace=False))
    runs = []
    for r in range(W):
        c = cap if full else int(rng.integers(cap // 2, cap + 1))
        own = rng.choice(prefix or N, c, replace=False)
        pick = rng.random(c) < overlap
        idx = np.unique(np.where(pick, shared[:c], own))[:c]
        v = rng.standard_normal(idx.size).astype(np.float32)
        if shuffled == 2 or (shuffled == 1 and r == W - 1):
            o = rng.permutation(idx.size)
            v, idx = v[o], idx[o]
        runs.append((v, idx.astype(np.int64)))
    return runs


class Split:
    def __init__(self, L, N, W, parts, cap, vd, idt):
        self.L, self.N, self.W, self.parts, self.cap, self.vd, self.idt = L, N, W, parts, cap, vd, idt
        pc = ctypes.c_int64(0)
        self.pbytes = L.dgc_payload_split_layout(cap, parts, vd, idt, ctypes.byref(pc))
        self.pc = pc.value
        self.sbytes = L.dgc_payload_split_bytes(cap, parts, vd, idt)
        assert self.sbytes >= parts * self.pbytes
        self.split = torch.zeros(self.sbytes, dtype=torch.uint8, device=DEV)   # scratch zero at rest
        wsz = L.dgc_decompress_split_workspace(N, W, parts, cap)
        assert wsz > 0
        self.ws = torch.empty(wsz, dtype=torch.uint8, device=DEV)

    def gather(self, runs):
        """Every rank's payload split on the device and placed part-major (the collectives' output)."""
        L, pb, W = self.L, self.pbytes, self.W
        g = torch.zeros(self.parts * W * pb, dtype=torch.uint8, device=DEV)
        heads = []
        for r, (v, i) in enumerate(runs):
            pay = _rank_payload(L, v, i, self.cap, self.vd, self.idt)
            check(L, L.dgc_payload_split(P(pay), self.cap, self.parts, self.vd, self.idt, P(self.split), stream()))
            for p in range(self.parts):
                g[(p * W + r) * pb: (p * W + r + 1) * pb].copy_(self.split[p * pb: (p + 1) * pb])
            heads.append(self.split[: self.parts * pb].view(self.parts, pb)[:, :16].clone().view(torch.int64))
        assert int(self.split[self.parts * pb:].count_nonzero()) == 0   # scratch left zero
        return g, heads

    def scatter(self, g, out, cleared, want=None):
        for p in range(self.parts):
            check(self.L, self.L.dgc_scatter_split(P(g), self.W, self.parts, p, self.cap, self.vd, self.idt, P(out),
                                                   self.N, 1.0 / self.W, int(cleared and p == 0), P(self.ws),
                                                   self.ws.numel(), stream()))
            if want is not None and p < self.parts - 1:   # every value written so far is final
                o = out.cpu().numpy()
                nz = o != 0
                assert np.array_equal(bits(o[nz]), bits(want[nz])), p

    def status(self):
        st = ctypes.c_int32(-1)
        check(self.L, self.L.dgc_decompress_status(P(self.ws), ctypes.byref(st), stream()))
        return st.value


@pytest.mark.parametrize("N,W,parts,cap,overlap,fp16,int32,shuffled", [
    (1_000_003, 2, 2, 1000, 0.5, False, False, 0),
    (1_000_003, 8, 4, 1000, 0.3, True, False, 0),
    (1_000_003, 8, 8, 1001, 0.3, False, True, 0),   # 8 parts of a ragged capacity
    (1_000_000, 4, 2, 10000, 0.2, False, False, 0),   # crowded super-chunks: the overflow path per phase
    (300_000, 8, 3, 30000, 0.3, False, True, 0),
    (1_000_003, 4, 2, 1000, 0.3, False, False, 1),  # the last rank in topk order: its bound is a true minimum
    (300_000, 8, 4, 30000, 0.3, True, True, 2),     # every rank shuffled: everything lands in the last phase
    (50_000, 2, 2, 7, 0.0, False, False, 0),        # fewer entries than parts * chunks
])
def test_split_scatter_matches_oracle(L, N, W, parts, cap, overlap, fp16, int32, shuffled):
    rng = np.random.default_rng(N + 31 * W + parts)
    runs = _runs(rng, N, W, cap, overlap, shuffled)
    vd, idt = int(fp16), int(int32)
    sp = Split(L, N, W, parts, cap, vd, idt)
    g, heads = sp.gather(runs)
    # headers: counts and bounds (the smallest index in the later parts)
    for (v, i), h in zip(runs, heads):
        h = h.cpu().numpy()
        for p in range(parts):
            lo, hi = p * sp.pc, min((p + 1) * sp.pc, len(i))
            assert h[p, 0] == max(0, hi - lo)
            later = i[(p + 1) * sp.pc:]
            assert h[p, 1] == (later.min() if later.size else np.iinfo(np.int64).max)
    wv = [v.astype(np.float16).astype(np.float32) if fp16 else v for v, _ in runs]
    want = O.decompress(wv, [i for _, i in runs], N, W)
    out = torch.full((N,), float("nan"), device=DEV)
    check(L, L.dgc_fill_zero(P(out), N, stream()))
    sp.scatter(g, out, False, want)
    torch.cuda.synchronize()
    assert sp.status() == (2 if shuffled else 0)
    assert np.array_equal(bits(out.cpu().numpy()), bits(want))


@pytest.mark.parametrize("N,W,parts,cap,fp16,int32,shuffled", [
    (1_000_003, 2, 2, 2000, False, False, 0),
    (500_000, 8, 4, 3000, True, True, 1),
])
def test_split_clear_over_previous_output(L, N, W, parts, cap, fp16, int32, shuffled):
    """dgc_clear_split re-zeroes the previous step's split gathered entries; the
    phases then write the new step's: three steps, each the oracle's result."""
    rng = np.random.default_rng(N + parts)
    vd, idt = int(fp16), int(int32)
    sp = Split(L, N, W, parts, cap, vd, idt)
    out = torch.full((N,), float("nan"), device=DEV)
    prev = None
    for step in range(3):
        runs = _runs(rng, N, W, cap, 0.3, shuffled, prefix=N // 3 if step == 1 else None)
        g, _ = sp.gather(runs)
        wv = [v.astype(np.float16).astype(np.float32) if fp16 else v for v, _ in runs]
        want = O.decompress(wv, [i for _, i in runs], N, W)
        if prev is None:
            check(L, L.dgc_fill_zero(P(out), N, stream()))
        else:
            check(L, L.dgc_clear_split(P(prev), W, parts, cap, vd, idt, P(out), N, P(sp.ws), sp.ws.numel(), stream()))
        sp.scatter(g, out, prev is not None)
        torch.cuda.synchronize()
        assert sp.status() == (2 if shuffled else 0), step
        assert np.array_equal(bits(out.cpu().numpy()), bits(want)), step
        prev = g


def test_split_refusals(L):
    assert L.dgc_payload_split_bytes(100, 0, 0, 0) == 0
    assert L.dgc_payload_split_bytes(100, 9, 0, 0) == 0
    assert L.dgc_decompress_split_workspace(1000, 16, 8, 100) == 0   # 128 runs > 64
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device=DEV)
    out = torch.zeros(1000, device=DEV)
    assert L.dgc_scatter_split(P(buf), 2, 2, 2, 100, 0, 0, P(out), 1000, 0.5, 0, P(buf), buf.numel(), stream()) != 0
    assert L.dgc_scatter_split(P(buf), 2, 1, 0, 100, 0, 0, P(out), 1000, 0.5, 0, P(buf), buf.numel(), stream()) != 0
