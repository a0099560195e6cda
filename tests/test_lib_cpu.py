"""C-ABI library: loads, exports every symbol include/dgc_hip.h declares, and its
pure-host entry points (layout / workspace sizing) behave. No GPU needed."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "dgc_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dgc_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def L():
    from dgc import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} missing: run __graft_entry__.build()")
    return _lib.lib()


def test_exports_every_declared_symbol(L):
    syms = declared_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(L, s), s


def test_version_and_error(L):
    assert b"gfx950" in L.dgc_version()
    assert isinstance(L.dgc_last_error(), bytes)


def test_payload_layout(L):
    v, i = ctypes.c_int64(), ctypes.c_int64()
    stride = L.dgc_payload_layout(1000, 0, 0, ctypes.byref(v), ctypes.byref(i))
    assert v.value == 16 and i.value == 16 + 4000 and stride >= i.value + 8000 and stride % 256 == 0
    stride16 = L.dgc_payload_layout(1001, 1, 1, ctypes.byref(v), ctypes.byref(i))
    assert v.value == 16 and i.value % 16 == 0 and i.value >= 16 + 2002 and stride16 >= i.value + 4004


def test_workspace_sizes_scale(L):
    small = L.dgc_select_workspace(4096, 4)
    big = L.dgc_select_workspace(10 ** 9, 10 ** 6)
    assert 0 < small < big
    # candidate lists: 6 B per slot, 64 slots per 1024-element segment (0.375 B/elem), the
    # per-segment counters and offsets (~24 B per segment), plus the resample area: 28 B
    # per candidate (queue entry 8, index 8, value 4, key 4, pair slot 4) for up to
    # min(N, 64k - 1) candidates
    assert big < (0.375 + 24 / 1024) * 10 ** 9 * 1.05 + 28 * 64 * 10 ** 6
    assert L.dgc_select_workspace(10 ** 6, 10) < L.dgc_select_workspace(10 ** 6, 1000)
    assert L.dgc_compress_workspace(10 ** 6, 1000, 10309) > L.dgc_select_workspace(10 ** 6, 1000)
    assert L.dgc_decompress_workspace(10 ** 9, 8) > L.dgc_decompress_workspace(10 ** 6, 8)
    # packed: + the regroup area for runs not in ascending order (12 B per entry per rank)
    assert L.dgc_decompress_packed_workspace(10 ** 6, 8, 1000) >= L.dgc_decompress_workspace(10 ** 6, 8) + 8 * 12000


def test_invalid_arguments_fail_without_gpu(L):
    from dgc import _lib
    p = _lib.SelectParams()
    p.numel, p.num_selects, p.num_samples = 10, 20, 10     # k > n
    rc = L.dgc_select(None, None, None, ctypes.byref(p), None, None, None, None, None, 0, 0, None)
    assert rc == 1 and b"num_selects" in L.dgc_last_error()
    p.num_selects, p.idtype = 5, 1
    p.numel = p.num_samples = 2 ** 31 + 5                  # int32 indices cannot address this
    rc = L.dgc_select(None, None, None, ctypes.byref(p), ctypes.c_void_p(16), ctypes.c_void_p(16), None,
                      None, None, 0, 0, None)
    assert rc == 3


def test_batch_desc_validation_without_gpu(L):
    """dgc_batch_workspace sizes a valid batch and refuses bad layouts (no GPU needed)."""
    import ctypes
    from dgc import _lib

    def desc(numels, offsets, flat):
        T = len(numels)
        arr = lambda xs: (ctypes.c_int64 * T)(*xs)   # noqa: E731
        keep = [arr(numels), arr(offsets), arr([max(1, n // 1000) for n in numels]), arr(numels),
                arr([max(1, n // 1000) for n in numels]), arr([1] * T)]
        d = _lib.BatchDesc()
        d.count = T
        d.numel, d.offset, d.num_selects, d.num_samples, d.top_k_samples, d.sample_stride = keep
        d.flat_numel, d.upper_bound, d.lower_bound, d.max_iters, d.resample = flat, 1.3, 0.8, 10, 1
        return d, keep

    d, keep = desc([5000, 3000], [0, 5120], 8192)
    assert L.dgc_batch_workspace(ctypes.byref(d)) > 0
    d, keep = desc([5000, 3000], [0, 5000], 8192)          # offset not a multiple of 1024
    assert L.dgc_batch_workspace(ctypes.byref(d)) == 0
    assert b"multiple of 1024" in L.dgc_last_error()
    d, keep = desc([5000, 3000], [0, 5120], 8000)          # past flat_numel
    assert L.dgc_batch_workspace(ctypes.byref(d)) == 0


def test_resample_replay_width_refusals_without_gpu(L):
    """The nth_element replay packs candidate positions in 32 bits (K5's queue): a tensor
    past that width is refused with DGC_ERR_OVERFLOW before anything runs, on every entry
    point — never a truncated payload. resample=False takes any size, and the
    partial_sort replay (K5b) any N (slots past 2^33)."""
    from dgc import _lib
    OVERFLOW = 3
    # more than 2^32 - 1 candidates: n >= 2^32, k > 2^26 (a 7B bucket at a warmup ratio)
    for n, k, what in ((2 ** 32 + 4096, 2 ** 26 + 1, b"2^32 - 1 candidates"),):
        p = _lib.SelectParams()
        p.numel, p.num_selects, p.num_samples = n, k, n // 100
        p.max_iters, p.resample = 10, 1
        out = ctypes.c_void_p(256)
        rc = L.dgc_select(None, None, None, ctypes.byref(p), out, out, None, None, None, 0, 0, None)
        assert rc == OVERFLOW and what in L.dgc_last_error(), L.dgc_last_error()
        rc = L.dgc_compress_begin(None, None, None, 0.9, 0, 0, 100, ctypes.byref(p), None, None, 0, None)
        assert rc == OVERFLOW and what in L.dgc_last_error()
        T = 1
        arr = lambda xs: (ctypes.c_int64 * T)(*xs)   # noqa: E731
        keep = [arr([n]), arr([0]), arr([k]), arr([n // 100]), arr([max(1, n // 100000)]), arr([100])]
        d = _lib.BatchDesc()
        d.count = T
        d.numel, d.offset, d.num_selects, d.num_samples, d.top_k_samples, d.sample_stride = keep
        d.flat_numel, d.upper_bound, d.lower_bound, d.max_iters, d.resample = n + 4, 1.3, 0.8, 10, 1
        assert L.dgc_batch_workspace(ctypes.byref(d)) == 0 and what in L.dgc_last_error()
        d.resample = 0                                     # no replay: no limit of its own
        assert L.dgc_batch_workspace(ctypes.byref(d)) > 0
    # past 2^33 elements (K5b's slots) and at the candidate limit the replays take the
    # tensor: the width check passes (and the call fails on the null vec after it)
    for n, k in ((2 ** 33 - 1, 2 ** 26), (2 ** 33, 1000), (10 ** 10, 10 ** 6)):
        p = _lib.SelectParams()
        p.numel, p.num_selects, p.num_samples, p.max_iters, p.resample = n, k, n // 100, 10, 1
        out = ctypes.c_void_p(256)
        rc = L.dgc_select(None, None, None, ctypes.byref(p), out, out, None, None, None, 0, 0, None)
        assert rc == 1 and b"null vec" in L.dgc_last_error(), (n, k, L.dgc_last_error())


def test_host_glue_tables_and_rebinding():
    """The batched optimizer's host glue (lib/_dgc_glue.so) on CPU tensors: the pointer
    table with its fallback positions (no gradient, misaligned, non-contiguous), the
    rebinding of p.grad to given views, and the release of every gradient."""
    import torch
    from dgc import _lib
    g = _lib.glue()
    ps = [torch.nn.Parameter(torch.zeros(8, 4)) for _ in range(5)]
    buf = torch.zeros(5 * 32 + 1)
    grads = [torch.randn(8, 4), None, buf[1:33].view(8, 4), torch.randn(4, 8).t(), torch.randn(8, 4)]
    for p, gr in zip(ps, grads):
        p.grad = gr
    tab = (ctypes.c_void_p * 5)()
    assert g.grad_table(ps, ctypes.addressof(tab), 16) == [1, 2, 3]
    assert tab[0] == grads[0].data_ptr() and tab[4] == grads[4].data_ptr()
    assert g.grad_table(ps, ctypes.addressof(tab), 4) == [1, 3]
    views = [buf[i * 32: (i + 1) * 32].view(8, 4) for i in range(5)]
    g.bind_grads(ps, views)
    assert all(p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(ps, views))
    views[2].fill_(3.0)     # the same storage: p.grad sees it
    assert float(ps[2].grad[0, 0]) == 3.0
    g.release_grads(ps)
    assert all(p.grad is None for p in ps)
