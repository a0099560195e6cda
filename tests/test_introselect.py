"""The restated CPU topk (oracle/introselect.py) equals torch.topk(sorted=False) —
the call the reference's resample makes (dgc/compression.py:134-137) — in order,
on tie-heavy and continuous inputs, for both libstdc++ paths."""
import numpy as np
import pytest
import torch

from oracle import introselect as I


def _cases(seed, count):
    rng = np.random.default_rng(seed)
    for t in range(count):
        n = int(rng.integers(1, 3000))
        k = int(rng.integers(1, n + 1))
        kind = t % 4
        if kind == 0:
            v = rng.standard_normal(n).astype(np.float32)
        elif kind == 1:
            v = rng.integers(0, int(rng.integers(1, 12)), n).astype(np.float32)
        elif kind == 2:
            v = rng.standard_normal(n).astype(np.float32)
            v = np.round(v * 8) / 8
            v[rng.random(n) < 0.2] *= -1
        else:
            v = np.zeros(n, np.float32)
            v[rng.random(n) < 0.3] = 1.0
        yield v.astype(np.float32), k


@pytest.mark.parametrize("seed", range(4))
def test_topk_order_matches_torch(seed):
    for v, k in _cases(seed, 400):
        want = torch.topk(torch.from_numpy(np.abs(v)), k, 0, largest=True, sorted=False)[1].numpy()
        got = I.topk_order(v, k)
        assert np.array_equal(got, want), (v.size, k)


def test_large_nth_element_path():
    rng = np.random.default_rng(9)
    for n, k in [(200_000, 150_000), (131_072, 100_000), (50_000, 1000)]:
        v = np.round(rng.standard_normal(n).astype(np.float32) * 16) / 16
        want = torch.topk(torch.from_numpy(np.abs(v)), k, 0, largest=True, sorted=False)[1].numpy()
        assert np.array_equal(I.topk_order(v, k), want)


def test_nan_and_inf_keys():
    v = np.array([1, np.nan, 3, np.inf, np.nan, 0, -np.inf, 2], np.float32)
    for k in range(1, v.size + 1):
        want = torch.topk(torch.from_numpy(np.abs(v)), k, 0, largest=True, sorted=False)[1].numpy()
        assert np.array_equal(I.topk_order(v, k), want), k
