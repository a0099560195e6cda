"""bench.py's launcher contract (CPU): ``--gpus N`` without torchrun spawns N ranks
on 127.0.0.1; under torchrun it must agree with WORLD_SIZE."""
import importlib.util
import os

import pytest

from conftest import REPO


def _bench():
    spec = importlib.util.spec_from_file_location("bench_cli", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_gpus_spawns_ranks_when_not_under_torchrun():
    b = _bench()
    assert b.launch_plan(1, {}) is None
    envs = b.launch_plan(4, {"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]


def test_gpus_must_match_world_size():
    b = _bench()
    assert b.launch_plan(2, {"WORLD_SIZE": "2"}) is None
    with pytest.raises(SystemExit):
        b.launch_plan(8, {"WORLD_SIZE": "1"})


def test_gpus_fail_fast_without_devices():
    b = _bench()
    b.check_devices(1, 1)
    b.check_devices(2, 8)
    with pytest.raises(SystemExit, match="needs 8 visible GPUs"):
        b.check_devices(8, 1)


def test_step_gradients_are_seeded_per_rank_and_step():
    """seed 0xD6C + 1000 * rank + step, one fresh gradient per step."""
    import torch
    b = _bench()
    assert b.gradient_seed(0, 0) == 0xD6C and b.gradient_seed(2, 7) == 0xD6C + 2007
    g1 = b.fill_gradient(torch.empty(5000), b.gradient_seed(0, 3), chunk=1024)
    g2 = b.fill_gradient(torch.empty(5000), b.gradient_seed(0, 3), chunk=1024)
    g3 = b.fill_gradient(torch.empty(5000), b.gradient_seed(0, 4), chunk=1024)
    assert torch.equal(g1, g2) and not torch.equal(g1, g3)
    h = b.fill_gradient(torch.empty(5000), 11, bf16=True)
    assert torch.equal(h, h.to(torch.bfloat16).float())   # bf16-origin values held in fp32


class _FakeFlat:
    def __init__(self, b, n, steps):
        import torch
        self.N = n
        self.grads = [b.fill_gradient(torch.empty(n), b.gradient_seed(0, s)) for s in range(steps)]

    def grad_of(self, i):
        return self.grads[i]


def test_cpu_baseline_times_the_runs_own_step_gradients():
    """bench.cpu_baseline on a small flat bucket: the whole bucket by default, the step
    gradients of the GPU run (here host tensors), one warm-up step."""
    b = _bench()
    wl = dict(kind="flat", numel=200_000, ratio=1e-3, nesterov=True)
    run = _FakeFlat(b, 200_000, 4)
    res = b.cpu_baseline(run, wl, 1e9, 2, 1)
    assert res["kind"] == "port" and res["cores"] == 1 and res["value"] > 0
    assert "the whole 200000-element bucket" in res["sample"] and "steps 1..2" in res["sample"]
    res = b.cpu_baseline(run, wl, 50_000, 2, 1)
    assert "the first 50000 elements" in res["sample"]
