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
