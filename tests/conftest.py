import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "adam-compression_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdgc_hip.so)")
    config.addinivalue_line("markers", "slow: large sizes")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_compress():
    return load_json("compress.json"), np.load(os.path.join(GOLDEN, "compress.npz"))


@pytest.fixture(scope="session")
def golden_decompress():
    return load_json("decompress.json"), np.load(os.path.join(GOLDEN, "decompress.npz"))


@pytest.fixture(scope="session")
def golden_attributes():
    return load_json("attributes.json")


@pytest.fixture(scope="session")
def golden_optimizer():
    return load_json("optimizer.json"), np.load(os.path.join(GOLDEN, "optimizer.npz"))


@pytest.fixture(scope="session")
def golden_half():
    return load_json("half.json"), np.load(os.path.join(GOLDEN, "half.npz"))
