"""Shared fixtures.  `-m "not gpu"` runs here (no GPU); `-m gpu` on an MI355X."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def hc():
    from hunddb_amd import crc
    crc.lib()
    return crc


@pytest.fixture(scope="session")
def cuda():
    """torch on cuda:0 -- the GPU tests fail (not skip) without a gfx950 device,
    so a GPU run can never pass on a silent fallback."""
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    from hunddb_amd import crc
    assert crc.device_count() >= 1, "no gfx950 device visible to libhundcrc"
    return torch
