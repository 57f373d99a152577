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
    config.addinivalue_line("markers", "default_thresholds: run with the library's own GPU/host crossovers")


LAST_PREFIX = "test_gpu_zz_"  # heavy full-size files: collected after every other test


def pytest_collection_modifyitems(session, config, items):
    """Run the test_gpu_zz_* files (config 5 at 10M records, ~108 GB of host
    memory) after everything else, whatever order the paths were given in, so
    that under -x a failure there cannot hide the parity suite."""
    last = [it for it in items if os.path.basename(str(it.fspath)).startswith(LAST_PREFIX)]
    if last:
        keep = [it for it in items if not os.path.basename(str(it.fspath)).startswith(LAST_PREFIX)]
        items[:] = keep + last


# The GPU tests were written for the round-3 crossover (256 blocks) and keep
# it, so every size they use still runs the GPU batch; the production
# thresholds (hc_util.hpp) have a test of their own
# (test_gpu_parity.py::test_default_thresholds_route).
GPU_TEST_THRESHOLDS = {"HC_ADD_CRCS_GPU_MIN_BLOCKS": "256", "HC_READ_GPU_MIN_BLOCKS": "256",
                       "HC_WAL_GPU_MIN_BLOCKS": "256"}


class Knobs:
    """The library's HC_* settings for one test.  libhundcrc reads them from
    the environment once, at first use (hc_util.hpp: a getenv racing with a Go
    os.Setenv would be a data race), so a test changes them through
    hc_debug_set -- and in the environment too, for the child processes it
    starts -- and they return to the compiled defaults afterwards."""

    def __init__(self, mp):
        self._mp, self._names = mp, set()

    def setenv(self, name, value):
        from hunddb_amd import crc
        self._mp.setenv(name, value)
        crc.debug_set(name, value)
        self._names.add(name)

    def delenv(self, name, raising=False):
        from hunddb_amd import crc
        self._mp.delenv(name, raising=raising)
        crc.debug_set(name, None)
        self._names.add(name)

    def restore(self):
        from hunddb_amd import crc
        for n in self._names:
            crc.debug_set(n, None)


@pytest.fixture
def knobs(monkeypatch):
    k = Knobs(monkeypatch)
    yield k
    k.restore()


@pytest.fixture(autouse=True)
def _gpu_test_thresholds(request, knobs):
    if request.node.get_closest_marker("gpu") is not None and not request.node.get_closest_marker("default_thresholds"):
        for k, v in GPU_TEST_THRESHOLDS.items():
            knobs.setenv(k, v)


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
