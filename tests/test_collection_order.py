"""The GPU suite's order (Next 1): the full-size config-5 file, which
needs ~108 GB of host memory, is collected after every parity test, so that a
failure there under `pytest -m gpu -x` cannot leave the parity suite unreached;
and it fails with the numbers (never skips, never OOMs) when memory is short."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _collect(*args):
    r = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-p", "no:cacheprovider", *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return [ln for ln in r.stdout.splitlines() if "::" in ln]


def test_config5_full_size_collects_last():
    ids = _collect("tests", "-m", "gpu")
    files = [i.split("::")[0] for i in ids]
    heavy = [k for k, f in enumerate(files) if os.path.basename(f).startswith("test_gpu_zz_")]
    assert heavy, "the config-5 full-size tests are missing from the GPU suite"
    assert heavy == list(range(len(ids) - len(heavy), len(ids))), "config 5 must be the last GPU tests"
    assert any("test_gpu_zz_config5_full.py" in f for f in files)
    before = set(files[:heavy[0]])
    for need in ("test_gpu_parity.py", "test_gpu_fuzz.py", "test_gpu_seg.py", "test_gpu_multi.py",
                 "test_gpu_merkle.py", "test_gpu_graphs.py"):
        assert any(f.endswith(need) for f in before), need


def test_config5_last_even_when_named_first():
    # paths given in the "wrong" order: the conftest hook still puts config 5 last
    ids = _collect("tests/test_gpu_zz_config5_full.py", "tests/test_gpu_parity.py", "-m", "gpu")
    files = [os.path.basename(i.split("::")[0]) for i in ids]
    k = files.index("test_gpu_zz_config5_full.py")
    assert all(f == "test_gpu_zz_config5_full.py" for f in files[k:])
    assert "test_gpu_parity.py" in files[:k]


def test_memory_check_fails_loudly(monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_gpu_zz_config5_full as c5
    room, desc = c5.host_memory_room()
    assert room is not None and room > 0 and "MemAvailable" in desc
    c5.require_host_bytes(1 << 20)
    try:
        c5.require_host_bytes(1 << 62)
    except AssertionError as e:
        assert "GiB of host memory" in str(e) and "MemAvailable" in str(e)
    else:
        raise AssertionError("a 4 EiB need passed the host-memory check")
