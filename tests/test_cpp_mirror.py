"""The C++ mirror of utils/crc (include/hunddb_crc.hpp) compiled against
libhundcrc.so and run: CPU-side drop-ins here, batched GPU entries on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_hunddb_crc")


@pytest.fixture(scope="module")
def binary(hc):
    src = os.path.join(ROOT, "tests", "cpp", "test_hunddb_crc.cpp")
    lib = os.path.join(ROOT, "hunddb_amd")
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O1", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"), src,
                               "-o", BIN, "-L", lib, "-lhundcrc", f"-Wl,-rpath,{lib}"])
    return BIN


def test_cpp_mirror_cpu(binary):
    r = subprocess.run([binary, "cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_cpp_mirror_no_gpu_fails_loudly(binary, hc):
    if hc.device_count() > 0:
        pytest.skip("a gfx950 device is present")
    r = subprocess.run([binary, "nogpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_mirror_gpu(binary, cuda):
    r = subprocess.run([binary, "gpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
