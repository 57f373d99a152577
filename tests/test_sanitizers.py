"""Sanitizer runs of the host code.

`make -C hunddb_amd sanitize` builds the library's host code twice -- ASan +
UBSan and ThreadSanitizer (`-Xarch_host -fsanitize=...`: device code is never
instrumented) -- and the oracle with ASan + UBSan.  Each test runs a slice of
the CPU suite in a child process with the clang sanitizer runtime preloaded
and the sanitized library selected through HUNDCRC_LIB / HC_ORACLE_LIB:

  * WAL replay (hc_wal.cpp: the three-phase parallel range merge, 16 threads,
    HC_WAL_MIN_RANGE 64 / 3 / 1 so range boundaries cut fragmented records),
  * ReadFromDisk on the host path (hc_read_from_disk),
  * concurrent drop-in calls from many threads (block_manager_test.go:259-349),
  * the Merkle host code (hc_merkle.cpp, parallel level build),
  * the oracle's own tests under its ASan build.

A sanitizer report aborts the child (halt_on_error / abort_on_error), which
fails the test with the report in its message.
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux")


def _runtime(name):
    for d in RT:
        p = os.path.join(d, f"libclang_rt.{name}-x86_64.so")
        if os.path.exists(p):
            return p
    return None


@pytest.fixture(scope="module")
def sanitized():
    if not _runtime("asan") or not _runtime("tsan"):
        pytest.skip("clang sanitizer runtimes not found")
    subprocess.check_call(["make", "-s", "-j", "8", "-C", os.path.join(ROOT, "hunddb_amd"), "sanitize"])
    return {"asan": os.path.join(ROOT, "hunddb_amd", "build-asan", "libhundcrc_asan.so"),
            "tsan": os.path.join(ROOT, "hunddb_amd", "build-tsan", "libhundcrc_tsan.so"),
            "oracle_asan": os.path.join(ROOT, "oracle", "liboracle_asan.so")}


def _run(env_extra, tests):
    env = {k: v for k, v in os.environ.items() if k != "HC_FORCE_GPU"}
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu"]
                       + tests, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, out
    assert " passed" in r.stdout, out
    return r.stdout


HOST_TESTS = ["tests/test_wal_replay.py", "tests/test_abi.py::test_read_from_disk_host",
              "tests/test_abi.py::test_concurrent_small_calls", "tests/test_merkle.py"]


def test_asan_ubsan_host_code(sanitized):
    _run({"LD_PRELOAD": _runtime("asan"), "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
          "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "HUNDCRC_LIB": sanitized["asan"]}, HOST_TESTS)


def test_tsan_host_code(sanitized):
    _run({"LD_PRELOAD": _runtime("tsan"), "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1",
          "HUNDCRC_LIB": sanitized["tsan"]}, HOST_TESTS)


def test_asan_oracle(sanitized):
    # the oracle is plain C built by gcc: gcc's ASan runtime goes first
    gcc_asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(gcc_asan):
        pytest.skip("gcc libasan not found")
    _run({"LD_PRELOAD": gcc_asan, "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
          "HC_ORACLE_LIB": sanitized["oracle_asan"]}, ["tests/test_oracle.py"])


def test_sanitized_builds_are_instrumented(sanitized):
    """The libraries under test really carry the instrumentation."""
    for key, sym in (("asan", "__asan_report"), ("tsan", "__tsan_"), ("oracle_asan", "__asan_report")):
        syms = subprocess.run(["nm", "-D", sanitized[key]], capture_output=True, text=True).stdout
        assert sym in syms, key
