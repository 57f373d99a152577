"""libhundcrc.so is loaded into processes that already hold PyTorch's own
libamdhip64.so (torch/lib, ROCm 7.0), and the dynamic loader binds the
library's HIP calls to that copy, not to /opt/rocm's (ROCm 7.2).  A HIP entry
point newer than torch's runtime (hipStreamGetId is hip_7.1) links here and
then fails to load on every GPU run: "version `hip_7.1' not found".  This test
checks every versioned HIP symbol the library imports against the symbols
torch's runtime defines."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hunddb_amd", "libhundcrc.so")


def _dynsyms(path):
    out = subprocess.run(["objdump", "-T", path], check=True, capture_output=True, text=True).stdout
    und, defined = set(), set()
    for line in out.splitlines():
        m = re.search(r"\s(\*UND\*|\.text|\S+)\s+[0-9a-f]+\s+(?:\(([^)]+)\)|(\S+))\s+(\S+)$", line)
        if not m or not (m.group(2) or m.group(3) or "").startswith("hip_"):
            continue
        ver = m.group(2) or m.group(3)
        (und if m.group(1) == "*UND*" else defined).add((m.group(4), ver))
    return und, defined


def _torch_hip():
    import torch

    p = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    return p if os.path.exists(p) else None


@pytest.mark.skipif(shutil.which("objdump") is None, reason="objdump not on PATH")
def test_hip_imports_resolve_in_torch_runtime():
    if not os.path.exists(LIB):
        pytest.skip("libhundcrc.so not built")
    hip = _torch_hip()
    if hip is None:
        pytest.skip("torch ships no libamdhip64.so")
    need, _ = _dynsyms(LIB)
    _, have = _dynsyms(hip)
    assert need, "no versioned HIP imports parsed from objdump -T"
    missing = sorted(f"{name}@{ver}" for name, ver in need if (name, ver) not in have)
    assert not missing, f"HIP symbols torch's runtime lacks: {missing}"
