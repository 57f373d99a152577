"""Every SGPR a kernel takes a memory address from is written on every path
from the kernel entry (tools/isa_sgpr_defs.py; DESIGN.md 4.2a, the round-5
fault).

Round 5's fused k_seg_combine (commit 4cd7616: k_crc_grp's body and
k_crc_any's body behind a runtime mode) faulted on the plain fallback.  Its
optimized IR was sound, but hipcc's backend left the implicit-argument pointer
(s[48:49], the source of gridDim.x) written only on the k_crc_grp path; the
plain fallback loaded gridDim.x through the stale pair (profiles/r6/fault/).
This checks the product kernels (hc_kernels.hip, hc_md5.hip) for that
pattern, and that the checker finds it in a CFG of the same shape.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_sgpr_defs as chk  # noqa: E402

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# the fused combine's shape: the pointer pair is written on one side of a
# uniform branch only and read after the join
_BAD = """\t.text
k:  ; @k
; %bb.0:
\ts_load_dword s33, s[0:1], 0x20
\ts_cmp_eq_u32 s33, 3
\ts_cbranch_scc0 .LBB0_2
; %bb.1:
\ts_add_u32 s48, s0, 0x60
\ts_addc_u32 s49, s1, 0
\ts_branch .LBB0_3
.LBB0_2:
                                        ; implicit-def: $sgpr48_sgpr49
\ts_mov_b32 s33, 0
.LBB0_3:
\ts_load_dword s26, s[48:49], 0x0
\ts_endpgm
.Lfunc_end0:
\t.amdhsa_kernel k
\t\t.amdhsa_user_sgpr_count 2
\t.end_amdhsa_kernel
"""


def test_checker_flags_a_pointer_written_on_one_path():
    res = chk.check_text(_BAD)
    assert list(res) == ["k"]
    (no, ins, miss), = res["k"]
    assert ins.startswith("s_load_dword s26, s[48:49]") and miss == [48, 49]


def test_checker_accepts_a_pointer_written_on_both_paths():
    good = _BAD.replace("\ts_mov_b32 s33, 0\n", "\ts_mov_b32 s33, 0\n\ts_add_u32 s48, s0, 0x60\n\ts_addc_u32 s49, s1, 0\n")
    assert chk.check_text(good) == {}


def test_checker_follows_loops():
    # a pair written only inside a loop body, read in the header: undefined on the entry edge
    src = _BAD.replace("\ts_load_dword s26, s[48:49], 0x0\n\ts_endpgm\n",
                       "\ts_load_dword s26, s[48:49], 0x0\n\ts_cbranch_scc1 .LBB0_3\n\ts_endpgm\n")
    assert "k" in chk.check_text(src)


@pytest.mark.parametrize("src", ["hc_kernels.hip", "hc_md5.hip"])
def test_product_kernels_define_every_address_sgpr(tmp_path, src):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not found")
    out = tmp_path / (src + ".s")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "-S",
                        os.path.join(ROOT, "hunddb_amd", "csrc", src), "-o", str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    text = out.read_text()
    assert text.count(".amdhsa_kernel ") >= (8 if src == "hc_kernels.hip" else 4)
    assert chk.check_text(text) == {}
