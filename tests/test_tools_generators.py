"""The A/B harness tools/kgrp3.hip builds its variant from the product kernel
source at build time (tools/gen_grp_perm.py: a textual copy with targeted
substitutions; round 3's kgrp4 / gen_grp_fin.py, which timed the
one-block-at-a-time finalise that round 4's paired placement replaced, and
kany3 / gen_any_x.py, whose k_crc_any copy round 4's move of that kernel's
body into a device function retired, are in git history), so a variant
always measures the product's current code.  Each generator asserts the text
it substitutes; this runs each against the current hc_kernels.hip so a product
change that breaks them fails here, not at the next GPU session."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hunddb_amd", "csrc", "hc_kernels.hip")


def _gen(script, tmp_path):
    out = tmp_path / (script + ".inc")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", script), SRC, str(out)], check=True)
    return out.read_text()


def test_gen_grp_perm_applies(tmp_path):
    k = _gen("gen_grp_perm.py", tmp_path)
    assert "void k_crc_grp_perm(" in k and "perm" in k and "nchunks" in k
