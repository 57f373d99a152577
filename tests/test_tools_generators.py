"""The A/B harnesses tools/kgrp3.hip and tools/kany3.hip build their variants
from the product kernel source at build time (tools/gen_grp_perm.py,
tools/gen_any_x.py: textual copies with targeted substitutions; round 3's
kgrp4 / gen_grp_fin.py, which timed the one-block-at-a-time finalise that
round 4's paired placement replaced, are in git history), so a variant
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


def test_gen_any_x_applies(tmp_path):
    k = _gen("gen_any_x.py", tmp_path)
    assert "void k_crc_any_x(" in k
    assert "lds[" not in k and "col[32]" not in k  # the tables and per-lane columns are gone
    assert "xapply(TM" in k and "place_lq(lq, lane" in k
