"""The library's HC_* settings (hc_util.hpp kKnobDefs): every name the header
documents is one the library knows, and the reverse; hc_debug_set takes each
of them and refuses an unknown name (HC_E_ARG).  No GPU needed."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_names():
    text = open(os.path.join(ROOT, "include", "hundcrc.h")).read()
    m = re.search(r"The library reads its HC_\* settings.*?race\):(.*?)\.\s+hc_debug_set", text, re.S)
    assert m, "hundcrc.h: the knob list before hc_debug_set"
    return {n.strip() for n in re.sub(r"[\s*]+", " ", m.group(1)).split(",")}


def _library_names():
    text = open(os.path.join(ROOT, "hunddb_amd", "csrc", "hc_util.hpp")).read()
    m = re.search(r"kKnobDefs\[kKnobCount\] = \{(.*?)\};", text, re.S)
    assert m
    return set(re.findall(r'\{"(HC_[A-Z0-9_]+)"', m.group(1)))


def test_documented_knobs_are_the_library_knobs():
    assert _header_names() == _library_names()


def test_debug_set_takes_every_knob(hc):
    for name in sorted(_library_names()):
        hc.debug_set(name, None)  # the compiled default
    with pytest.raises(hc.HundCRCError):
        hc.debug_set("HC_NO_SUCH_KNOB", "1")
