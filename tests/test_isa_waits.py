"""The compiled kernels keep the properties their speed rests on (DESIGN.md
4.1a, 4.2a), checked on the gfx950 assembly hipcc emits for the product
source (CPU: hipcc cross-compiles):

* every kernel runs without scratch (private segment 0);
* the 1024-thread streaming kernels fit 4 waves per SIMD (<= 128 VGPRs);
* k_crc_grp's row folds wait for exactly their own row (vmcnt(3): the three
  rows behind it stay in flight);
* k_seg_stream's row folds and window waits count exactly the VMEM ops issued
  after the load they wait for (vmcnt(6): three rows, the event window, the
  group's two stores; vmcnt(7) in the two gapped loops, whose window is two loads),
  and no loop-latch register copies wait for refills
  (round 4 found hipcc copying the loop-carried rows at the latch after small
  unrelated edits; that shows as vmcnt(2)/vmcnt(3) waits before the header);
* k_unframe has no readfirstlane (waterfall) loops around its buffer stores.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not found")
    out = tmp_path_factory.mktemp("isa") / "hc_kernels.s"
    src = os.path.join(ROOT, "hunddb_amd", "csrc", "hc_kernels.hip")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "-S",
                        src, "-o", str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    text = out.read_text()
    kernels = {}
    for m in re.finditer(r"^\t\.amdhsa_kernel (\S+)\n(.*?)\t\.end_amdhsa_kernel", text, re.S | re.M):
        kernels[m.group(1)] = m.group(2)
    bodies = {}
    for name in kernels:
        start = text.index(f"\n{name}:")
        end = text.index(f"\t.amdhsa_kernel {name}\n")
        bodies[name] = text[start:end]
    return kernels, bodies


def _find(names, key):
    hits = [n for n in names if key in n]
    assert hits, f"no kernel matching {key}"
    return hits


def _field(meta, name):
    return int(re.search(rf"\.{name} (\d+)", meta).group(1))


def _waits(body):
    return [int(x) for x in re.findall(r"s_waitcnt vmcnt\((\d+)\)", body)]


def test_no_scratch_anywhere(isa):
    kernels, _ = isa
    assert len(kernels) >= 10
    for name, meta in kernels.items():
        assert _field(meta, "amdhsa_private_segment_fixed_size") == 0, name


def test_streaming_kernels_fit_four_waves_per_simd(isa):
    kernels, _ = isa
    for key in ("k_crc_grp", "k_seg_stream", "k_crc_any", "k_crc_fast", "k_seg_combine"):
        for name in _find(kernels, key):
            assert _field(kernels[name], "amdhsa_next_free_vgpr") <= 128, (name, key)


def test_crc_grp_folds_wait_for_their_row_only(isa):
    _, bodies = isa
    for name in _find(bodies, "k_crc_grp"):
        w = _waits(bodies[name])
        assert w.count(3) >= 3, (name, w)  # the row folds of the group loop


def _stream_loops(body):
    """(latch text before the loop, loop text) of every depth-1 loop whose body
    refills rows (buffer_load_dwordx4 ... nt)."""
    out = []
    for m in re.finditer(r"^(\.LBB\d+_\d+):[ \t]*; =>This Loop Header: Depth=1\n", body, re.M):
        h, label = m.start(), m.group(1)
        back = [b.end() for b in re.finditer(rf"s_c?branch\w* {re.escape(label)}\n", body[h:])]
        if not back:  # (a header whose back edge is a fall-through: not a stream loop)
            continue
        loop = body[h:h + back[-1]]  # to the last back edge
        if re.search(r"buffer_load_dwordx4 .* nt", loop):
            out.append((body[body.rfind("buffer_load_dwordx4", 0, h):h], loop))
    return out


def test_seg_stream_waits_are_exact(isa):
    """The stream loops: the small-gap and the zeroed-gap ones, whose event
    windows are two loads (off[] and len[]), fold at vmcnt(7); the packed one
    at vmcnt(6).  Round 6 instantiates each twice (the batch's own arrays and
    the sorted view's, whose first_ev is read by an asm scalar load so that no
    vmcnt(0) drains the refills once a unit); hipcc may merge the loop headers
    of a pair, so at least the three of round 5 are found."""
    _, bodies = isa
    (name,) = _find(bodies, "k_seg_stream")
    loops = _stream_loops(bodies[name])
    assert 3 <= len(loops) <= 6, len(loops)
    for latch, loop in loops:
        w = _waits(loop)
        exact = 7 if w.count(7) >= 4 else 6
        assert w.count(exact) >= 4, (exact, w)  # the four row folds
        assert not [x for x in w if x < exact - 1], (exact, w)  # no wait drains a refill or the window
        assert not re.search(rf"s_waitcnt vmcnt\([0-{exact - 1}]\)", latch), "loop-latch copies wait for the refills"
    assert sum(1 for _, loop in loops if _waits(loop).count(7) >= 4) >= 2


def test_framing_kernels_have_no_waterfall_loops(isa):
    """k_unframe's buffer stores take their descriptors from wave-uniform values.
    A base computed through a per-lane value makes hipcc wrap the store in a
    readfirstlane loop (s_cbranch_execnz). Round 4's first 8/16 KiB head-store
    variant met that and lost 1.7 points (profiles/r4/r4qq/)."""
    _, bodies = isa
    for name in _find(bodies, "k_unframe"):
        assert "s_cbranch_execnz" not in bodies[name], name
