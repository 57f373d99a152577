"""Row f3: WAL recovery (lsm/wal/wal.go:362-455) through hc_wal_replay.

The product path (one verify batch + parallel block scan + sequential
fragment merge) against the golden replay fixtures and the oracle's
sequential restatement, on WAL images framed exactly as wal.go:177-283
(oracle oc_wal_frame).  Host-only sizes here (< 256 blocks verify on the CPU);
the GPU-verified sizes are in test_gpu_parity.py.
"""
import hashlib

import numpy as np
import pytest

from test_oracle import ERRS, _replay_case_blocks


def test_wal_replay_golden(hc, oracle, golden):
    for name, c in golden["wal_replay"].items():
        blocks = _replay_case_blocks(oracle, golden, c)
        recs, err, bad, pos = hc.wal_replay(blocks, 4096, max_records=c["max_records"])
        assert (0 if err is None else err.code) == ERRS[c["err"]], name
        if err is not None and c["err"] != "truncated":
            assert str(err) == c["err"]
        assert [hashlib.sha256(r).hexdigest() for r in recs] == c["sha256"], name
        assert list(pos) == c["pos"] and bad == c["bad_block"], name


def _image(oracle, seed, nrec, lo=64, hi=20000):
    sizes = [oracle.lib().oc_wal_record_size(seed, i, lo, hi) for i in range(nrec)]
    b, st, _ = oracle.wal_frame(seed, sizes)
    assert len(b) // 4096 < 256, "host-only test: keep the image under the GPU batch threshold"
    return bytearray(b.tobytes()), sizes, st


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_wal_replay_vs_oracle(hc, oracle, seed):
    img, sizes, st = _image(oracle, seed, 120)
    nb = len(img) // 4096
    rng = np.random.default_rng(seed)
    cases = [(0, 4, 0, None)]
    cases += [(int(rng.integers(0, nb)), 4, 0, None) for _ in range(3)]           # start mid-log
    cases += [(0, 4, int(rng.integers(1, 40)), None) for _ in range(3)]            # memtable full
    cases += [(0, 4, 0, int(rng.integers(0, nb))) for _ in range(3)]               # corrupt block
    for sb, so, mr, corrupt in cases:
        view = bytearray(img)
        if corrupt is not None:
            view[corrupt * 4096 + 2000] ^= 0x20
        want, wrc, wbad, wpos = oracle.wal_replay(bytes(view), 4096, sb, so, mr)
        got, err, bad, pos = hc.wal_replay(bytes(view), 4096, sb, so, mr)
        assert (0 if err is None else err.code) == wrc
        assert got == want and pos == wpos and bad == wbad


def test_wal_replay_records_match_writer(hc, oracle):
    """Every record the writer accepted comes back byte-identical, in order."""
    seed = 0x5EED
    img, sizes, st = _image(oracle, seed, 200)
    recs, err, bad, pos = hc.wal_replay(bytes(img), 4096)
    assert err is None and pos == (len(img) // 4096, 4)
    assert len(recs) == st.records
    # regenerate the serialized records the writer framed (oc_wal_frame's byte formula)
    kept = [s for s in sizes if not (4092 < 17 + s <= 4096)]
    assert [len(r) for r in recs] == kept


def test_wal_replay_capacity_resume(hc, oracle):
    """Output capacity smaller than the image: resuming at the returned position
    yields exactly the unlimited replay's records."""
    img, sizes, st = _image(oracle, 9, 150)
    full, err, _, end = hc.wal_replay(bytes(img), 4096)
    assert err is None
    got, pos = [], (0, 4)
    for _ in range(10000):
        part, err, _, pos = hc.wal_replay(bytes(img), 4096, pos[0], pos[1], buf_cap=150_000, slots=7)
        assert err is None
        got += part
        if pos == end:
            break
        assert part, "no progress"
    assert got == full


def test_wal_replay_bad_args(hc):
    with pytest.raises(hc.HundCRCError):
        hc.wal_replay(bytes(4096), 4096, 0, 0)   # start_offset < CRC_SIZE
