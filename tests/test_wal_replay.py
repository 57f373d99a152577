"""Row f3: WAL recovery (lsm/wal/wal.go:362-455) through hc_wal_replay.

The product path (one verify batch + per-range scan and merge + a short
sequential pass over the ranges + parallel copy-out) against the golden replay fixtures and the oracle's
sequential restatement, on WAL images framed exactly as wal.go:177-283
(oracle oc_wal_frame).  Host-only sizes here (< 256 blocks verify on the CPU);
the GPU-verified sizes are in test_gpu_parity.py.
"""
import hashlib

import numpy as np
import pytest

from test_oracle import ERRS, _replay_case_blocks


@pytest.fixture(params=[64, 3, 1], ids=["range64", "range3", "range1"])
def ranges(knobs, request, monkeypatch):
    """Blocks per parallel range (HC_WAL_MIN_RANGE): 1 and 3 put range
    boundaries inside fragmented records, so the cross-range merge runs."""
    knobs.setenv("HC_WAL_MIN_RANGE", str(request.param))
    return request.param


def test_wal_replay_golden(hc, oracle, golden, ranges):
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
def test_wal_replay_vs_oracle(hc, oracle, seed, ranges):
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


@pytest.mark.parametrize("seed", [4, 5])
def test_wal_replay_end_blocks_give_the_memtable_full_position(hc, oracle, seed, ranges):
    """hc_wal_replay_v's rec_end_block: the block each record completes in.  A
    caller whose memtable.IsFull depends on the keys replays without a limit and
    stops itself; stopping after record j must land where wal.go:392-397 (and
    max_records = j, pinned by the oracle) lands: block end[j-1] + 1, offset 4."""
    img, sizes, st = _image(oracle, seed, 140)
    for sb in (0, 3):
        full, err, _, end, ends, _pend = hc.wal_replay(bytes(img), 4096, sb, 4, end_blocks=True)
        assert err is None and len(ends) == len(full)
        assert (np.diff(ends.astype(np.int64)) >= 0).all() and ends[0] >= sb and ends[-1] < end[0]
        for j in sorted({1, 2, len(full) // 3, len(full) // 2, len(full) - 1, len(full)}):
            want, wrc, _, wpos = oracle.wal_replay(bytes(img), 4096, sb, 4, j)
            assert wrc == 0 and want == full[:j]
            assert wpos == (int(ends[j - 1]) + 1, 4), (sb, j)


@pytest.mark.parametrize("win", [1, 2, 5, 17])
def test_wal_replay_in_windows_equals_one_replay(hc, oracle, win, ranges):
    """How integration/go/lsm/wal/wal_recover_gpu.go replays a long WAL: windows
    of `win` blocks, each starting where the previous one's pending fragments
    start (pend_pos) or at its end.  The records, their end blocks and the final
    position are exactly those of one replay over the whole image."""
    img, sizes, st = _image(oracle, 8, 160)
    nb = len(img) // 4096
    full, err, _, end, ends, pend = hc.wal_replay(bytes(img), 4096, end_blocks=True)
    assert err is None and pend is None
    got, got_ends = [], []
    blk, off = 0, 4
    w = win
    while blk < nb:
        hi = min(nb, blk + w)
        part, err, _, pos, pe, pd = hc.wal_replay(bytes(img[:hi * 4096]), 4096, blk, off, end_blocks=True)
        assert err is None and pos == (hi, 4)
        got += part
        got_ends += pe.tolist()
        if pd is None or hi == nb:
            blk, off, w = hi, 4, win
        elif pd == (blk, off):  # one record longer than the window: widen it
            w *= 2
        else:
            blk, off, w = pd[0], pd[1], win
    assert got == full and got_ends == ends.tolist()


def test_wal_replay_capacity_resume(hc, oracle, ranges):
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


def _random_image(rng, nblocks, bs=4096):
    """Blocks of random FIRST/MIDDLE/LAST/FULL pieces (any order, not only what
    the writer produces), some ending in padding, some filled to the end."""
    import struct
    import zlib
    out = bytearray()
    for _ in range(nblocks):
        b = bytearray(bs)
        off = 4
        while off + 17 < bs:
            if rng.random() < 0.15:  # padding tail
                break
            room = bs - off - 17
            size = int(rng.integers(0, min(room, 1500) + 1)) if rng.random() < 0.8 else room
            typ = int(rng.choice([1, 2, 3, 4]))
            b[off:off + 17] = struct.pack("<QBQ", size, typ, 7)
            b[off + 17:off + 17 + size] = rng.integers(1, 256, size, dtype=np.uint8).tobytes()
            off += 17 + size
        b[0:4] = struct.pack("<I", zlib.crc32(bytes(b[4:])))
        out += b
    return bytes(out)


@pytest.mark.parametrize("seed", range(6))
def test_wal_replay_random_pieces_vs_oracle(hc, oracle, seed, ranges):
    """Arbitrary piece sequences across blocks (FULL between fragments, LAST
    with nothing pending, padding clearing fragments) through the per-range
    merge, against the oracle's sequential restatement of wal.go:362-455;
    with memtable-full stops, start offsets and a corrupt block."""
    rng = np.random.default_rng(100 + seed)
    img = _random_image(rng, 40)
    nb = len(img) // 4096
    for sb, mr, corrupt in [(0, 0, None), (int(rng.integers(1, nb)), 0, None), (0, int(rng.integers(1, 30)), None),
                            (0, 0, int(rng.integers(0, nb)))]:
        view = bytearray(img)
        if corrupt is not None:
            view[corrupt * 4096 + 9] ^= 0x40
        want, wrc, wbad, wpos = oracle.wal_replay(bytes(view), 4096, sb, 4, mr)
        got, err, bad, pos = hc.wal_replay(bytes(view), 4096, sb, 4, mr)
        assert (0 if err is None else err.code) == wrc
        assert got == want and pos == wpos and bad == wbad


@pytest.mark.parametrize("inject", ["", "wal_replay", "wal_replay:nomem"])
def test_wal_replay_gpu_batch_failure_finishes_on_host(knobs, hc, oracle, monkeypatch, inject):
    """A replay above the GPU threshold whose verify batch cannot run (no gfx950
    here, or a simulated HC_E_HIP / HC_E_NOMEM) verifies on the host path and
    returns what the oracle's wal.go:362-455 does -- including a corrupt block
    -- counted in hc_stats; recovery fails only where the reference does."""
    sizes = [oracle.lib().oc_wal_record_size(7, i, 64, 20000) for i in range(400)]
    b, _, _ = oracle.wal_frame(7, sizes)
    img = bytearray(b.tobytes())
    nb = len(img) // 4096
    assert nb >= 256
    knobs.setenv("HC_WAL_GPU_MIN_BLOCKS", "256")
    if inject:
        knobs.setenv("HC_INJECT_FAIL", inject)
    for corrupt in (None, nb // 2):
        view = bytearray(img)
        if corrupt is not None:
            view[corrupt * 4096 + 100] ^= 1
        hc.stats_reset()
        want, wrc, wbad, wpos = oracle.wal_replay(bytes(view), 4096, 0, 4, 0)
        got, err, bad, pos = hc.wal_replay(bytes(view), 4096)
        assert (0 if err is None else err.code) == wrc and got == want and pos == wpos and bad == wbad
        st = hc.stats()
        if inject:
            assert st["wal_gpu_fallback"] == 1 and st["wal_gpu"] == 0
            assert st["last_fallback_error"] == (hc.HC_E_NOMEM if "nomem" in inject else hc.HC_E_HIP)
        elif hc.device_count() == 0:
            assert st["nodev_host"] == 1 and st["wal_gpu"] == 0 and st["wal_gpu_fallback"] == 0
        else:
            assert st["wal_gpu"] == 1 and st["wal_gpu_fallback"] == 0
    knobs.setenv("HC_FORCE_GPU", "1")
    if inject or hc.device_count() == 0:
        with pytest.raises(hc.HundCRCError):
            hc.wal_replay(bytes(img), 4096)
