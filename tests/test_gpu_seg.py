"""Packed-record stream (k_seg_*): GetCRC of every record of a
batch whose records lie back to back (config 5's per-record variant,
crc_util.go:15-17 per record), hashed as ONE stream over the span, against the
oracle's restatement of Go's crc32.ChecksumIEEE; and the device-side fallback
to k_crc_any for batches the stream does not take (overlaps, unsorted, runs of
records under 64 B, gaps over a quarter of the payload).  Sorted records with
gaps between them (round 5) are taken by the same stream over 2n events.
`check(..., taken)`: "packed", "gapped" or None (k_crc_any)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def packed(lens, start):
    off = np.zeros(len(lens), dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return off + np.uint64(start)


def run(torch, hc, buf, off, lens):
    n = len(off)
    out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).cuda()
    hc.dev_crc32_blocks(buf, out, nblocks=n, off=doff, lens=dlen, flags=hc.HC_F_MESSAGES)
    torch.cuda.synchronize()
    return u32(out), hc.seg_mode()


@pytest.fixture
def seg_all(knobs, monkeypatch):
    knobs.setenv("HC_SEG_MIN_MSGS", "1")  # offer every message batch to the stream


def check(torch, hc, oracle, host, buf, off, lens, taken):
    got, was = run(torch, hc, buf, off, lens)
    want = oracle.crc32_messages(host, off, lens.astype(np.uint32), threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], lens[bad[:8]], off[bad[:8]])
    assert was == taken
    return got


@pytest.mark.parametrize("start", [0, 1, 1023, 1024, 4093, 16384 - 5])
def test_seg_log_uniform_records(cuda, hc, oracle, seg_all, start):
    """Config 5b's law (log-uniform 64 B - 64 KiB), packed at several start
    alignments (row, group and unit boundaries): taken by the stream, bit-exact."""
    torch = cuda
    rng = np.random.default_rng(start + 5)
    n = 20_000
    lens = (64.0 * np.exp(rng.random(n) * np.log(1024.0))).astype(np.uint64)
    off = packed(lens, start)
    total = int(off[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    assert int(off[-1] + lens[-1]) <= total
    check(torch, hc, oracle, host, buf, off, lens, "packed")
    assert "k_seg_stream" in hc.last_launch()["kernel"]


@pytest.mark.parametrize("lg", ["0", "1", "5", "7", "12"])
def test_seg_chunk_slots(cuda, hc, oracle, seg_all, knobs, lg):
    """HC_SEG_LG_CHUNK: the stream deals its 16 KiB units to the workgroups in
    round-robin slots of 2^lg units (default 3, round 6; 0: one unit a slot; 12
    is cut down until every workgroup has 4 slots).  Packed, 17-B gapped and
    permuted (sorted view) batches stay bit-exact at other slot sizes."""
    torch = cuda
    knobs.setenv("HC_SEG_LG_CHUNK", lg)
    knobs.setenv("HC_SEG_SORT_MIN", "16384")  # the permuted case below is sorted
    rng = np.random.default_rng(int(lg) + 91)
    n = 60_000
    lens = (64.0 * np.exp(rng.random(n) * np.log(1024.0))).astype(np.uint64)
    off = packed(lens, 3)
    goff = gapped(lens, np.full(n, 17, dtype=np.uint64), 7)
    total = int(goff[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    check(torch, hc, oracle, host, buf, off, lens, "packed")
    check(torch, hc, oracle, host, buf, goff, lens, "gapped")
    p = rng.permutation(n)
    check(torch, hc, oracle, host, buf, off[p], lens[p], "sorted_packed")


def test_seg_boundaries_and_shapes(cuda, hc, oracle, seg_all):
    """Records ending exactly on row / group / unit boundaries, empty records,
    records of 64 B .. 1 MiB (spanning many units), one record, two records."""
    torch = cuda
    rng = np.random.default_rng(7)
    total = 48 << 20
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    cases = [
        np.array([1024] * 3000, dtype=np.uint64),                  # row-aligned ends
        np.array([4096, 16384, 64, 1023, 1025, 16383, 16385] * 500, dtype=np.uint64),
        np.array([3000, 0, 0, 2000, 0, 64, 0] * 1000, dtype=np.uint64),  # empty records
        np.array([1 << 20] * 20 + [77] * 100, dtype=np.uint64),    # 1 MiB records
        np.array([5000], dtype=np.uint64),
        np.array([64, 65], dtype=np.uint64),
        np.array([12345678], dtype=np.uint64),                      # one record over many units
    ]
    for i, lens in enumerate(cases):
        for start in (0, 3, 1024 - 1):
            off = packed(lens, start)
            assert int(off[-1] + lens[-1]) <= total
            check(torch, hc, oracle, host, buf, off, lens, "packed")


def test_seg_falls_back_on_the_device(cuda, hc, oracle, seg_all):
    """Batches the stream does not take are hashed by k_crc_any (the device
    flag): a gap, an overlap, unsorted records, and 65 events in one 4 KiB
    group (records under 64 B)."""
    torch = cuda
    rng = np.random.default_rng(11)
    total = 8 << 20
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    lens = rng.integers(64, 4000, 3000).astype(np.uint64)
    off = packed(lens, 5)
    g = off.copy()
    g[1500:] += 1  # one byte gap: sorted, the gapped stream
    check(torch, hc, oracle, host, buf, g, lens, "gapped")
    o = off.copy()
    o[700:] -= 1  # one byte overlap
    check(torch, hc, oracle, host, buf, o, lens, None)
    p = rng.permutation(len(off))
    check(torch, hc, oracle, host, buf, off[p], lens[p], None)
    dense = np.array([100, 0, 0, 200, 0, 64, 0] * 1000, dtype=np.uint64)  # empty records, dense
    check(torch, hc, oracle, host, buf, packed(dense, 3), dense, None)
    small = np.full(5000, 63, dtype=np.uint64)  # 65 events in a 4 KiB group
    check(torch, hc, oracle, host, buf, packed(small, 0), small, None)
    small[:] = 64  # exactly 64 per group: still the stream
    check(torch, hc, oracle, host, buf, packed(small, 0), small, "packed")
    # 63 records and the span's end in the last group (64 events, no 65th): the stream
    edge = np.full(64 * 10 + 63, 64, dtype=np.uint64)
    check(torch, hc, oracle, host, buf, packed(edge, 0), edge, "packed")
    # 64 records fill the last group exactly; the span's end opens the next one: the stream
    edge = np.full(64 * 10 + 64, 64, dtype=np.uint64)
    check(torch, hc, oracle, host, buf, packed(edge, 0), edge, "packed")
    # 63 records of 64 B and one of 60 B (64 events), then the span's end in the same group
    # (the 65th event): the fallback
    edge = np.r_[np.full(64 * 10 + 63, 64), [60]].astype(np.uint64)
    check(torch, hc, oracle, host, buf, packed(edge, 0), edge, None)


def test_seg_record_cap(cuda, hc, oracle, seg_all):
    """k_seg_combine chains the raw CRCs of the whole units a record spans, so
    the stream takes records up to 16 MiB (1024 units) and a batch with a
    longer one falls back to k_crc_any on the device."""
    torch = cuda
    rng = np.random.default_rng(17)
    total = 40 << 20
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    for big, taken in [((1 << 24), "packed"), ((1 << 24) + 1, None), ((1 << 24) - 3, "packed")]:
        lens = np.array([1000] * 300 + [big] + [777, 64, 5000] * 100, dtype=np.uint64)
        off = packed(lens, 9)
        assert int(off[-1] + lens[-1]) <= total
        check(torch, hc, oracle, host, buf, off, lens, taken)


def test_seg_without_crc_out(cuda, hc, oracle, seg_all):
    """crc_out is optional (hundcrc.h): a packed whole-message batch with no
    crc_out is not offered to the stream, whose only output is crc_out
    (k_seg_combine), and runs without touching a null pointer."""
    torch = cuda
    rng = np.random.default_rng(13)
    lens = rng.integers(64, 3000, 4000).astype(np.uint64)
    off = packed(lens, 7)
    host = rng.integers(0, 256, int(off[-1] + lens[-1]) + 16, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).cuda()
    hc.dev_crc32_blocks(buf, None, nblocks=len(off), off=doff, lens=dlen, flags=hc.HC_F_MESSAGES)
    torch.cuda.synchronize()
    assert not hc.seg_taken()
    assert hc.last_launch()["kernel"] == "k_crc_grp+k_crc_any"
    check(torch, hc, oracle, host, buf, off, lens, "packed")  # the same batch with crc_out: the stream


def test_seg_threshold(knobs, cuda, hc, oracle, monkeypatch):
    """By default every whole-message batch with crc_out is offered to the
    stream (it beats k_crc_grp + k_crc_any from 16 records up, profiles/r4/r4s,
    r4t); below HC_SEG_MIN_MSGS the batch is not offered."""
    torch = cuda
    rng = np.random.default_rng(3)
    lens = rng.integers(64, 3000, 5000).astype(np.uint64)
    off = packed(lens, 0)
    total = int(off[-1] + lens[-1])
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    knobs.delenv("HC_SEG_MIN_MSGS", raising=False)
    check(torch, hc, oracle, host, buf, off, lens, "packed")
    assert "k_seg_stream" in hc.last_launch()["kernel"]
    for n in (1, 2, 17):  # tiny batches at the default
        check(torch, hc, oracle, host, buf, off[:n], lens[:n], "packed")
    knobs.setenv("HC_SEG_MIN_MSGS", "5001")
    check(torch, hc, oracle, host, buf, off, lens, None)
    assert hc.last_launch()["kernel"] == "k_crc_grp+k_crc_any"


def test_seg_config5b_size(cuda, hc, oracle):
    """Config 5's per-record variant at 2M records (18.9 GB) with the default
    threshold: taken by the stream; the oracle checks a sample of 20k records
    (every record of the first MiB, then random ones) and the words are
    identical to k_crc_any's (the stream's fallback, forced by a gap)."""
    torch = cuda
    n = 2_000_000
    rng = np.random.default_rng(55)
    lens = (64.0 * np.exp(rng.random(n) * np.log(1024.0))).astype(np.uint64)
    off = packed(lens, 1)
    total = (int(off[-1] + lens[-1]) + 64 + (1 << 20) - 1) >> 20 << 20
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    hc.dev_fill_range(buf, 0x5B, 0, total >> 20, stride=1 << 20, ulen=1 << 20)  # every byte, in 1 MiB blocks
    got, was = run(torch, hc, buf, off, lens)
    assert was == "packed"
    # oracle on 20k records of the first 512 MB (all of the first 200)
    head = int(np.searchsorted(off, 512 << 20))
    pick = np.unique(np.r_[np.arange(200), rng.choice(head, 20_000, replace=False)])
    hi = int((off[pick] + lens[pick]).max())
    sample = buf[:hi].cpu().numpy()
    want = oracle.crc32_messages(sample, off[pick], lens[pick].astype(np.uint32), threads=16)
    assert (got[pick] == want).all()
    # every word against k_crc_any: the same records with the next-to-last one
    # a byte longer (an overlap: the device flag sends the batch to k_crc_any)
    l3 = lens.copy()
    l3[-2] += 1
    got3, was3 = run(torch, hc, buf, off, l3)
    assert was3 is None
    assert (got3[:-2] == got[:-2]).all()


def test_seg_workspace_streams(cuda, hc, oracle, seg_all):
    """On the null stream the workspace is kept across calls and grown there
    (hc_api.cpp seg_cached_ws); calls on other streams allocate per call.
    Batches of growing and shrinking size alternate between the null stream and
    a side stream, each launched without waiting for the other's, and every
    word is checked."""
    torch = cuda
    rng = np.random.default_rng(23)
    streams = [torch.cuda.default_stream(), torch.cuda.Stream()]
    assert streams[0].cuda_stream == 0
    jobs = []
    for i, n in enumerate([3000, 9000, 2000, 30000, 40000, 5000, 60000, 1000]):
        lens = rng.integers(64, 6000, n).astype(np.uint64)
        off = packed(lens, 1 + i)
        host = rng.integers(0, 256, int(off[-1] + lens[-1]) + 16, dtype=np.uint8)
        s = streams[i % 2]
        with torch.cuda.stream(s):
            buf = torch.from_numpy(host).cuda()
            doff = torch.from_numpy(off.view(np.int64)).cuda()
            dlen = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).cuda()
            out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
            hc.dev_crc32_blocks(buf, out, nblocks=n, off=doff, lens=dlen, flags=hc.HC_F_MESSAGES, stream=s)
        assert "k_seg_stream" in hc.last_launch()["kernel"]
        jobs.append((host, off, lens, out, buf, doff, dlen))
    torch.cuda.synchronize()
    for host, off, lens, out, *_ in jobs:
        want = oracle.crc32_messages(host, off, lens.astype(np.uint32), threads=16)
        assert (u32(out) == want).all()


@pytest.mark.parametrize("plan_wgs", [1, 3])
def test_seg_plan_grid_stride(cuda, hc, oracle, plan_wgs):
    """k_seg_plan grid-strides over the events once they outnumber its grid cap
    (default 2048 workgroups, 524288 events a stride; config 5b strides 4 times).
    A child process caps it at 1 or 3 workgroups (HC_SEG_PLAN_WGS, read once per
    process) so 60k events take 79 or 27 strides: a packed batch is taken and
    bit-exact, and a gap found in a late stride of one workgroup still sends the
    batch to k_crc_any."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys; sys.path.insert(0, {root!r}); sys.path.insert(0, {root + '/tests'!r})
import numpy as np, torch
from hunddb_amd import crc as hc
from oracle import oracle as O
import test_gpu_seg as T
rng = np.random.default_rng(31)
n = 60_000
lens = rng.integers(64, 3000, n).astype(np.uint64)
off = T.packed(lens, 3)
host = rng.integers(0, 256, int(off[-1] + lens[-1]) + 64, dtype=np.uint8)
buf = torch.from_numpy(host).cuda()
T.check(torch, hc, O, host, buf, off, lens, "packed")
o = lens.copy(); o[n - 700] += 1  # an overlap near the end: the last strides
T.check(torch, hc, O, host, buf, off, o, None)
g = off.copy(); g[n - 700:] += np.uint64(1)  # a gap near the end: still sorted
T.check(torch, hc, O, host, buf, g, lens, "gapped")
print("ok")
"""
    env = dict(os.environ, HC_SEG_PLAN_WGS=str(plan_wgs), HC_SEG_MIN_MSGS="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def expected_mode(base, off, lens):
    """The plan's decision (k_seg_plan + k_seg_stream's prologue) restated:
    "packed" when every record starts where the previous one ends and no 4 KiB
    group (from the span's 1 KiB-aligned origin) holds 65 of the n + 1 events;
    else "gapped" when the records are sorted and do not overlap, no gap is over
    4 MiB, no group holds 65 of the 2n events s_j, e_j, and the gap bytes are at
    most a quarter of the payload; else None (k_crc_any)."""
    s = np.uint64(base) + off.astype(np.uint64)
    e = s + lens.astype(np.uint64)
    pend = int(e[-1])
    a0 = int(s[0]) & ~1023
    if (lens > (1 << 24)).any() or int(s.min()) < a0 or int(e.max()) > pend:
        return None

    def dense(ev):
        g = (ev - np.uint64(a0)) >> np.uint64(12)
        return len(ev) > 64 and bool((g[64:] == g[:-64]).any())
    if (s[1:] == e[:-1]).all() and not dense(np.r_[s, np.uint64(pend)]):
        return "packed"
    if (s[1:] >= e[:-1]).all() and (s[1:] - e[:-1] <= (1 << 22)).all():  # gaps up to kSegMaxGap (4 MiB)
        ev = np.empty(2 * len(s), dtype=np.uint64)
        ev[0::2], ev[1::2] = s, e
        gaps = int((s[1:] - e[:-1]).sum()) if len(s) > 1 else 0
        if not dense(ev) and 4 * gaps <= int(lens.astype(np.uint64).sum()):
            return "gapped"
    return None


def expected_path(base, off, lens):
    """seg_path() of a batch: "gapped" (every gap <= 64 B, the combine hashes
    them, its n + 1 record-end events at most 64 per 4 KiB group) before
    "gapped_wide" (the zeroed-gap stream over 2n events)."""
    m = expected_mode(base, off, lens)
    if m == "packed":
        return m
    s = np.uint64(base) + off.astype(np.uint64)
    e = s + lens.astype(np.uint64)
    if (s[1:] >= e[:-1]).all() and (s[1:] - e[:-1] <= 64).all() and len(s):
        ev = np.r_[s[:1], e]
        g = (ev - np.uint64(int(s[0]) & ~1023)) >> np.uint64(12)
        dense = len(ev) > 64 and bool((g[64:] == g[:-64]).any())
        gaps = int((s[1:] - e[:-1]).sum()) if len(s) > 1 else 0
        if not dense and 4 * gaps <= int(lens.astype(np.uint64).sum()):
            return "gapped"
    return "gapped_wide" if m == "gapped" else m


def gapped(lens, gaps, start):
    """Records in order with gaps[j] bytes before record j (j > 0)."""
    off = np.zeros(len(lens), dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[1:].astype(np.uint64), dtype=np.uint64)
    return off + np.uint64(start)


@pytest.mark.parametrize("start", [0, 5, 1023, 4093, 16384 - 17])
def test_seg_gapped_wal_records(cuda, hc, oracle, seg_all, start):
    """Config 5's record law with a 17-B gap before every record (the WAL header
    of /root/reference/lsm/wal/wal_header.go:5-23 sits between payloads): taken
    by the stream over the 2n record boundaries, bit-exact against the oracle's
    ChecksumIEEE of each record (crc_util.go:15-17)."""
    torch = cuda
    rng = np.random.default_rng(start + 77)
    n = 20_000
    lens = (64.0 * np.exp(rng.random(n) * np.log(1024.0))).astype(np.uint64)
    off = gapped(lens, np.full(n, 17, dtype=np.uint64), start)
    total = int(off[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    assert expected_path(buf.data_ptr(), off, lens) == "gapped"
    check(torch, hc, oracle, host, buf, off, lens, "gapped")
    assert hc.seg_path() == "gapped"  # 17-B gaps: the combine hashes them
    assert "k_seg_stream" in hc.last_launch()["kernel"]


def test_seg_gapped_shapes(cuda, hc, oracle, seg_all):
    """Gapped batches of every shape, each against the oracle and against the
    restated decision: random gaps with zeros among them (records that touch),
    empty records, records ending on row / group / unit boundaries, one 12 MB
    record, one and two records, gaps of whole units, gaps just under and just
    over a quarter of the payload, dense small records at the 64-event limit,
    an overlap and an unsorted batch (both k_crc_any)."""
    torch = cuda
    rng = np.random.default_rng(99)
    total = 64 << 20
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    cases = []
    lens = rng.integers(64, 5000, 4000).astype(np.uint64)
    gaps = rng.integers(0, 40, 4000).astype(np.uint64)
    gaps[rng.random(4000) < 0.3] = 0
    cases.append((lens, gaps))
    cases.append((np.array([3000, 0, 0, 2000, 0, 64, 0] * 700, dtype=np.uint64),
                  np.array([5, 0, 7, 1, 0, 0, 9] * 700, dtype=np.uint64)))
    cases.append((np.array([1024 - 17, 4096 - 17, 16384 - 17] * 600, dtype=np.uint64), np.full(1800, 17, np.uint64)))
    cases.append((np.array([12_345_678], dtype=np.uint64), np.zeros(1, np.uint64)))
    cases.append((np.array([64, 65], dtype=np.uint64), np.array([0, 3], dtype=np.uint64)))
    cases.append((np.array([1 << 20] * 10, dtype=np.uint64), np.array([0] + [16384] * 9, dtype=np.uint64)))
    L = rng.integers(1000, 3000, 3000).astype(np.uint64)
    q = int(L.sum()) // 4
    g = np.zeros(3000, dtype=np.uint64)
    g[1:] = q // 2999
    cases.append((L, g))                            # just under a quarter: gapped
    g2 = g.copy()
    g2[1:1 + (q - int(g.sum())) + 1] += 1           # one byte over a quarter: k_crc_any
    cases.append((L, g2))
    big = np.full(20, 1 << 20, dtype=np.uint64)      # one 4 MiB gap (kSegMaxGap): gapped; one byte more: k_crc_any
    bg = np.zeros(20, dtype=np.uint64)
    bg[7] = 1 << 22
    cases.append((big, bg))
    bg2 = bg.copy()
    bg2[7] += 1
    cases.append((big, bg2))
    small = np.full(5000, 120, dtype=np.uint64)      # 32 records + 8-B gaps per 4 KiB: 64 events a group
    cases.append((small, np.full(5000, 8, np.uint64)))
    small2 = np.full(5000, 100, dtype=np.uint64)     # 34 records per group: 68 of the 2n events, but
    cases.append((small2, np.full(5000, 20, np.uint64)))  # 34 record ends: the small-gap mode
    small3 = np.full(5000, 50, dtype=np.uint64)      # 68 record ends per group: k_crc_any
    cases.append((small3, np.full(5000, 10, np.uint64)))
    paths = set()
    for lens, gaps in cases:
        for start in (0, 3, 1024 - 1):
            off = gapped(lens, gaps, start)
            assert int(off[-1] + lens[-1]) <= total
            want = expected_path(buf.data_ptr(), off, lens)
            check(torch, hc, oracle, host, buf, off, lens, "gapped" if want == "gapped_wide" else want)
            assert hc.seg_path() == (want or "fallback"), (want, hc.seg_path())
            paths.add(want)
    assert paths == {"packed", "gapped", "gapped_wide", None}, paths
    lens, gaps = cases[0]
    off = gapped(lens, gaps, 1)
    o = lens.copy()
    o[100] = off[101] - off[100] + 1  # record 100 overlaps 101 by one byte
    check(torch, hc, oracle, host, buf, off, o, None)
    p = rng.permutation(len(off))
    check(torch, hc, oracle, host, buf, off[p], lens[p], None)


def test_seg_fallback_runs_crc_grp_on_aligned_records(knobs, cuda, hc, oracle, seg_all):
    """a whole-message batch whose records are all 16-B
    aligned 4 KiB multiples goes to k_crc_grp in any order or layout (since
    r5s ahead of the stream's own modes), launched after the combine and gated
    on the stream's mode word ("fallback_grp"); one record that is not:
    k_crc_any inside the combine, or the stream when it takes the batch.  Batches from HC_SEG_GRP_MIN records (2^18; 1000 here) may take
    it, smaller ones never do.  Every word against the oracle."""
    knobs.setenv("HC_SEG_GRP_MIN", "1000")
    torch = cuda
    rng = np.random.default_rng(41)
    n = 6000
    lens = (4096 << rng.integers(0, 3, n)).astype(np.uint64)   # 4 / 8 / 16 KiB
    off = packed(lens, 0)
    total = int(off[-1] + lens[-1]) + 4096
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    assert buf.data_ptr() % 16 == 0
    p = rng.permutation(n)
    check(torch, hc, oracle, host, buf, off[p], lens[p], None)          # out of order: all k_crc_grp's
    assert hc.seg_path() == "fallback_grp"
    check(torch, hc, oracle, host, buf, off, lens, None)                # in order: still k_crc_grp's (r5s)
    assert hc.seg_path() == "fallback_grp"
    gp = packed(lens + np.uint64(16), 0)                                # 16-B gaps: ditto
    check(torch, hc, oracle, host, buf, gp[: n // 2], lens[: n // 2], None)
    assert hc.seg_path() == "fallback_grp"
    far = (np.arange(n, dtype=np.uint64) * np.uint64(16384 * 2))[: n // 4]  # gaps over a quarter
    fl = np.full(n // 4, 16384, dtype=np.uint64)
    big = torch.zeros(int(far[-1]) + 16384 + 64, dtype=torch.uint8, device="cuda")
    bh = rng.integers(0, 256, big.numel(), dtype=np.uint8)
    big.copy_(torch.from_numpy(bh))
    check(torch, hc, oracle, bh, big, far, fl, None)
    assert hc.seg_path() == "fallback_grp"
    mixed = lens[p].copy()
    mixed[n // 2] -= np.uint64(100)  # one record not a 4 KiB multiple: k_crc_any
    check(torch, hc, oracle, host, buf, off[p], mixed, None)
    assert hc.seg_path() == "fallback"
    mis = off[p] + np.uint64(4)  # misaligned 4 KiB multiples (sizes stay in the buffer: -4 from each)
    check(torch, hc, oracle, host, buf, mis, lens[p] - np.uint64(4096), None)
    assert hc.seg_path() == "fallback"
    knobs.setenv("HC_SEG_GRP_MIN", str(n + 1))  # under the threshold: k_crc_any in the combine
    check(torch, hc, oracle, host, buf, off[p], lens[p], None)
    assert hc.seg_path() == "fallback"
