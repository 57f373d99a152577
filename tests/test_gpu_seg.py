"""Packed-record stream (k_seg_*): GetCRC of every record of a
batch whose records lie back to back (config 5's per-record variant,
crc_util.go:15-17 per record), hashed as ONE stream over the span, against the
oracle's restatement of Go's crc32.ChecksumIEEE; and the device-side fallback
to k_crc_any for batches the stream does not take (gaps, overlaps, unsorted,
runs of records under 64 B)."""
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
    return u32(out), hc.seg_taken()


@pytest.fixture
def seg_all(monkeypatch):
    monkeypatch.setenv("HC_SEG_MIN_MSGS", "1")  # offer every message batch to the stream


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
    check(torch, hc, oracle, host, buf, off, lens, True)
    assert "k_seg_stream" in hc.last_launch()["kernel"]


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
            check(torch, hc, oracle, host, buf, off, lens, True)


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
    g[1500:] += 1  # one byte gap
    check(torch, hc, oracle, host, buf, g, lens, False)
    o = off.copy()
    o[700:] -= 1  # one byte overlap
    check(torch, hc, oracle, host, buf, o, lens, False)
    p = rng.permutation(len(off))
    check(torch, hc, oracle, host, buf, off[p], lens[p], False)
    dense = np.array([100, 0, 0, 200, 0, 64, 0] * 1000, dtype=np.uint64)  # empty records, dense
    check(torch, hc, oracle, host, buf, packed(dense, 3), dense, False)
    small = np.full(5000, 63, dtype=np.uint64)  # 65 events in a 4 KiB group
    check(torch, hc, oracle, host, buf, packed(small, 0), small, False)
    small[:] = 64  # exactly 64 per group: still the stream
    check(torch, hc, oracle, host, buf, packed(small, 0), small, True)
    # 63 records and the span's end in the last group (64 events, no 65th): the stream
    edge = np.full(64 * 10 + 63, 64, dtype=np.uint64)
    check(torch, hc, oracle, host, buf, packed(edge, 0), edge, True)
    # 64 records fill the last group exactly; the span's end opens the next one: the stream
    edge = np.full(64 * 10 + 64, 64, dtype=np.uint64)
    check(torch, hc, oracle, host, buf, packed(edge, 0), edge, True)
    # 63 records of 64 B and one of 60 B (64 events), then the span's end in the same group
    # (the 65th event): the fallback
    edge = np.r_[np.full(64 * 10 + 63, 64), [60]].astype(np.uint64)
    check(torch, hc, oracle, host, buf, packed(edge, 0), edge, False)


def test_seg_record_cap(cuda, hc, oracle, seg_all):
    """k_seg_combine chains the raw CRCs of the whole units a record spans, so
    the stream takes records up to 16 MiB (1024 units) and a batch with a
    longer one falls back to k_crc_any on the device."""
    torch = cuda
    rng = np.random.default_rng(17)
    total = 40 << 20
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    for big, taken in [((1 << 24), True), ((1 << 24) + 1, False), ((1 << 24) - 3, True)]:
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
    check(torch, hc, oracle, host, buf, off, lens, True)  # the same batch with crc_out: the stream


def test_seg_threshold(cuda, hc, oracle, monkeypatch):
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
    monkeypatch.delenv("HC_SEG_MIN_MSGS", raising=False)
    check(torch, hc, oracle, host, buf, off, lens, True)
    assert "k_seg_stream" in hc.last_launch()["kernel"]
    for n in (1, 2, 17):  # tiny batches at the default
        check(torch, hc, oracle, host, buf, off[:n], lens[:n], True)
    monkeypatch.setenv("HC_SEG_MIN_MSGS", "5001")
    check(torch, hc, oracle, host, buf, off, lens, False)
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
    assert was
    # oracle on 20k records of the first 512 MB (all of the first 200)
    head = int(np.searchsorted(off, 512 << 20))
    pick = np.unique(np.r_[np.arange(200), rng.choice(head, 20_000, replace=False)])
    hi = int((off[pick] + lens[pick]).max())
    sample = buf[:hi].cpu().numpy()
    want = oracle.crc32_messages(sample, off[pick], lens[pick].astype(np.uint32), threads=16)
    assert (got[pick] == want).all()
    # every word against k_crc_any: the same records with the last one moved one
    # byte up (a gap: not packed, so the device flag sends it to k_crc_any)
    g = off.copy()
    g[-1] += 1
    l3 = lens.copy()
    l3[-1] -= 1
    got3, was3 = run(torch, hc, buf, g, l3)
    assert not was3
    assert (got3[:-1] == got[:-1]).all()


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
T.check(torch, hc, O, host, buf, off, lens, True)
g = off.copy(); g[n - 700:] += np.uint64(1)  # a gap near the end: the last strides
T.check(torch, hc, O, host, buf, g, lens, False)
print("ok")
"""
    env = dict(os.environ, HC_SEG_PLAN_WGS=str(plan_wgs), HC_SEG_MIN_MSGS="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
