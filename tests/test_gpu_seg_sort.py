"""The sorted view (round 6): a whole-message
batch listed out of order, from HC_SEG_SORT_MIN records (2^18; 2^14 in these
tests, through the knob, so that the small cases stay cheap), is sorted by
record start inside k_seg_stream (grid barriers), planned again and streamed in
that order; k_seg_combine writes every word through the permutation.  Every
word against the oracle's GetCRC per record (crc_util.go:15-17), and the path
against the plan's restatement (test_gpu_seg.expected_path) of the sorted
arrays: permuted packed / small-gap / wide-gap records, zero-length and
duplicate starts, records spanning many units, overlaps (sorted, then refused:
k_crc_any), the threshold, and the residency check's abort (HC_SEG_SYNC_SPINS)."""
import numpy as np
import pytest
from test_gpu_seg import expected_path, gapped, packed, u32

pytestmark = pytest.mark.gpu

SORT_MIN = 1 << 14      # these tests' threshold (HC_SEG_SORT_MIN, set below)
DEFAULT_SORT_MIN = 1 << 18  # the library's (hc_kernels.hpp kSegSortMin)


@pytest.fixture(autouse=True)
def _sort_from_16k(knobs):
    knobs.setenv("HC_SEG_SORT_MIN", str(SORT_MIN))


def run(torch, hc, buf, off, lens):
    n = len(off)
    out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    doff = torch.from_numpy(off.astype(np.uint64).view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).cuda()
    hc.dev_crc32_blocks(buf, out, nblocks=n, off=doff, lens=dlen, flags=hc.HC_F_MESSAGES)
    torch.cuda.synchronize()
    return u32(out), hc.seg_path()


def sorted_path(ptr, off, lens):
    """seg_path() of a permuted batch the library sorts: the plan of its sorted view."""
    o = np.argsort(off, kind="stable")
    want = expected_path(ptr, off[o], lens[o].astype(np.uint64))
    return "sorted_" + want if want else "fallback"


def check(torch, hc, oracle, host, buf, off, lens, path=None):
    got, was = run(torch, hc, buf, off, lens)
    want = oracle.crc32_messages(host, off.astype(np.uint64), lens.astype(np.uint32), threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], off[bad[:8]], lens[bad[:8]], was)
    if path is not None:
        assert was == path, (was, path)
    return was


def loguniform(rng, n, lo=64.0, span=1024.0):
    return (lo * np.exp(rng.random(n) * np.log(span))).astype(np.uint64)


@pytest.fixture(scope="module")
def buf_host(cuda):
    rng = np.random.default_rng(2024)
    host = rng.integers(0, 256, 640 << 20, dtype=np.uint8)
    yield host, cuda.from_numpy(host).cuda()


@pytest.mark.parametrize("n", [SORT_MIN, 50_000, 300_000])
@pytest.mark.parametrize("start", [0, 5])
def test_permuted_packed_records(cuda, hc, oracle, buf_host, n, start):
    """Config 5's records back to back, listed in a permuted order: sorted, then
    the packed stream."""
    host, buf = buf_host
    rng = np.random.default_rng(n + start)
    lens = loguniform(rng, n, span=64.0 if n > 100_000 else 1024.0)
    off = packed(lens, start)
    assert int(off[-1] + lens[-1]) <= host.size
    p = rng.permutation(n)
    was = check(cuda, hc, oracle, host, buf, off[p], lens[p], sorted_path(buf.data_ptr(), off[p], lens[p]))
    assert was == "sorted_packed"


@pytest.mark.parametrize("gap", [17, 200])
def test_permuted_gapped_records(cuda, hc, oracle, buf_host, gap):
    """WAL-like records behind 17-B headers (the small-gap mode) and 200-B gaps
    (the zeroed-gap mode), permuted."""
    host, buf = buf_host
    n = 40_000
    rng = np.random.default_rng(gap)
    lens = loguniform(rng, n)
    off = gapped(lens, np.full(n, gap, np.uint64), 3)
    p = rng.permutation(n)
    was = check(cuda, hc, oracle, host, buf, off[p], lens[p], sorted_path(buf.data_ptr(), off[p], lens[p]))
    assert was == ("sorted_gapped" if gap <= 64 else "sorted_gapped_wide")


def test_zero_length_and_shared_starts(cuda, hc, oracle, buf_host):
    """Zero-length records (GetCRC of nothing: 0) sharing a start with each
    other and with the next record: the sort orders them by batch index."""
    host, buf = buf_host
    n = 30_000
    rng = np.random.default_rng(9)
    lens = loguniform(rng, n)
    lens[::7] = 0
    off = packed(lens, 1)
    dup = np.flatnonzero(lens == 0)[:500]  # a second zero-length record at each of these starts
    off2 = np.concatenate([off, off[dup]])
    lens2 = np.concatenate([lens, np.zeros(len(dup), np.uint64)])
    p = rng.permutation(len(off2))
    check(cuda, hc, oracle, host, buf, off2[p], lens2[p], sorted_path(buf.data_ptr(), off2[p], lens2[p]))


def test_long_records_across_units(cuda, hc, oracle, buf_host):
    """Records of 64 KiB - 1 MiB (up to 64 units each) permuted: the unit counts
    hold few records and many units hold none."""
    host, buf = buf_host
    n = SORT_MIN + 100
    rng = np.random.default_rng(77)
    lens = loguniform(rng, n, lo=16.0, span=2048.0)
    lens[::97] = rng.integers(1 << 16, 1 << 20, len(lens[::97]))
    off = packed(lens, 1023)
    assert int(off[-1] + lens[-1]) <= host.size
    p = rng.permutation(n)
    check(cuda, hc, oracle, host, buf, off[p], lens[p], sorted_path(buf.data_ptr(), off[p], lens[p]))


def test_overlapping_records_sorted_then_refused(cuda, hc, oracle, buf_host):
    """Permuted records of which two overlap: sorted, the plan of the sorted view
    refuses them, k_crc_any's work in the combine (words still exact)."""
    host, buf = buf_host
    n = 20_000
    rng = np.random.default_rng(5)
    lens = loguniform(rng, n)
    off = packed(lens, 0)
    lens[1000] += 5  # overlaps record 1001
    p = rng.permutation(n)
    check(cuda, hc, oracle, host, buf, off[p], lens[p], "fallback")


def test_below_threshold_and_disabled(cuda, hc, oracle, buf_host, knobs):
    """Under HC_SEG_SORT_MIN records (or with it 0) a permuted batch stays on
    k_crc_any's work in the combine."""
    host, buf = buf_host
    rng = np.random.default_rng(3)
    n = SORT_MIN - 1
    lens = loguniform(rng, n)
    off = packed(lens, 0)
    p = rng.permutation(n)
    check(cuda, hc, oracle, host, buf, off[p], lens[p], "fallback")
    knobs.setenv("HC_SEG_SORT_MIN", str(n))
    check(cuda, hc, oracle, host, buf, off[p], lens[p], "sorted_packed")
    knobs.setenv("HC_SEG_SORT_MIN", "0")
    check(cuda, hc, oracle, host, buf, off[p], lens[p], "fallback")


def test_default_threshold(cuda, hc, oracle, buf_host, knobs):
    """At the library's own threshold (2^18 records: where the sorted view's fixed
    cost meets k_crc_any's, profiles/r6/r6bb/) a permuted batch one record short
    of it stays on k_crc_any; one at it is sorted."""
    host, buf = buf_host
    knobs.delenv("HC_SEG_SORT_MIN", raising=False)
    rng = np.random.default_rng(44)
    n = DEFAULT_SORT_MIN
    lens = loguniform(rng, n, span=64.0)
    off = packed(lens, 1)
    assert int(off[-1] + lens[-1]) <= host.size
    p = rng.permutation(n)
    check(cuda, hc, oracle, host, buf, off[p], lens[p], "sorted_packed")
    q = p[p != n - 1]  # the same records less the last: one short of the threshold
    check(cuda, hc, oracle, host, buf, off[q], lens[q], "fallback")


def test_residency_check_abort_falls_back(cuda, hc, oracle, buf_host, knobs):
    """HC_SEG_SYNC_SPINS=0: the first grid barrier gives up at once unless the
    whole grid is already there; every workgroup then agrees (the CAS on the
    barrier word) and the batch takes k_crc_any's work -- never a partial sort.
    Either outcome leaves every word exact."""
    host, buf = buf_host
    rng = np.random.default_rng(31)
    n = 60_000
    lens = loguniform(rng, n)
    off = packed(lens, 2)
    p = rng.permutation(n)
    knobs.setenv("HC_SEG_SYNC_SPINS", "0")
    seen = set()
    for _ in range(5):
        seen.add(check(cuda, hc, oracle, host, buf, off[p], lens[p]))
    assert seen <= {"fallback", "sorted_packed"}, seen
    knobs.setenv("HC_SEG_SYNC_SPINS", "1")
    seen.add(check(cuda, hc, oracle, host, buf, off[p], lens[p]))
    assert seen <= {"fallback", "sorted_packed"}, seen


def test_repeated_calls_reuse_the_workspace(cuda, hc, oracle, buf_host):
    """A sorted batch, then a smaller unsorted one, then an in-order one on the
    kept workspace (null stream): the barrier words are reset by each plan."""
    host, buf = buf_host
    rng = np.random.default_rng(8)
    for n, perm in [(50_000, True), (SORT_MIN + 7, True), (40_000, False), (50_000, True)]:
        lens = loguniform(rng, n)
        off = packed(lens, int(rng.integers(0, 4096)))
        if perm:
            p = rng.permutation(n)
            off, lens = off[p], lens[p]
        was = check(cuda, hc, oracle, host, buf, off, lens)
        assert was == ("sorted_packed" if perm else "packed"), (n, perm, was)


@pytest.mark.parametrize("uc", ["64", "7"])
def test_several_coarse_buckets_per_workgroup(cuda, hc, oracle, buf_host, knobs, uc):
    """HC_SEG_SORT_UC (test hook) caps the units of a coarse bucket, so a span of
    a few hundred MiB runs several buckets a workgroup (the path a span past
    ~137 GB takes at the default cap): words and path as at the default."""
    host, buf = buf_host
    knobs.setenv("HC_SEG_SORT_UC", uc)
    rng = np.random.default_rng(int(uc))
    n = 40_000
    lens = loguniform(rng, n)
    off = packed(lens, 9)
    p = rng.permutation(n)
    check(cuda, hc, oracle, host, buf, off[p], lens[p], "sorted_packed")


def test_too_many_records_in_one_unit(cuda, hc, oracle, buf_host):
    """More than 1024 records starting in one 16 KiB unit (zero-length ones at one
    start) stop the sort on every workgroup: k_crc_any's work, words exact."""
    host, buf = buf_host
    rng = np.random.default_rng(12)
    n = 30_000
    lens = loguniform(rng, n)
    off = packed(lens, 0)
    off2 = np.concatenate([off, np.full(1500, off[777], np.uint64)])
    lens2 = np.concatenate([lens, np.zeros(1500, np.uint64)])
    p = rng.permutation(len(off2))
    check(cuda, hc, oracle, host, buf, off2[p], lens2[p], "fallback")
