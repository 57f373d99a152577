"""The device entries under HIP graph capture (torch.cuda.CUDAGraph on ROCm =
hipGraph): every launch they make is stream-ordered, with no host sync inside
a call, so a batch can be captured once and replayed on new contents of the
same buffers -- the way a caller removes the per-call launch cost of small,
repeated batches (one WAL segment, one SSTable component).  Each captured
graph is replayed after the inputs change and checked against the oracle:
uniform blocks (k_crc_grp), unaligned messages (k_crc_any), packed records
(the k_seg_* dispatch: its workspace comes from the stream-ordered allocator
inside the graph), verify mode with its bitmap reset (k_verify_prepare), and
the framing pair (k_frame, k_unframe)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def capture(torch, fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm-up outside the graph (first-call setup, device init)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def test_graph_uniform_blocks_and_verify(cuda, hc, oracle):
    torch = cuda
    n, B = 3000, 8192
    rng = np.random.default_rng(1)
    buf = torch.empty(n * B, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    bm = torch.empty((n + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")

    def step():
        hc.dev_crc32_blocks(buf, out, stride=B, ulen=B, nblocks=n)
        hc.dev_verify_prepare(bm, fb, n)
        hc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=n, bad_bitmap=bm, first_bad=fb)

    g = capture(torch, step)
    for it in range(3):
        host = rng.integers(0, 256, n * B, dtype=np.uint8)
        want = oracle.crc32_blocks(host, stride=B, ulen=B)
        host.view(np.uint32).reshape(n, B // 4)[:, 0] = want  # stamped: every block verifies ...
        bad = 17 + 401 * it
        host[bad * B + 9] ^= 0x20  # ... but one
        buf.copy_(torch.from_numpy(host))
        want = oracle.crc32_blocks(host, stride=B, ulen=B)
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(u32(out), want)
        bits = np.unpackbits(u32(bm).view(np.uint8), bitorder="little")[:n]
        assert np.nonzero(bits)[0].tolist() == [bad] and int(fb.item()) == bad


@pytest.mark.parametrize("packed", [False, True])
def test_graph_messages(knobs, cuda, hc, oracle, monkeypatch, packed):
    """Whole messages offered to the packed-record stream (the default at any
    batch size: the k_seg_* dispatch captured, workspace allocated inside the
    graph): packed ones and sorted ones with gaps taken by the stream, the
    gapped ones in an order the stream refuses by k_crc_any on the device flag."""
    torch = cuda
    knobs.delenv("HC_SEG_MIN_MSGS", raising=False)
    rng = np.random.default_rng(2 + packed)
    n = 5000
    lens = rng.integers(64, 9000, n).astype(np.uint64)
    gaps = np.zeros(n, dtype=np.uint64) if packed else rng.integers(1, 40, n).astype(np.uint64)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum((lens + gaps)[:-1], dtype=np.uint64)
    off += np.uint64(3)
    total = int(off[-1] + lens[-1]) + 64
    if not packed:  # out of order (sorted gapped records are the stream's since round 5)
        p = rng.permutation(n)
        off, lens = off[p], lens[p]
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    g = capture(torch, lambda: hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=n, flags=hc.HC_F_MESSAGES))
    assert hc.last_launch()["kernel"] == "k_seg_plan+k_seg_stream+k_seg_combine"
    for _ in range(3):
        host = rng.integers(0, 256, total, dtype=np.uint8)
        buf.copy_(torch.from_numpy(host))
        g.replay()
        torch.cuda.synchronize()
        want = oracle.crc32_messages(host, off, lens.astype(np.uint32), threads=8)
        assert np.array_equal(u32(out), want)
    assert hc.seg_taken() == packed


def test_graph_framing_pair(cuda, hc, oracle):
    torch = cuda
    rng = np.random.default_rng(4)
    n = 4092 * 300 + 1234
    raw = torch.empty(n + 5, dtype=torch.uint8, device="cuda")
    src = raw[5:]  # unaligned payload
    nb = hc.lib().hc_add_crcs_size(n) // 4096
    framed = torch.empty(nb * 4096, dtype=torch.uint8, device="cuda")
    words = torch.empty(nb, dtype=torch.int32, device="cuda")
    pay = torch.empty(nb * 4092 + 16, dtype=torch.uint8, device="cuda")
    rwords = torch.empty(nb, dtype=torch.int32, device="cuda")
    bm = torch.empty((nb + 31) // 32, dtype=torch.int32, device="cuda")
    fb = torch.empty(1, dtype=torch.int64, device="cuda")

    def step():
        hc.dev_add_crcs(src, framed, crc_out=words, n=n)
        hc.dev_verify_prepare(bm, fb, nb)
        hc.dev_read_blocks(framed, 4096, out=pay, crc_out=rwords, bad_bitmap=bm, first_bad=fb)

    g = capture(torch, step)
    for _ in range(3):
        host = rng.integers(0, 256, n, dtype=np.uint8)
        src.copy_(torch.from_numpy(host))
        g.replay()
        torch.cuda.synchronize()
        want = np.zeros(nb * 4096, dtype=np.uint8)
        assert oracle.lib().oc_add_crcs_to_data(host.tobytes(), n, want.ctypes.data) == nb * 4096
        assert framed.cpu().numpy().tobytes() == want.tobytes()
        assert np.array_equal(u32(words), want.view(np.uint32)[::1024])
        assert np.array_equal(u32(rwords), u32(words)) and int(fb.item()) == 2**63 - 1
        assert pay[:n].cpu().numpy().tobytes() == host.tobytes()
