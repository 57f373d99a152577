"""Uniform block batches that k_crc_grp refuses, on the message stream (round 5).

A block is CRC'd over block[4:len] (crc_util.go:88-100, `CheckBlockIntegrity`;
:21-33 `AddCRCToBlockData`).  Blocks of a length that is not a 4 KiB multiple
(utils/config/config.go:241 accepts any BlockSize >= 1024) or at an address
that is not 16-B aligned used to take k_crc_any (57-62 %).  From
HC_SEG_MIN_BLOCKS blocks a uniform batch with stride >= len now goes to
launch_seg_blocks: the messages block[4:len] lie 4 + stride - len bytes apart,
which the stream's small-gap mode takes (wider gaps: the zeroed-gap mode), and
k_seg_block_out writes the verify bitmap / first_bad and the stamps.  Every
word, bit and stamped byte is compared with the oracle."""
import numpy as np
import pytest
from test_gpu_seg import expected_path

pytestmark = pytest.mark.gpu


@pytest.fixture
def seg_blocks(knobs):
    knobs.setenv("HC_SEG_MIN_BLOCKS", "1")  # every size below is offered to the stream


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def run(torch, hc, buf, n, stride, ulen, flags=0, verify=False):
    out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    bm = fb = None
    if verify:
        bm = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
        fb = torch.zeros(1, dtype=torch.int64, device="cuda")
        hc.dev_verify_prepare(bm, fb, n)
    hc.dev_crc32_blocks(buf, out, stride=stride, ulen=ulen, nblocks=n, bad_bitmap=bm, first_bad=fb, flags=flags)
    torch.cuda.synchronize()
    return u32(out), bm, fb


CASES = [  # (ulen, stride - ulen, start, path; None: as the plan's restatement says)
    (4092, 0, 0, "gapped"),       # config.go:241's non-4 KiB BlockSize, back to back: 4-B gaps (the stored
    (4092, 0, 3, "gapped"),       # words); aligned too since round 6 (k_crc_any kept them before)
    (4096, 0, 1, "gapped"),       # 4 KiB blocks at an odd address (k_crc_grp needs 16-B alignment)
    (1000, 0, 0, "gapped"),
    (5000, 24, 2, "gapped"),      # 28-B gaps
    (8188, 60, 0, "gapped"),      # 64-B gaps: the small-gap mode's widest
    (8188, 61, 0, "gapped_wide"), # 65-B gaps: the zeroed-gap mode
    (3000, 1000, 5, "fallback"),  # gaps over a quarter of the payload: k_crc_any
    (64, 0, 0, None),             # 60-B messages, 64 record ends a 4 KiB group: at the stream's limit
    (32, 0, 0, "fallback"),       # 128 a group: k_crc_any
    (4, 0, 0, "fallback"),        # empty messages
    (7, 9, 1, "fallback"),
]


@pytest.mark.parametrize("ulen,extra,start,path", CASES)
def test_uniform_blocks_on_the_stream(seg_blocks, cuda, hc, oracle, ulen, extra, start, path):
    torch = cuda
    stride = ulen + extra
    n = max(3000, (24 << 20) // stride) if ulen > 64 else 5000
    rng = np.random.default_rng(ulen * 7 + extra + start)
    host = rng.integers(0, 256, start + n * stride + 64, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    view = buf[start:]
    want = oracle.crc32_blocks(host[start:], stride=stride, ulen=ulen, nblocks=n)
    got, _, _ = run(torch, hc, view, n, stride, ulen)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])
    moff = np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(4)
    want_path = expected_path(view.data_ptr(), moff, np.full(n, ulen - 4, np.uint64)) or "fallback"
    assert path is None or path == want_path
    assert hc.seg_path() == want_path


@pytest.mark.parametrize("ulen,extra,start", [(8188, 0, 0), (4092, 0, 1), (6000, 100, 2), (1020, 0, 0)])
def test_uniform_blocks_verify_and_stamp(seg_blocks, cuda, hc, oracle, ulen, extra, start):
    torch = cuda
    stride = ulen + extra
    n = 6000
    rng = np.random.default_rng(ulen + start)
    host = rng.integers(0, 256, start + n * stride + 64, dtype=np.uint8)
    want = oracle.crc32_blocks(host[start:], stride=stride, ulen=ulen, nblocks=n)
    # stamp on the device: every block's word becomes its CRC, nothing else changes
    buf = torch.from_numpy(host.copy()).cuda()
    got, _, _ = run(torch, hc, buf[start:], n, stride, ulen, flags=hc.HC_F_STAMP)
    assert (got == want).all()
    assert hc.seg_path() in ("gapped", "gapped_wide")
    stamped = host.copy()
    blk = stamped[start:start + n * stride].reshape(n, stride)
    blk[:, :4] = want.view(np.uint8).reshape(n, 4)
    dev = buf.cpu().numpy()
    assert np.array_equal(dev, stamped), np.nonzero(dev != stamped)[0][:8]
    # verify the stamped image: clean
    _, bm, fb = run(torch, hc, buf[start:], n, stride, ulen, verify=True)
    assert int(fb.item()) == np.iinfo(np.int64).max and not bm.cpu().numpy().any()
    # corrupt some blocks (a payload byte or the stored word) and verify again
    bad_blocks = np.array(sorted({7, 63, 64, 65, 1000, 4095, n - 1}))
    host2 = stamped.copy()
    for i, k in enumerate(bad_blocks):
        pos = start + k * stride + (1 if i % 2 else 4 + (k * 37) % (ulen - 4))
        host2[pos] ^= 0x40
    buf2 = torch.from_numpy(host2).cuda()
    _, bm, fb = run(torch, hc, buf2[start:], n, stride, ulen, verify=True)
    assert int(fb.item()) == int(bad_blocks[0])
    bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(np.nonzero(bits)[0], bad_blocks)


def test_threshold_keeps_small_batches_on_k_crc_any(cuda, hc, oracle, knobs):
    """Below HC_SEG_MIN_BLOCKS (default 4096) the batch stays on k_crc_any."""
    torch = cuda
    n, ulen = 1000, 8188
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, n * ulen, dtype=np.uint8)
    got, _, _ = run(torch, hc, torch.from_numpy(host).cuda(), n, ulen, ulen)
    assert (got == oracle.crc32_blocks(host, stride=ulen, ulen=ulen, nblocks=n)).all()
    assert hc.seg_path() == "fallback"
    knobs.setenv("HC_SEG_MIN_BLOCKS", "500")
    got, _, _ = run(torch, hc, torch.from_numpy(host).cuda(), n, ulen, ulen)
    assert (got == oracle.crc32_blocks(host, stride=ulen, ulen=ulen, nblocks=n)).all()
    assert hc.seg_path() == "gapped"


MSG_CASES = [  # (ulen, stride - ulen, start): uniform HC_F_MESSAGES batches k_crc_grp refuses
    (100, 0, 0),     # 100-B messages back to back: packed
    (1000, 3, 1),    # odd address, 3-B gaps
    (4096, 0, 1),    # 4 KiB messages at an odd address
    (8190, 2, 2),    # 8 KiB-ish, 2-B gaps
    (4000, 96, 0),   # 4-B aligned 4004-B equivalent blocks (k_crc_any's until round 6)
    (5, 11, 3),      # tiny messages
]


@pytest.mark.parametrize("ulen,extra,start", MSG_CASES)
def test_uniform_messages_route(cuda, hc, oracle, ulen, extra, start):
    """a uniform whole-message batch (HC_F_MESSAGES with stride/ulen,
    no off/len) of >= HC_SEG_MIN_BLOCKS entries that k_crc_grp cannot take went to
    launch_seg_blocks, which refused message mode: HC_E_HIP and no words.  Now the
    route builds whole-message off/len (j * stride, ulen); every word against the
    oracle's GetCRC (crc_util.go:15-17), at the default threshold."""
    torch = cuda
    stride = ulen + extra
    n = max(5000, (16 << 20) // stride)
    rng = np.random.default_rng(ulen * 3 + extra + start)
    host = rng.integers(0, 256, start + n * stride + 64, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    view = buf[start:]
    got, _, _ = run(torch, hc, view, n, stride, ulen, flags=hc.HC_F_MESSAGES)
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(start)
    want = oracle.crc32_messages(host, off, np.full(n, ulen, np.uint32))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])
    ptr = view.data_ptr()
    if ulen < 4:
        assert hc.last_launch()["kernel"] == "k_crc_any"
    else:
        assert hc.last_launch()["kernel"].startswith("k_seg_plan")
        moff = np.arange(n, dtype=np.uint64) * np.uint64(stride)
        assert hc.seg_path() == (expected_path(ptr, moff, np.full(n, ulen, np.uint64)) or "fallback")
