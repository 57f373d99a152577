"""Several host threads enqueueing device batches at once.
k_crc_grp's "left a block to the sweep" word (Batch::skip_slot) is shared by
every call on a device and raised to per-call tags that increase across
calls, so a call can only run a sweep it did not need, never skip one it
needs.  The packed-record stream's mode word is word 0 of its workspace: kept
on the null stream (one stream orders every use) and allocated per call on
other streams, so concurrent calls never share it.  4 threads, each on its own
stream, alternate conforming off/len batches with ones holding non-conforming
blocks (misaligned, short), and packed record batches with ones that the
stream refuses; every word of every call is checked against the oracle
(crc_util.go:15-17 / ChecksumIEEE per block)."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_concurrent_threads_share_the_device_slots(knobs, cuda, hc, oracle, monkeypatch):
    torch = cuda
    knobs.setenv("HC_SEG_MIN_MSGS", "1")  # every whole-message batch is offered to the stream
    rng = np.random.default_rng(404)
    n = 1500
    host = rng.integers(0, 256, n * 16384 + 8192, dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    base_off = np.arange(n, dtype=np.uint64) * 16384
    base_len = (4096 * rng.integers(1, 5, n)).astype(np.uint32)
    blk_want = oracle.crc32_blocks(host, off=base_off, lens=base_len)
    rec_len = rng.integers(64, 9000, n).astype(np.uint64)
    rec_off = np.zeros(n, dtype=np.uint64)
    rec_off[1:] = np.cumsum(rec_len[:-1], dtype=np.uint64)
    rec_off += np.uint64(5)
    rec_want = oracle.crc32_messages(host, rec_off, rec_len.astype(np.uint32), threads=8)
    gap_off = rec_off.copy()
    gap_off[n // 3:] += np.uint64(1)
    gap_want = oracle.crc32_messages(host, gap_off, rec_len.astype(np.uint32), threads=8)
    ovl_off = rec_off.copy()
    ovl_off[n // 3:] -= np.uint64(1)  # records n/3 - 1 and n/3 overlap: the stream's fallback
    ovl_want = oracle.crc32_messages(host, ovl_off, rec_len.astype(np.uint32), threads=8)

    def variant(k):
        """(off, len, flags, want) of call k of a thread"""
        kind = k % 4
        if kind == 0:
            return base_off, base_len, 0, blk_want
        if kind == 1:
            off, lens = base_off.copy(), base_len.copy()
            pos = (k * 37) % n
            if k % 8 == 1:
                off[pos] += 3
            else:
                lens[pos] -= 100
            want = blk_want.copy()
            want[pos] = oracle.crc32_blocks(host, off=off[pos:pos + 1], lens=lens[pos:pos + 1])[0]
            return off, lens, 0, want
        if kind == 2:
            return rec_off, rec_len.astype(np.uint32), hc.HC_F_MESSAGES, rec_want
        if k % 8 == 3:  # sorted with a gap: the stream's gapped mode
            return gap_off, rec_len.astype(np.uint32), hc.HC_F_MESSAGES, gap_want
        return ovl_off, rec_len.astype(np.uint32), hc.HC_F_MESSAGES, ovl_want

    errors = []

    def worker(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for k in range(t, t + 24):
                    off, lens, flags, want = variant(k)
                    doff = torch.from_numpy(off.view(np.int64)).cuda()
                    dlen = torch.from_numpy(lens.view(np.int32)).cuda()
                    out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
                    hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=n, flags=flags, stream=s)
                    s.synchronize()
                    got = out.cpu().numpy().view(np.uint32)
                    bad = np.nonzero(got != want)[0]
                    if bad.size:
                        errors.append((t, k, k % 4, bad[:5].tolist()))
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    [x.start() for x in th]
    [x.join(timeout=300) for x in th]
    assert not any(x.is_alive() for x in th)
    assert not errors, errors[:8]
