"""BASELINE.json configs[4] (config 5) at its full size: 10M WAL records of
64 B - 64 KiB (log-uniform), framed into 4 KiB blocks exactly as
lsm/wal/wal.go:177-283 (tools/walgen.c, byte-identical to the oracle's
framing: tests/test_walgen.py).  That is 26.3M blocks, 100 GiB in host memory,
the blocks starting where the WAL segment files put them.

- Every block's CRC word through the host-resident entry (hc_crc32_blocks:
  pageable image, staged over PCIe) against the oracle's restatement of
  crc_util.go's arithmetic on all 26.3M blocks, and against the word the
  writer stamped.
- The batched CheckBlockIntegrity (hc_verify_blocks, recoverMemtable's
  per-block check, wal.go:383) over the whole image: clean, then with one
  corrupted block found at its index with the reference's error text.
- The per-record variant on the device: GetCRC of all 10M records packed back
  to back in HBM (the packed-record stream), every word against the oracle
  (the span copied back in 4 GiB segments); the same records with a 17-B WAL
  header gap before each (the gapped stream), every word against the oracle
  again (its own copy-back of the gapped span); and word for word against
  k_crc_any (an overlap forces the fallback).

Host memory: ~108 GB (one image); the box allows ~270 GiB per command.

The file is named test_gpu_zz_* so that it is collected after every other GPU
test (tests/conftest.py also moves it last, and
tests/test_collection_order.py asserts the order): under `pytest -x` a failure
here can never leave the parity suite unreached.  Before allocating, each test
compares its need with the cgroup's memory limit and MemAvailable (host) or
the device's free memory, and FAILS with those numbers when it does not fit --
no skip, and no OOM kill of the whole pytest process."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NREC = 10_000_000
SEED = 0x57414C


def host_memory_room():
    """(bytes this process may still allocate, description): the smaller of
    /proc/meminfo's MemAvailable and the cgroup limit minus its usage (v2
    memory.max / memory.current, or v1 memory.limit_in_bytes / usage_in_bytes)."""
    avail = None
    with open("/proc/meminfo") as f:
        for line in f:
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    parts = [f"MemAvailable {avail / 2**30:.1f} GiB"]
    room = avail
    for lim_p, use_p in (("/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory.current"),
                         ("/sys/fs/cgroup/memory/memory.limit_in_bytes",
                          "/sys/fs/cgroup/memory/memory.usage_in_bytes")):
        try:
            with open(lim_p) as f:
                lim = f.read().strip()
            with open(use_p) as f:
                use = int(f.read().strip())
        except OSError:
            continue
        if lim == "max" or int(lim) >= 1 << 60:
            parts.append(f"cgroup {lim_p}: unlimited")
        else:
            free = int(lim) - use
            parts.append(f"cgroup {lim_p} {int(lim) / 2**30:.1f} GiB, used {use / 2**30:.1f} GiB")
            room = free if room is None else min(room, free)
        break
    return room, "; ".join(parts)


def require_host_bytes(need):
    room, desc = host_memory_room()
    assert room is None or room >= need, (
        f"config 5 needs {need / 2**30:.1f} GiB of host memory; this box has {room / 2**30:.1f} GiB ({desc})")


def require_device_bytes(torch, need):
    free, total = torch.cuda.mem_get_info()
    assert free >= need, (
        f"config 5 needs {need / 2**30:.1f} GiB on the device; {free / 2**30:.1f} of {total / 2**30:.1f} GiB free")


def _walgen():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import walgen
    return walgen


def test_config5_wal_blocks_full_size(cuda, hc, oracle):
    walgen = _walgen()
    plan = walgen.WalPlan(SEED, nrec=NREC)
    nb = plan.nblocks
    assert nb > 26_000_000
    require_host_bytes(nb * 4096 + (4 << 30))  # the image + pipelines, the oracle's words, headroom
    host = np.empty(nb * 4096, dtype=np.uint8)
    step = 1 << 18
    for b0 in range(0, nb, step):
        b1 = min(nb, b0 + step)
        plan.render(b0, b1, out=host[b0 * 4096:b1 * 4096], threads=16)
    try:
        got = hc.crc32_blocks(host, stride=4096, ulen=4096, nblocks=nb)
        want = oracle.crc32_blocks(host, stride=4096, ulen=4096, nblocks=nb, threads=16)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, bad[:8]
        stamped = host.reshape(nb, 4096)[:, :4].copy().view("<u4").reshape(-1)
        assert np.array_equal(stamped, want), "the writer's stamped words differ from the oracle's"
        err, bm, fb = hc.verify_blocks(host, stride=4096, ulen=4096, nblocks=nb)
        assert err is None and fb == -1 and not bm.any()
        victim = (2 * nb) // 3 + 1
        host[victim * 4096 + 2000] ^= 0x10
        err, bm, fb = hc.verify_blocks(host, stride=4096, ulen=4096, nblocks=nb)
        host[victim * 4096 + 2000] ^= 0x10
        assert str(err) == "CRC mismatch in block" and fb == victim
        assert int(np.unpackbits(bm.view(np.uint8)).sum()) == 1 and (bm[victim >> 5] >> (victim & 31)) & 1
    finally:
        del host


def oracle_all(buf, off, sizes, got, oracle, seg_cap=4 << 30):
    """Every record's word against the oracle: the span back to the host in
    segments of at most seg_cap bytes that end on record boundaries."""
    n = len(off)
    i = 0
    while i < n:
        lo = int(off[i])
        j = max(i + 1, int(np.searchsorted(off, np.uint64(lo + seg_cap), side="left")))
        while j > i + 1 and int(off[j - 1]) + int(sizes[j - 1]) > lo + seg_cap:
            j -= 1
        hi = int(off[j - 1]) + int(sizes[j - 1])
        seg = buf[lo:hi].cpu().numpy()
        want = oracle.crc32_messages(seg, off[i:j] - np.uint64(lo), sizes[i:j], threads=16)
        bad = np.flatnonzero(got[i:j] != want)
        assert bad.size == 0, (i + bad[:8])
        del seg
        i = j


def test_config5_records_full_size_on_device(cuda, hc, oracle):
    torch = cuda
    walgen = _walgen()
    sizes = np.zeros(NREC, dtype=np.uint32)
    walgen.lib().wg_record_sizes(SEED, NREC, 64, 65536, sizes.ctypes.data)
    off = np.zeros(NREC, dtype=np.uint64)
    off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    off += np.uint64(3)  # back to back from an odd address
    gp = off + np.arange(NREC, dtype=np.uint64) * np.uint64(17)  # the gapped layout (below)
    total = (int(gp[-1]) + int(sizes[-1]) + 64 + (1 << 20) - 1) >> 20 << 20
    assert total > 90e9
    require_device_bytes(torch, total + NREC * 16 + (2 << 30))
    require_host_bytes((6 << 30))  # the 4 GiB segments copied back for the oracle
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    hc.dev_fill_range(buf, 0x5C, 0, total >> 20, stride=1 << 20, ulen=1 << 20)  # every byte, in 1 MiB blocks
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    dlen = torch.from_numpy(sizes.view(np.int32)).cuda()
    out = torch.empty(NREC, dtype=torch.int32, device="cuda")
    hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=NREC, flags=hc.HC_F_MESSAGES)
    torch.cuda.synchronize()
    assert hc.seg_mode() == "packed", "10M packed records should take the packed-record stream"
    got = out.cpu().numpy().view(np.uint32).copy()
    # every record against the oracle, packed and gapped
    oracle_all(buf, off, sizes, got, oracle)
    # the same records with a 17-B gap before each (WAL headers between the
    # payloads, wal_header.go:5-23): the stream over 2n events
    doff.copy_(torch.from_numpy(gp.view(np.int64)))
    hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=NREC, flags=hc.HC_F_MESSAGES)
    torch.cuda.synchronize()
    assert hc.seg_mode() == "gapped", "sorted records with 17-B gaps should take the gapped stream"
    gotg = out.cpu().numpy().view(np.uint32).copy()
    oracle_all(buf, gp, sizes, gotg, oracle)
    # every word against k_crc_any: the gapped batch with record 0 one byte
    # longer overlaps record 1 (17-B gap -> -1): the device flag sends it there;
    # records 1.. are the gapped stream's words
    l2 = sizes.copy()
    l2[0] += 18
    dlen.copy_(torch.from_numpy(l2.view(np.int32)))
    hc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=NREC, flags=hc.HC_F_MESSAGES)
    torch.cuda.synchronize()
    assert not hc.seg_taken()
    got2 = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got2[1:], gotg[1:])
