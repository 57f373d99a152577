"""Row f1's caller-side rule, driven through the C ABI (CPU suite).

integration/go/lsm/block_manager/block_manager_gpu.go changes the block
cache's value to (data, verified, exposed) so ReadFromDisk skips the CRC of
cache entries it can trust.  No Go toolchain exists here or on the GPU box, so
this file restates both block managers over an in-memory disk, op for op:

  * RefBM   -- /root/reference/lsm/block_manager/block_manager.go:72-242: the
               cache holds the caller's slices (aliases), ReadFromDisk checks
               every block it reads (:215) with the oracle's
               CheckBlockIntegrity;
  * PatchBM -- block_manager_gpu.go: WriteBlock caches a copy, verified only
               if its CRC checks; ReadBlock hands out the cached slice and
               marks the entry exposed; ReadFromDisk reads every touched block
               and calls hc_read_from_disk_v (hunddb_amd.crc.ReadFromDisk) with
               the mask of trusted entries.

Both run the same operation sequences (the PersistLSM raw write,
lsm.go:148-156 + LoadLSM's reads :281,295; wal_test.go:878-898's
ReadBlock-corrupt-WriteBlock; a caller writing into a ReadBlock slice; random
sequences) and must return identical (payload, final offset, error).  The
reads stay under 256 blocks, where the library verifies on the host CPU, so
this runs without a GPU; tests/test_gpu_parity.py covers the GPU batch.
"""
import numpy as np
import pytest

BS = 4096


class Disk:
    """Files as byte arrays; a read past the end gives zeros (block_manager.go:135-140)."""

    def __init__(self):
        self.files = {}

    def read(self, path, idx, bs):
        f = self.files.get(path, bytearray())
        blk = bytearray(bs)
        chunk = f[idx * bs:(idx + 1) * bs]
        blk[:len(chunk)] = chunk
        return blk

    def write(self, path, idx, data, bs=BS):  # writeBlockToDisk (:144-158): at idx * blockSize
        f = self.files.setdefault(path, bytearray())
        end = idx * bs + len(data)
        if len(f) < end:
            f.extend(bytes(end - len(f)))
        f[idx * bs:end] = bytes(data)


class RefBM:
    """block_manager.go:72-242 (the cache holds aliases of callers' slices)."""

    def __init__(self, disk, oracle, bs=BS):
        self.disk, self.O, self.bs, self.cache = disk, oracle, bs, {}

    def ReadBlock(self, loc):  # :72-98
        if loc not in self.cache:
            self.cache[loc] = self.disk.read(loc[0], loc[1], self.bs)
        return self.cache[loc]

    def WriteBlock(self, loc, data):  # :101-114
        self.disk.write(loc[0], loc[1], data)
        self.cache[loc] = data

    def WriteToDisk(self, data, path, start):  # :165-181 (slices alias `data`)
        mv = memoryview(data)
        for i in range(len(data) // self.bs):
            self.WriteBlock((path, start // self.bs + i), mv[i * self.bs:(i + 1) * self.bs])

    def evict(self, loc):
        self.cache.pop(loc, None)

    def ReadFromDisk(self, path, start, size):  # :189-242
        L = self.O.lib()
        idx, boff = start // self.bs, max(start % self.bs, 4)
        out, rem = bytearray(), size
        while rem > 0:
            blk = bytes(self.ReadBlock((path, idx)))
            rc = L.oc_check_block_integrity(blk, len(blk))
            if rc:
                return None, 0, L.oc_strerror(rc).decode()
            take = min(rem, self.bs - boff)
            out += blk[boff:boff + take]
            rem -= take
            idx += 1
            boff = 4
        final = L.oc_size_after_adding_crcs(L.oc_size_without_crcs(start) + size)
        return bytes(out), final, None


class Entry:
    def __init__(self, data, verified=False):
        self.data, self.verified, self.exposed = data, verified, False

    def trusted(self):
        return self.verified and not self.exposed


class PatchBM:
    """integration/go/lsm/block_manager/block_manager_gpu.go over the C ABI."""

    def __init__(self, disk, hc, bs=BS):
        self.disk, self.hc, self.bs, self.cache = disk, hc, bs, {}
        self.hashed = []  # blocks hashed per ReadFromDisk (hc.last_hashed())

    def _cached(self, loc):  # readCached
        if loc not in self.cache:
            self.cache[loc] = Entry(self.disk.read(loc[0], loc[1], self.bs))
        return self.cache[loc]

    def ReadBlock(self, loc):
        e = self._cached(loc)
        e.exposed = True
        return e.data

    def WriteBlock(self, loc, data):
        self.disk.write(loc[0], loc[1], data)
        copy = bytearray(data)
        self.cache[loc] = Entry(copy, self.hc.CheckBlockIntegrity(copy) is None)

    def WriteToDisk(self, data, path, start):
        mv = memoryview(data)
        for i in range(len(data) // self.bs):
            self.WriteBlock((path, start // self.bs + i), mv[i * self.bs:(i + 1) * self.bs])

    def evict(self, loc):
        self.cache.pop(loc, None)

    def ReadFromDisk(self, path, start, size):
        k = self.hc.read_blocks_touched(self.bs, start, size)
        first = start // self.bs
        entries = [self._cached((path, first + i)) for i in range(k)]
        mask = np.zeros(max(1, (k + 31) // 32), dtype=np.uint32)
        for i, e in enumerate(entries):
            if e.trusted():
                mask[i >> 5] |= np.uint32(1 << (i & 31))
        raw = b"".join(bytes(e.data) for e in entries)
        out, final, err = self.hc.ReadFromDisk(raw, self.bs, start, size, verified=mask)
        self.hashed.append(self.hc.last_hashed())
        for i, e in enumerate(entries):
            if (int(mask[i >> 5]) >> (i & 31)) & 1:
                e.verified = True
        return out, final, None if err is None else str(err)


@pytest.fixture
def pair(hc, oracle):
    disk_r, disk_p = Disk(), Disk()
    return RefBM(disk_r, oracle), PatchBM(disk_p, hc)


def both(pair, op, *args):
    r, p = pair
    a = getattr(r, op)(*args)
    b = getattr(p, op)(*args)
    return a, b


def framed(hc, rng, nbytes):
    return hc.AddCRCsToData(bytes(rng.integers(0, 256, nbytes, dtype=np.uint8)))


def test_persist_lsm_raw_write_is_caught(hc, oracle, pair):
    """PersistLSM writes lsm.serialize() WITHOUT AddCRCsToData (lsm.go:148-156)
    and LoadLSM reads it back with ReadFromDisk (lsm.go:281,295): the reference
    fails the read with "CRC mismatch in block" (block_manager.go:215), and so
    must the patched cache -- the raw block is cached unverified."""
    r, p = pair
    rng = np.random.default_rng(1)
    raw = bytearray(rng.integers(0, 256, 3 * BS, dtype=np.uint8))
    for bm in pair:
        bm.WriteToDisk(bytearray(raw), "lsm.db", 0)
    assert not any(e.verified for e in p.cache.values())
    a, b = both(pair, "ReadFromDisk", "lsm.db", 0, 8)
    assert a == b == (None, 0, "CRC mismatch in block")
    assert hc.last_bad_block() == 0
    a, b = both(pair, "ReadFromDisk", "lsm.db", 8 + 4, 5000)
    assert a == b and b[2] == "CRC mismatch in block"


def test_framed_write_is_trusted_and_skipped(hc, oracle, pair):
    """Blocks written framed (AddCRCsToData before WriteToDisk) are cached
    verified: a read returns the reference's bytes without hashing them."""
    r, p = pair
    data = framed(hc, np.random.default_rng(2), 10 * 4092 + 100)
    for bm in pair:
        bm.WriteToDisk(bytearray(data), "sst_1.db", 0)
    assert all(e.trusted() for e in p.cache.values())
    a, b = both(pair, "ReadFromDisk", "sst_1.db", 4, 9 * 4092)
    assert a == b and b[2] is None
    assert p.hashed[-1] == 0


def test_wal_corruption_rewrite_is_caught(hc, oracle, pair):
    """wal_test.go:878-898: ReadBlock, flip a payload byte in the returned
    slice, WriteBlock it back; the next read must fail the CRC check."""
    r, p = pair
    data = framed(hc, np.random.default_rng(3), 4 * 4092)
    for bm in pair:
        bm.WriteToDisk(bytearray(data), "wal_1.log", 0)
    assert both(pair, "ReadFromDisk", "wal_1.log", 4, 4 * 4092)[0][2] is None
    off = 4 + 9 + 10  # CRC_SIZE + HEADER_TOTAL_SIZE + 10
    for bm in pair:
        blk = bm.ReadBlock(("wal_1.log", 0))
        blk[off] ^= 0xFF
        bm.WriteBlock(("wal_1.log", 0), blk)
    assert not p.cache[("wal_1.log", 0)].verified
    a, b = both(pair, "ReadFromDisk", "wal_1.log", 4, 4 * 4092)
    assert a == b == (None, 0, "CRC mismatch in block")


def test_caller_writes_into_read_block_slice(hc, oracle, pair):
    """ReadBlock returns the cached slice itself (block_manager.go:76): a caller
    that writes into it, with no WriteBlock, changes what the next ReadFromDisk
    sees.  The reference then fails the CRC; the patched cache must not skip
    the entry it handed out, even one it had verified before."""
    r, p = pair
    data = framed(hc, np.random.default_rng(4), 3 * 4092)
    for bm in pair:
        bm.WriteToDisk(bytearray(data), "sst_2.db", 0)
        assert bm.ReadFromDisk("sst_2.db", 4, 3 * 4092)[2] is None
    for bm in pair:
        bm.ReadBlock(("sst_2.db", 1))[100] ^= 1
    a, b = both(pair, "ReadFromDisk", "sst_2.db", 4, 3 * 4092)
    assert a == b == (None, 0, "CRC mismatch in block")
    assert hc.last_bad_block() == 1
    # restored by the caller: the reference reads clean again, so must the patch,
    # which keeps re-checking the exposed entry
    for bm in pair:
        bm.ReadBlock(("sst_2.db", 1))[100] ^= 1
    a, b = both(pair, "ReadFromDisk", "sst_2.db", 4, 3 * 4092)
    assert a == b and b[2] is None
    assert p.hashed[-1] == 1


def test_caller_mutating_its_buffer_after_write_does_not_reach_the_cache(hc, oracle):
    """The one documented difference: the reference
    caches the slice the caller passed to WriteBlock, the patch a copy.  A caller
    that writes into its buffer after WriteToDisk changes the reference's cached
    view but not the disk; the patched cache holds what is on disk, i.e. what the
    reference itself returns once the entry is evicted."""
    rng = np.random.default_rng(5)
    data = framed(hc, rng, 2 * 4092)
    r, p = RefBM(Disk(), oracle), PatchBM(Disk(), hc)
    buf_r, buf_p = bytearray(data), bytearray(data)
    r.WriteToDisk(buf_r, "f", 0)
    p.WriteToDisk(buf_p, "f", 0)
    buf_r[5000] ^= 1
    buf_p[5000] ^= 1
    assert r.ReadFromDisk("f", 4, 2 * 4092)[2] == "CRC mismatch in block"
    got = p.ReadFromDisk("f", 4, 2 * 4092)
    r.evict(("f", 1))
    assert got == r.ReadFromDisk("f", 4, 2 * 4092) and got[2] is None


@pytest.mark.parametrize("seed", range(12))
def test_random_operation_sequences(hc, oracle, seed):
    """Random interleavings of framed and raw writes, single-block rewrites
    (clean and corrupt), caller writes into ReadBlock slices, evictions and
    ReadFromDisk at random offsets and sizes (start inside the CRC field,
    block-crossing, past the end of the file): every read returns the same
    (payload, final offset, error) from both block managers."""
    rng = np.random.default_rng(1000 + seed)
    r, p = RefBM(Disk(), oracle), PatchBM(Disk(), hc)
    paths = ["a.db", "b.db"]
    nblk = 24
    seeded = {path: framed(hc, rng, nblk * 4092) for path in paths}
    for path in paths:
        r.WriteToDisk(bytearray(seeded[path]), path, 0)
        p.WriteToDisk(bytearray(seeded[path]), path, 0)
    reads = 0
    for step in range(120):
        path = paths[int(rng.integers(0, 2))]
        op = int(rng.integers(0, 10))
        blk = int(rng.integers(0, nblk))
        if op == 0:  # rewrite a run framed
            n = int(rng.integers(1, 6)) * 4092
            d = framed(hc, rng, n)
            r.WriteToDisk(bytearray(d), path, blk * BS)
            p.WriteToDisk(bytearray(d), path, blk * BS)
        elif op == 1:  # raw write (no CRCs), as PersistLSM
            d = rng.integers(0, 256, BS * int(rng.integers(1, 3)), dtype=np.uint8).tobytes()
            r.WriteToDisk(bytearray(d), path, blk * BS)
            p.WriteToDisk(bytearray(d), path, blk * BS)
        elif op == 2:  # ReadBlock, corrupt, WriteBlock (wal_test.go:878-898)
            pos = int(rng.integers(0, BS))
            for bm in (r, p):
                b = bm.ReadBlock((path, blk))
                b[pos] ^= 0x40
                bm.WriteBlock((path, blk), b)
        elif op == 3:  # caller writes into a ReadBlock slice, no WriteBlock
            pos = int(rng.integers(0, BS))
            for bm in (r, p):
                bm.ReadBlock((path, blk))[pos] ^= 0x08
        elif op == 4:  # restamp a block read through ReadBlock (AddCRCToBlockData + WriteBlock)
            for bm in (r, p):
                b = bytearray(bm.ReadBlock((path, blk)))
                hc.AddCRCToBlockData(b)
                bm.WriteBlock((path, blk), b)
        elif op == 5:
            r.evict((path, blk))
            p.evict((path, blk))
        else:  # ReadFromDisk
            start = blk * BS + int(rng.choice([0, 2, 4, 5, int(rng.integers(0, BS))]))
            size = int(rng.integers(1, 6 * BS))
            a = r.ReadFromDisk(path, start, size)
            b = p.ReadFromDisk(path, start, size)
            assert a == b, (seed, step, path, start, size, a[2], b[2])
            reads += 1
    assert reads > 20
