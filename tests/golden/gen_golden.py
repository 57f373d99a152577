#!/usr/bin/env python3
"""Generate the golden fixtures that pin the CPU oracle (oracle/hc_oracle.c).

Run in the build container:  python3 tests/golden/gen_golden.py
Writes tests/golden/golden.json.

Source of truth: Python's zlib.crc32 (zlib 1.2.11), which computes the same
CRC-32/ISO-HDLC function as Go's crc32.ChecksumIEEE used by
/root/reference/utils/crc/crc_util.go:16,94.  The reference (Go) cannot be
built or run here (no Go toolchain) and ships no CRC golden
vectors of its own, so the expected outputs of every utils/crc function below
are derived from zlib plus a line-by-line Python restatement of
crc_util.go:10-122 and, for the structural fixtures, of the WAL framing in
lsm/wal/wal.go:177-283 / wal_header.go:5-77 / model/record/record.go:85-119.
This file reads nothing under /root/reference at run time.
"""
import hashlib
import json
import math
import os
import struct
import zlib

import numpy as np

BLOCK_SIZE = 4096  # crc_util.go:11
CRC_SIZE = 4       # crc_util.go:12
M64 = (1 << 64) - 1


# ---- utils/crc restated (Go semantics) -----------------------------------
def get_crc(b):                      # crc_util.go:15-17
    return zlib.crc32(bytes(b)) & 0xFFFFFFFF


def add_crc_to_block_data(b):        # crc_util.go:21-33 (in place)
    b = bytearray(b)
    if len(b) < CRC_SIZE:
        return b
    b[0:4] = struct.pack("<I", get_crc(b[4:]))
    return b


def add_crcs_to_data(src):           # crc_util.go:41-64
    per = BLOCK_SIZE - CRC_SIZE
    out = bytearray()
    for i in range(0, len(src), per):
        blk = bytearray(BLOCK_SIZE)
        chunk = src[i:i + per]
        blk[4:4 + len(chunk)] = chunk
        out += add_crc_to_block_data(blk)
    return out


def size_after_adding_crcs(n):       # crc_util.go:69-74, float64 math
    nb = int(math.ceil(float(n) / float(BLOCK_SIZE - CRC_SIZE)))
    return (n + nb * CRC_SIZE) & M64


def size_without_crcs(n):            # crc_util.go:79-83, uint64 wrap
    nb = int(math.ceil(float(n) / float(BLOCK_SIZE)))
    return (n - nb * CRC_SIZE) & M64


def check_block_integrity(b):        # crc_util.go:88-100
    if len(b) < CRC_SIZE:
        return "invalid block data"
    if struct.unpack("<I", bytes(b[0:4]))[0] != get_crc(b[4:]):
        return "CRC mismatch in block"
    return None


def fix_last_block_crc(b):           # crc_util.go:106-122
    b = bytearray(b)
    if len(b) < BLOCK_SIZE:
        return "data is too short to contain a complete block", b
    last = (len(b) // BLOCK_SIZE - 1) * BLOCK_SIZE
    b[last:last + BLOCK_SIZE] = add_crc_to_block_data(b[last:last + BLOCK_SIZE])
    return None, b


def read_from_disk(image, B, start, size):
    """lsm/block_manager/block_manager.go:189-242 over an in-memory file image
    (blocks from index start//B on; zeros past the end, as readBlockFromDisk's
    short read leaves them).  Returns (payload, final_offset, err, bad_block)."""
    off = start % B
    if off < CRC_SIZE:                                  # :198-201
        off = CRC_SIZE
    out, cur, rem = bytearray(), 0, size
    while rem > 0:
        blk = bytes(image[cur * B:(cur + 1) * B]).ljust(B, b"\0")   # ReadBlock
        err = check_block_integrity(blk)                # :215
        if err is not None:
            return None, 0, err, cur
        take = min(rem, B - off)                        # :221-225
        out += blk[off:off + take]
        rem -= take
        cur += 1
        off = CRC_SIZE
    return bytes(out), size_after_adding_crcs((size_without_crcs(start) + size) & M64), None, -1  # uint64 wrap


def wal_replay(blocks, bs, start_block=0, start_off=CRC_SIZE, max_records=0):
    """lsm/wal/wal.go:362-455 (recoverMemtable + processBlockForRecovery) over
    written blocks; one call = one memtable, max_records = IsFull (0: never).
    Returns (records, err, bad_block, pos).  Where Go panics (header or payload
    past the block end) this returns "truncated"."""
    frag, recs = bytearray(), []
    blk, off = start_block, start_off
    while blk < len(blocks):
        b = blocks[blk]
        err = check_block_integrity(b)
        if err is not None:
            return recs, err, blk, (blk, off)
        full = False
        while off < bs:
            if not any(b[off:]):                       # padding (:415-419)
                frag.clear()
                break
            if off + WAL_HDR > bs:
                return recs, "truncated", -1, (blk, off)
            size, typ, _log = struct.unpack("<QBQ", bytes(b[off:off + WAL_HDR]))
            off += WAL_HDR
            if size > bs - off:
                return recs, "truncated", -1, (blk, off)
            pay = bytes(b[off:off + size])
            off += size
            if typ == 4:
                recs.append(pay)
            elif typ in (1, 2):
                frag += pay
                continue
            elif typ == 3:
                frag += pay
                recs.append(bytes(frag))
                frag.clear()
            else:
                return recs, "unknown fragment type", -1, (blk, off)
            if max_records and len(recs) >= max_records:
                full = True
                break
        blk, off = blk + 1, CRC_SIZE                   # :392-393
        if full:
            break
    return recs, None, -1, (blk, off)


# ---- synthetic inputs: splitmix64 finaliser over (seed, block, word) -----
def splitmix64(seed, block, words):
    w = np.asarray(words, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + ((np.uint64(block) << np.uint64(21)) + w) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def fill_block(seed, block, length):
    return splitmix64(seed, block, np.arange(length // 8)).astype("<u8").tobytes()


def mixed_size(seed, block):
    r = int(splitmix64(seed ^ 0x5A5A5A5A5A5A5A5A, block, [(1 << 21) - 1])[0])
    return 4096 << (r % 3)


# ---- WAL framing restated (lsm/wal/wal.go:177-283) -----------------------
WAL_HDR = 17  # wal_header.go:16


def wal_payload_byte(seed, rec, total_len, pos):
    if pos < 8:
        return (rec >> (8 * pos)) & 0xFF                       # timestamp
    if pos == 8:
        return 0                                               # tombstone
    ksz = min(16, total_len - 25)                              # records are >= 25 bytes
    if pos < 17:
        return (ksz >> (8 * (pos - 9))) & 0xFF                 # key size
    if pos < 25:
        return ((total_len - 25 - ksz) >> (8 * (pos - 17))) & 0xFF  # value size
    w = int(splitmix64(seed, rec, [(pos - 25) >> 3])[0])
    return (w >> (8 * ((pos - 25) & 7))) & 0xFF


def wal_frame(seed, sizes, bs=4096, log_size=16):
    blocks = []
    st = {"cur": bytearray(bs), "off": CRC_SIZE, "in_log": 0, "log": 1}
    refused = 0

    def flush():                                   # wal.go:260-271
        blocks.append(bytes(add_crc_to_block_data(st["cur"])))
        st["in_log"] += 1

    def new_block():                               # wal.go:273-283
        st["cur"] = bytearray(bs)
        st["off"] = CRC_SIZE
        if st["in_log"] >= log_size:
            st["log"] += 1
            st["in_log"] = 0

    def write_to_block(rec, pay_off, n, total, typ):   # wal.go:229-257
        if st["off"] + WAL_HDR + n > bs:
            return False
        o = st["off"]
        st["cur"][o:o + WAL_HDR] = struct.pack("<QBQ", n, typ, st["log"])
        st["cur"][o + WAL_HDR:o + WAL_HDR + n] = bytes(
            wal_payload_byte(seed, rec, total, pay_off + k) for k in range(n))
        st["off"] += WAL_HDR + n
        if st["off"] == bs:
            flush()
            new_block()
        return True

    for rec, S in enumerate(sizes):                # wal.go:177-195
        need = WAL_HDR + S
        if bs - st["off"] < need:
            flush()
            new_block()
            if need > bs:                          # wal.go:199-225
                maxp = bs - WAL_HDR - CRC_SIZE
                nf = int(math.ceil(S / maxp))
                po = 0
                for i in range(nf):
                    fl = min(maxp, S - po)
                    typ = 1 if i == 0 else (3 if i == nf - 1 else 2)
                    write_to_block(rec, po, fl, S, typ)
                    po += fl
                continue
        if not write_to_block(rec, 0, S, S, 4):
            refused += 1
    flush()                                        # Close()
    return blocks, refused


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def main():
    g = {"generator": "tests/golden/gen_golden.py", "zlib_version": zlib.ZLIB_VERSION,
         "crc": "CRC-32/ISO-HDLC (Go crc32.ChecksumIEEE)"}
    rng = np.random.default_rng(0x48756E64)

    # 1. known answers
    g["known"] = {
        "check_123456789": get_crc(b"123456789"),
        "empty": get_crc(b""),
        "zero_payload": {str(B): get_crc(bytes(B - 4)) for B in (4096, 8192, 16384)},
        "vectors": [],
    }
    for n in [1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 32, 63, 64, 65, 127, 128, 255, 256, 1000, 1023,
              1024, 1025, 4092, 4095, 4096, 4097, 8188, 16380, 65536, 100003]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        g["known"]["vectors"].append({"hex": b.hex() if n <= 4096 else None,
                                      "seed_fill": None if n <= 4096 else [0x1234, n],
                                      "len": n, "crc": get_crc(b if n <= 4096 else
                                                               fill_block(0x1234, n, (n + 7) // 8 * 8)[:n])})

    # 2. per-function edge cases
    fx = {}
    fx["add_crc_to_block_data"] = []
    for n in [0, 1, 2, 3, 4, 5, 8, 4096, 8192]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        fx["add_crc_to_block_data"].append({"in": b.hex(), "out": add_crc_to_block_data(b).hex()})
    cbi = []
    for n in [0, 3]:
        cbi.append({"in": bytes(n).hex(), "err": check_block_integrity(bytes(n))})
    cbi.append({"in": bytes(4).hex(), "err": check_block_integrity(bytes(4))})  # CRC("")==0 -> ok
    for B in (4096, 8192, 16384):
        blk = add_crc_to_block_data(rng.integers(0, 256, B, dtype=np.uint8).tobytes())
        cbi.append({"in": blk.hex(), "err": check_block_integrity(blk)})
        flipped = bytearray(blk)
        bit = int(rng.integers(32, B * 8))
        flipped[bit // 8] ^= 1 << (bit % 8)
        cbi.append({"in": flipped.hex(), "err": check_block_integrity(flipped), "flipped_bit": bit})
        hdr = bytearray(blk)
        hdr[1] ^= 0x10  # corrupt the stored CRC itself
        cbi.append({"in": hdr.hex(), "err": check_block_integrity(hdr)})
    fx["check_block_integrity"] = cbi
    fx["add_crcs_to_data"] = []
    for n in [0, 1, 4091, 4092, 4093, 8184, 8185, 12276, 50000]:
        src = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        out = add_crcs_to_data(src)
        fx["add_crcs_to_data"].append({
            "in": src.hex() if n <= 8185 else None, "seed_fill": None if n <= 8185 else [0x77, n],
            "len_out": len(out), "sha256": sha(out),
            "crcs": [struct.unpack("<I", out[i:i + 4])[0] for i in range(0, len(out), BLOCK_SIZE)]})
        if n > 8185:  # regenerate deterministically from the seed instead of storing hex
            src2 = fill_block(0x77, n, (n + 7) // 8 * 8)[:n]
            out2 = add_crcs_to_data(src2)
            fx["add_crcs_to_data"][-1].update({"len_out": len(out2), "sha256": sha(out2),
                                               "crcs": [struct.unpack("<I", out2[i:i + 4])[0]
                                                        for i in range(0, len(out2), BLOCK_SIZE)]})
    fx["fix_last_block_crc"] = []
    for n in [0, 4095, 4096, 8191, 8192, 12300]:
        src = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        err, out = fix_last_block_crc(src)
        fx["fix_last_block_crc"].append({"in": src.hex(), "err": err, "sha256": sha(out)})
    sizes = [0, 1, 2, 3, 4, 5, 4091, 4092, 4093, 4096, 4097, 8184, 8185, 8192, 8193,
             (1 << 53) - 1, (1 << 53) + 1, (1 << 63) + 12345, M64]
    fx["size_after_adding_crcs"] = [[n, size_after_adding_crcs(n)] for n in sizes]
    fx["size_without_crcs"] = [[n, size_without_crcs(n)] for n in sizes]
    g["functions"] = fx

    # 3. structural fixtures from the reference's own layouts
    wal = {}
    for name, recsizes in [("one_full_record", [35]),          # wal_test.go:230-279 shape
                           ("record_1_5_blocks", [6138]),       # wal_test.go:385-449
                           ("record_3_blocks", [12000]),        # wal_test.go:451-496
                           ("exact_fill", [4092 - 17 - 17 - 100, 100]),   # wal_test.go:1100-1162
                           ("refused_size", [4076, 64]),        # 4092 < 17+S <= 4096
                           ("mixed_small", [64, 300, 1000, 4000, 70, 5000, 64])]:
        blocks, refused = wal_frame(0xABCDEF, recsizes)
        wal[name] = {"seed": 0xABCDEF, "record_sizes": recsizes, "blocks": len(blocks),
                     "refused": refused, "sha256": [sha(b) for b in blocks],
                     "crcs": [struct.unpack("<I", b[:4])[0] for b in blocks]}
    g["wal"] = wal
    # WAL recovery (wal.go:362-455, row f3) over the same fixtures
    rep = {}
    for name, recsizes in [("one_full_record", [35]), ("record_1_5_blocks", [6138]),
                           ("record_3_blocks", [12000]), ("exact_fill", [4092 - 17 - 17 - 100, 100]),
                           ("refused_size", [4076, 64]),
                           ("mixed_small", [64, 300, 1000, 4000, 70, 5000, 64])]:
        blocks, _ = wal_frame(0xABCDEF, recsizes)
        for mr in (0, 1, 2):
            recs, err, bad, pos = wal_replay(blocks, 4096, max_records=mr)
            rep[f"{name}/max{mr}"] = {"fixture": name, "max_records": mr, "err": err, "bad_block": bad,
                                      "pos": list(pos), "lens": [len(r) for r in recs],
                                      "sha256": [sha(r) for r in recs]}
        if len(blocks) > 1:  # corrupt the last block: records before it are still returned
            bb = [bytearray(x) for x in blocks]
            bb[-1][100] ^= 1
            recs, err, bad, pos = wal_replay([bytes(x) for x in bb], 4096)
            rep[f"{name}/corrupt_last"] = {"fixture": name, "corrupt": [len(blocks) - 1, 100, 1],
                                           "max_records": 0, "err": err, "bad_block": bad, "pos": list(pos),
                                           "lens": [len(r) for r in recs], "sha256": [sha(r) for r in recs]}
    # hand-built blocks: unknown fragment type; header past the block end
    odd = {}
    b = bytearray(4096)
    b[4:21] = struct.pack("<QBQ", 10, 7, 1)
    b[21:31] = bytes(range(1, 11))
    odd["unknown_type"] = bytes(add_crc_to_block_data(b))
    b = bytearray(4096)
    b[4:21] = struct.pack("<QBQ", 4064, 4, 1)
    b[21:4085] = bytes((i * 7 + 1) & 0xFF for i in range(4064))
    b[4090] = 9                                          # 11 bytes left: a header cannot fit
    odd["truncated_header"] = bytes(add_crc_to_block_data(b))
    b = bytearray(4096)
    b[4:21] = struct.pack("<QBQ", 5000, 4, 1)            # payload past the block end
    b[21] = 1
    odd["truncated_payload"] = bytes(add_crc_to_block_data(b))
    # hand-built multi-block images: a FULL between fragments leaves the fragment
    # buffer alone (wal.go:432-437); padding clears it (:415-419); a LAST with
    # nothing pending is a record by itself
    def wal_block(items, pad_tail=True):
        b = bytearray(4096)
        off = 4
        for typ, pay in items:
            b[off:off + 17] = struct.pack("<QBQ", len(pay), typ, 1)
            b[off + 17:off + 17 + len(pay)] = pay
            off += 17 + len(pay)
        return bytes(add_crc_to_block_data(b))
    pb = lambda k, n: bytes(((i * 13 + k * 29 + 1) & 0xFF) or 1 for i in range(n))  # noqa: E731
    multi = {
        # (block 1 is filled to its end: no padding between the fragments)
        "full_between_fragments": [wal_block([(1, pb(1, 300)), (4, pb(2, 200)), (2, pb(3, 4092 - 51 - 500))]),
                                   wal_block([(4, pb(4, 50)), (3, pb(5, 70)), (4, pb(6, 10))])],
        "padding_clears_fragments": [wal_block([(4, pb(1, 40)), (1, pb(2, 500))]),
                                     wal_block([(3, pb(3, 60)), (1, pb(4, 30)), (3, pb(5, 30))])],
        "last_without_first": [wal_block([(3, pb(1, 80)), (3, pb(2, 90))]),
                               wal_block([(2, pb(3, 4075))]),
                               wal_block([(3, pb(4, 20)), (4, pb(5, 5))])],
    }
    for name, bl in multi.items():
        odd[name] = b"".join(bl)
    for name, blk in odd.items():
        recs, err, bad, pos = wal_replay([blk[i:i + 4096] for i in range(0, len(blk), 4096)], 4096)
        rep[f"hand/{name}"] = {"block_hex": blk.hex(), "max_records": 0, "err": err, "bad_block": bad,
                               "pos": list(pos), "lens": [len(r) for r in recs],
                               "sha256": [sha(r) for r in recs]}
    g["wal_replay"] = rep
    # global_key_dict header block: [crc4 | count u64 | zero pad], recomputed CRC
    # (utils/global_key_dict/global_key_dict_test.go:31-38 builds it by hand)
    hdr = bytearray(4096)
    hdr[4:12] = struct.pack("<Q", 7)
    g["global_key_dict_header"] = {"count": 7, "crc": get_crc(hdr[4:])}

    # 4. seeded synthetic batches
    seed = 0x48756E64
    crcs = []
    h = hashlib.sha256()
    for i in range(1000):                          # config 1: 1000 x 4 KiB
        b = fill_block(seed, i, 4096)
        h.update(b)
        crcs.append(get_crc(b[4:]))
    g["config1"] = {"seed": seed, "n": 1000, "block": 4096, "sha256_inputs": h.hexdigest(),
                    "crcs": crcs}
    mseed = 0x4D495845
    ms, mc = [], []
    for i in range(256):                           # config 3 shape, small
        s = mixed_size(mseed, i)
        b = fill_block(mseed, i, s)
        ms.append(s)
        mc.append(get_crc(b[4:]))
    g["mixed"] = {"seed": mseed, "n": 256, "sizes": ms, "crcs": mc}

    # 5. ReadFromDisk (block_manager.go:189-242) over framed images (f1)
    rrng = np.random.default_rng(0x52464431)
    rfd, images = [], {}
    for B in (4096, 8192):
        nb = 5
        image = bytearray()
        for i in range(nb):
            image += add_crc_to_block_data(rrng.integers(0, 256, B, dtype=np.uint8).tobytes())
        bad = bytearray(image)
        bad[3 * B + 1000] ^= 0x04                        # corrupt block 3
        for name, img in (("clean", image), ("bad3", bad)):
            for start, size in [(0, 0), (0, 1), (0, B - 4), (1, 10), (3, B), (4, B - 4), (5, B - 5),
                                (B - 1, 2), (B, 1), (B + 2, 3 * B), (B + 7, 4 * (B - 4) - 3),
                                (2 * B + 100, 5 * B)]:
                got, fo, err, badblk = read_from_disk(img, B, start, size)
                rfd.append({"block_size": B, "image": name, "start": start, "size": size,
                            "sha256": None if got is None else sha(got), "final_offset": fo,
                            "err": err, "bad_block": badblk})
        images[str(B)] = bytes(image).hex()       # small enough to store (5 blocks)
    g["read_from_disk"] = {"seed": 0x52464431, "blocks": 5, "flip": "image[3*B+1000] ^= 0x04",
                           "cases": rfd, "image_hex": images}

    # 6. row f4: MD5 (hashlib, the RFC 1321 function of Go crypto/md5) and the
    # Merkle tree of lsm/sstable/merkle_tree/merkle_tree.go restated below
    rfc = ["", "a", "abc", "message digest", "abcdefghijklmnopqrstuvwxyz",
           "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
           "1234567890" * 8]
    md5k = {"rfc1321": [[m, hashlib.md5(m.encode()).hexdigest()] for m in rfc]}
    rng = np.random.default_rng(0x4D4435)
    rnd = []
    for n in list(range(0, 130)) + [255, 256, 1000, 4092, 4096, 9815, 65536, 100000]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        rnd.append({"seed_len": n, "sha256": sha(b), "md5": hashlib.md5(b).hexdigest()})
    md5k["random"] = {"seed": 0x4D4435, "note": "rng = numpy default_rng(seed); b = rng.integers(0,256,n,uint8) in order",
                      "cases": rnd}
    g["md5"] = md5k

    def merkle_levels(leaves):  # NewMerkleTree(leaves, true) (:36-81) as level lists
        if not leaves:
            return [[hashlib.md5(b"").digest()]], 0
        lv = [list(leaves)]
        real = [len(leaves)]
        while len(lv[-1]) > 1:
            cur = lv[-1]
            if len(cur) % 2:
                cur.append(bytes(16))                    # neutral node (:60-66)
            lv.append([hashlib.md5(cur[i] + cur[i + 1]).digest() for i in range(0, len(cur), 2)])
            real.append(len(lv[-1]))
        return lv, real

    def merkle_serialize(leaves):  # Serialize (:173-187): DFS pre-order
        lv, real = merkle_levels(leaves)
        if not leaves:
            return lv[0][0]
        out, stack = [], [(len(lv) - 1, 0)]
        while stack:
            L, i = stack.pop()
            out.append(lv[L][i])
            if L > 0 and i < real[L]:
                stack += [(L - 1, 2 * i + 1), (L - 1, 2 * i)]
        return b"".join(out)

    # expected roots from the reference's own test (merkle_tree_test.go:11-21)
    ref_roots = [[["block1", "block2", "block3", "block4"], "52b6ec49b1ed0eed625adcef9073f0c2"],
                 [["block1", "block2", "block3"], "ac491d1ea728dc2fb488cf3bc8b3a898"],
                 [["block1", "block2"], "423a3d793bb8c91da536a90361dc09ff"],
                 [["block1"], "9dd085e96a8813854138d29b8a6fdf58"]]
    trees = []
    for n in list(range(0, 18)) + [31, 32, 33, 100, 255]:
        leaves = [hashlib.md5(b"record-%d" % i).digest() for i in range(n)]
        ser = merkle_serialize(leaves)
        trees.append({"n": n, "leaves": "md5(b'record-%d' % i)", "root": merkle_levels(leaves)[0][-1][0].hex(),
                      "serialized_nodes": len(ser) // 16, "serialized_sha256": sha(ser)})
    g["merkle"] = {"reference_test_roots": ref_roots, "trees": trees}

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as f:
        json.dump(g, f, indent=0)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
