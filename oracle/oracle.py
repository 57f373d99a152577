"""ctypes loader for the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  Never imported by hunddb_amd/.
"""
import ctypes
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
# HC_ORACLE_LIB: load another build (the ASan/UBSan build of `make -C oracle asan`)
_PATH = os.environ.get("HC_ORACLE_LIB") or os.path.join(_DIR, "liboracle.so")
_L = None


def build():
    subprocess.check_call(["make", "-s", "-C", _DIR])


def lib():
    global _L
    if _L is None:
        if not os.path.exists(_PATH):
            build()
        L = ctypes.CDLL(_PATH)
        P, S, U32, U64, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        for name, res, args in [
            ("oc_crc32_bitwise", U32, [U32, P, S]), ("oc_crc32_sarwate", U32, [U32, P, S]),
            ("oc_crc32_slicing8", U32, [U32, P, S]), ("oc_crc32_go_amd64", U32, [U32, P, S]),
            ("oc_have_pclmul", I, []), ("oc_checksum_ieee", U32, [P, S]),
            ("oc_strerror", ctypes.c_char_p, [I]), ("oc_get_crc", U32, [P, S]),
            ("oc_add_crc_to_block_data", None, [P, S]), ("oc_add_crcs_to_data", S, [P, S, P]),
            ("oc_size_after_adding_crcs", U64, [U64]), ("oc_size_without_crcs", U64, [U64]),
            ("oc_check_block_integrity", I, [P, S]), ("oc_fix_last_block_crc", I, [P, S]),
            ("oc_crc32_blocks", None, [P, P, P, U64, U32, P, S, I]),
            ("oc_crc32_messages", None, [P, P, P, P, S, I]),
            ("oc_splitmix64", U64, [U64, U64, U64]), ("oc_fill_block", None, [U64, U64, P, S]),
            ("oc_fill_blocks_mt", None, [U64, U64, U64, U64, P, I]),
            ("oc_mixed_size", U32, [U64, U64]),
            ("oc_wal_frame", U64, [U64, P, U64, U32, P, U64, I, P, P]),
            ("oc_wal_record_size", U32, [U64, U64, U32, U32]),
            ("oc_read_from_disk", I, [P, U64, U32, U64, U64, P, P, P]),
            ("oc_wal_replay", I, [P, U64, U32, U64, U64, U64, P, P, P, P, P, P, P]),
            ("oc_md5", None, [P, S, P]), ("oc_md5_messages", None, [P, P, P, P, S]),
            ("oc_merkle_root", None, [P, U64, P]), ("oc_merkle_serialize", U64, [P, U64, P]),
            ("oc_merkle_validate", I, [P, U64, P, U64, P, P, U64, P]),
            ("oc_merkle_validate_trees", I, [P, U64, P, U64, P, P, U64, P]),
        ]:
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _L = L
    return _L


class WalStats(ctypes.Structure):
    _fields_ = [("records", ctypes.c_uint64), ("blocks", ctypes.c_uint64),
                ("refused", ctypes.c_uint64), ("fragments", ctypes.c_uint64)]


def _p(a):
    return None if a is None else a.ctypes.data


def checksum(data) -> int:
    a = np.frombuffer(bytes(data), dtype=np.uint8)
    return int(lib().oc_checksum_ieee(_p(a) if a.size else None, a.size))


def crc32_blocks(buf: np.ndarray, off=None, lens=None, stride=4096, ulen=4096, nblocks=None, threads=8):
    """CRC of blk[4:len] per block (reference utils/crc CheckBlockIntegrity arithmetic)."""
    buf = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    o = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    l = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint32)
    n = nblocks if nblocks is not None else (len(o) if o is not None else len(l) if l is not None else buf.size // stride)
    out = np.zeros(n, dtype=np.uint32)
    lib().oc_crc32_blocks(_p(buf), _p(o), _p(l), stride, ulen, _p(out), n, threads)
    return out


def crc32_messages(buf: np.ndarray, off, lens, threads=8):
    buf = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    o = np.ascontiguousarray(off, dtype=np.uint64)
    l = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.zeros(len(o), dtype=np.uint32)
    lib().oc_crc32_messages(_p(buf), _p(o), _p(l), _p(out), len(o), threads)
    return out


def fill_blocks(seed, n, size=None, sizes=None):
    """Host copy of the synthetic batch hc_dev_fill_blocks writes (packed)."""
    if sizes is None:
        sizes = np.full(n, size, dtype=np.uint32)
    sizes = np.asarray(sizes, dtype=np.uint32)
    off = np.zeros(len(sizes), dtype=np.uint64)
    off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    buf = np.zeros(int(sizes.sum(dtype=np.uint64)), dtype=np.uint8)
    L = lib()
    base = buf.ctypes.data
    for i in range(len(sizes)):
        L.oc_fill_block(seed, i, base + int(off[i]), int(sizes[i]))
    return buf, off, sizes


def fill_range(seed, first, n, block_bytes, out=None, threads=16):
    """Blocks first .. first+n-1 of a uniform synthetic batch (the bytes
    hc_dev_fill_range writes for them), regenerated on the host by index."""
    if out is None:
        out = np.empty(n * block_bytes, dtype=np.uint8)
    assert out.size >= n * block_bytes and out.flags.c_contiguous
    lib().oc_fill_blocks_mt(seed, first, n, block_bytes, _p(out), threads)
    return out


def mixed_sizes(seed, n):
    L = lib()
    return np.array([L.oc_mixed_size(seed, i) for i in range(n)], dtype=np.uint32)


def wal_frame(seed, rec_sizes, bs=4096, max_blocks=None, stamp=True):
    rs = np.ascontiguousarray(rec_sizes, dtype=np.uint32)
    L = lib()
    st = WalStats()
    if max_blocks is None:
        L.oc_wal_frame(seed, _p(rs), len(rs), bs, None, 1 << 62, 0, ctypes.byref(st), None)
        max_blocks = st.blocks
    buf = np.zeros(max_blocks * bs, dtype=np.uint8)
    nxt = ctypes.c_uint64(0)
    nb = L.oc_wal_frame(seed, _p(rs), len(rs), bs, _p(buf), max_blocks, 1 if stamp else 0,
                        ctypes.byref(st), ctypes.byref(nxt))
    return buf[: nb * bs], st, nxt.value


def read_from_disk(blocks: bytes, block_size: int, start_offset: int, size: int):
    """block_manager.go:189-242 over an in-memory image (see oc_read_from_disk):
    returns (payload bytes or None, final offset, error code, bad block)."""
    out = ctypes.create_string_buffer(max(1, size))
    fo, bad = ctypes.c_uint64(0), ctypes.c_int64(0)
    rc = lib().oc_read_from_disk(blocks, len(blocks), block_size, start_offset, size, out,
                                 ctypes.byref(fo), ctypes.byref(bad))
    return (out.raw[:size] if rc == 0 else None), fo.value, rc, bad.value


def wal_replay(blocks: bytes, bs: int = 4096, start_block: int = 0, start_offset: int = 4, max_records: int = 0):
    """wal.go:362-455 over written blocks (see oc_wal_replay): returns
    (list of record bytes, error code, bad block, (pos_block, pos_offset))."""
    import numpy as np
    nb = len(blocks) // bs
    buf = ctypes.create_string_buffer(max(1, nb * bs))
    slots = nb * ((bs - 4) // 17 + 1) + 1
    off = np.zeros(slots, dtype=np.uint64)
    ln = np.zeros(slots, dtype=np.uint64)
    n, pb, po, bad = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_int64(0)
    rc = lib().oc_wal_replay(blocks, nb, bs, start_block, start_offset, max_records, buf,
                             off.ctypes.data, ln.ctypes.data, ctypes.byref(n), ctypes.byref(pb),
                             ctypes.byref(po), ctypes.byref(bad))
    raw = buf.raw
    recs = [raw[int(off[i]):int(off[i]) + int(ln[i])] for i in range(n.value)]
    return recs, rc, bad.value, (pb.value, po.value)



def md5(data) -> bytes:
    b = bytes(data)
    out = ctypes.create_string_buffer(16)
    lib().oc_md5(b, len(b), out)
    return out.raw


def merkle_root(leaves: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().oc_merkle_root(leaves, len(leaves) // 16, out)
    return out.raw


def merkle_serialize(leaves: bytes) -> bytes:
    n = len(leaves) // 16
    size = lib().oc_merkle_serialize(leaves, n, None)
    out = ctypes.create_string_buffer(max(1, size))
    lib().oc_merkle_serialize(leaves, n, out)
    return out.raw[:size]


def merkle_validate(leaves: bytes, stored: bytes, cap: int = 1 << 16):
    """(valid, [(tree1 hash, tree2 hash) of mismatched leaves]) or (None, []) when Go panics."""
    m1 = ctypes.create_string_buffer(16 * cap)
    m2 = ctypes.create_string_buffer(16 * cap)
    nm = ctypes.c_uint64(0)
    r = lib().oc_merkle_validate(leaves, len(leaves) // 16, stored, len(stored), m1, m2, cap, ctypes.byref(nm))
    if r < 0:
        return None, []
    k = min(nm.value, cap)
    return bool(r), [(m1.raw[16 * i:16 * i + 16], m2.raw[16 * i:16 * i + 16]) for i in range(k)]


def merkle_validate_trees(leaves1: bytes, leaves2: bytes, cap: int = 1 << 16):
    m1 = ctypes.create_string_buffer(16 * cap)
    m2 = ctypes.create_string_buffer(16 * cap)
    nm = ctypes.c_uint64(0)
    r = lib().oc_merkle_validate_trees(leaves1, len(leaves1) // 16, leaves2, len(leaves2) // 16, m1, m2, cap,
                                       ctypes.byref(nm))
    k = min(nm.value, cap)
    return bool(r), [(m1.raw[16 * i:16 * i + 16], m2.raw[16 * i:16 * i + 16]) for i in range(k)]
