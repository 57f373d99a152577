"""Python mirror of HundDB's ``utils/crc`` package over libhundcrc.so.

Same names, argument meaning and error behaviour as
/root/reference/utils/crc/crc_util.go:10-122, so the parity tests read like the
reference's own Go tests:

=========================  ==========================================  ====================
Go (crc_util.go)           here                                        C ABI (hundcrc.h)
=========================  ==========================================  ====================
BLOCK_SIZE, CRC_SIZE :11   BLOCK_SIZE, CRC_SIZE                        HC_BLOCK_SIZE/CRC_SIZE
GetCRC :15                 GetCRC(data) -> int                         hc_crc32_ieee
AddCRCToBlockData :21      AddCRCToBlockData(bytearray) -> same obj    hc_add_crc_block
AddCRCsToData :41          AddCRCsToData(data) -> bytearray            hc_add_crcs
SizeAfterAddingCRCs :69    SizeAfterAddingCRCs(n) -> int               hc_size_after_crcs
SizeWithoutCRCs :79        SizeWithoutCRCs(n) -> int                   hc_size_without_crcs
CheckBlockIntegrity :88    CheckBlockIntegrity(data) -> error|None     hc_check_block
FixLastBlockCRC :106       FixLastBlockCRC(bytearray) -> error|None    hc_fix_last_block
=========================  ==========================================  ====================

Go returns ``error`` values instead of raising, so these functions return
``None`` or a :class:`CRCError` whose ``str()`` is the exact ``errors.New``
text.  Library failures (no GPU for a batch entry, HIP errors) raise
:class:`HundCRCError`: the batched GPU path never falls back to the CPU.

The batched entries (``crc32_blocks``, ``verify_blocks``, ``stamp_blocks``,
``crc32_messages`` and their ``dev_*`` forms on torch device tensors) are the
GPU hot path.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

BLOCK_SIZE = 4096  # crc_util.go:11
CRC_SIZE = 4       # crc_util.go:12

HC_OK = 0
HC_ERR_INVALID_BLOCK = 1
HC_ERR_CRC_MISMATCH = 2
HC_ERR_TOO_SHORT = 3
HC_ERR_WAL_FRAGMENT_TYPE = 4
HC_ERR_WAL_TRUNCATED = 5
HC_E_ARG, HC_E_HIP, HC_E_NODEV, HC_E_NOMEM, HC_E_LAYOUT = -1, -2, -3, -4, -5
HC_F_STAMP = 1
HC_F_MESSAGES = 2

# HUNDCRC_LIB: load another build of the library (A/B timing of kernel variants)
_LIB_PATH = os.environ.get("HUNDCRC_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          "libhundcrc.so")


class HundCRCError(RuntimeError):
    """A library-level failure (argument, HIP, no device)."""

    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {_lib().hc_strerror(code).decode()} (code {code})")


class CRCError(Exception):
    """Mirror of the Go ``error`` values returned by utils/crc."""

    def __init__(self, code: int):
        self.code = code
        super().__init__(_lib().hc_strerror(code).decode())

    def __eq__(self, other):  # errors.New values compare by identity in Go; by text here
        return isinstance(other, CRCError) and str(other) == str(self)

    __hash__ = Exception.__hash__


class LaunchInfo(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_char_p), ("fast_blocks", ctypes.c_uint64),
                ("general_blocks", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("grid", ctypes.c_uint32), ("block_threads", ctypes.c_uint32),
                ("lds_bytes", ctypes.c_uint32)]


class Stats(ctypes.Structure):  # hc_stats_t (include/hundcrc.h)
    _fields_ = [("add_crcs_gpu", ctypes.c_uint64), ("add_crcs_host_small", ctypes.c_uint64),
                ("add_crcs_host_nodev", ctypes.c_uint64), ("add_crcs_gpu_fallback", ctypes.c_uint64),
                ("last_fallback_error", ctypes.c_int64), ("read_gpu", ctypes.c_uint64),
                ("read_gpu_fallback", ctypes.c_uint64), ("wal_gpu", ctypes.c_uint64),
                ("wal_gpu_fallback", ctypes.c_uint64), ("nodev_host", ctypes.c_uint64)]


class DevShard(ctypes.Structure):  # hc_dev_shard (include/hundcrc.h)
    _fields_ = [("device", ctypes.c_int), ("base", ctypes.c_void_p), ("off", ctypes.c_void_p),
                ("len", ctypes.c_void_p), ("stride", ctypes.c_uint64), ("ulen", ctypes.c_uint32),
                ("nblocks", ctypes.c_uint64), ("crc_out", ctypes.c_void_p), ("bad_bitmap", ctypes.c_void_p),
                ("first_bad", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


_LIB = None
_u8p = ctypes.c_void_p


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_LIB_PATH):
            raise ImportError(f"{_LIB_PATH} is missing: run `make -C hunddb_amd` or "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(_LIB_PATH)
        P, S, U32, U64, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        sig = {
            "hc_strerror": (ctypes.c_char_p, [I]),
            "hc_version": (ctypes.c_char_p, []),
            "hc_crc32_ieee": (U32, [P, S]),
            "hc_add_crc_block": (I, [P, S]),
            "hc_add_crcs_size": (S, [S]),
            "hc_add_crcs": (S, [P, S, P, S]),
            "hc_size_after_crcs": (U64, [U64]),
            "hc_size_without_crcs": (U64, [U64]),
            "hc_check_block": (I, [P, S]),
            "hc_fix_last_block": (I, [P, S]),
            "hc_crc32_blocks": (I, [P, P, P, U64, U32, U64, P]),
            "hc_verify_blocks": (I, [P, P, P, U64, U32, U64, P, P]),
            "hc_stamp_blocks": (I, [P, P, P, U64, U32, U64]),
            "hc_crc32_messages": (I, [P, P, P, U64, P]),
            "hc_shard_plan": (I, [U64, P, I, P]),
            "hc_multi_crc32_blocks": (I, [P, P, P, U64, U32, U64, P, I, P, P]),
            "hc_multi_verify_blocks": (I, [P, P, P, U64, U32, U64, P, P, I, P, P]),
            "hc_multi_stamp_blocks": (I, [P, P, P, U64, U32, U64, I, P, P]),
            "hc_dev_multi_crc32_blocks": (I, [ctypes.POINTER(DevShard), I, U32]),
            "hc_dev_crc32_blocks": (I, [I, P, P, P, U64, U32, U64, P, P, P, U32, P]),
            "hc_dev_verify_prepare": (I, [I, P, P, U64, P]),
            "hc_dev_fill_blocks": (I, [I, P, P, P, U64, U32, U64, U64, P]),
            "hc_dev_fill_range": (I, [I, P, P, P, U64, U32, U64, U64, U64, P]),
            "hc_dev_add_crcs": (I, [I, P, U64, P, P, P]),
            "hc_read_from_disk": (I, [P, U64, U32, U64, U64, P, P, P]),
            "hc_read_from_disk_v": (I, [P, U64, U32, U64, U64, P, P, P, P, P]),
            "hc_read_blocks_touched": (U64, [U32, U64, U64]),
            "hc_dev_read_blocks": (I, [I, P, U64, U32, P, P, P, P, P]),
            "hc_wal_replay": (I, [P, U64, U32, U64, U64, U64, P, U64, P, P, U64, P, P, P, P]),
            "hc_wal_replay_v": (I, [P, U64, U32, U64, U64, U64, P, U64, P, P, P, U64, P, P, P, P, P]),
            "hc_last_launch": (I, [ctypes.POINTER(LaunchInfo)]),
            "hc_debug_tables": (I, [P, S]),
            "hc_debug_seg_taken": (I, []),
            "hc_debug_seg_prof": (I, [P]),
            "hc_debug_set": (I, [ctypes.c_char_p, ctypes.c_char_p]),
            "hc_device_count": (I, []),
            "hc_host_pipelines": (I, []),
            "hc_stats": (I, [ctypes.POINTER(Stats)]),
            "hc_stats_reset": (None, []),
            "hc_md5": (None, [P, S, P]),
            "hc_md5_messages": (I, [P, P, P, U64, P]),
            "hc_dev_md5_messages": (I, [I, P, P, P, U64, U32, U64, P, P, P]),
            "hc_merkle_nodes": (U64, [U64]),
            "hc_md5_workspace_bytes": (U64, [U64]),
            "hc_merkle_levels": (I, [P, U64, P]),
            "hc_dev_merkle_levels": (I, [I, P, U64, P]),
            "hc_merkle_serialize": (I, [P, U64, P, U64, P]),
            "hc_merkle_validate": (I, [P, U64, P, U64, P, P, P, P]),
        }
        for name, (res, args) in sig.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                if os.environ.get("HUNDCRC_LIB"):  # an older A/B build: entries it lacks fail when called
                    continue
                raise
            fn.restype, fn.argtypes = res, args
        _LIB = L
    return _LIB


def lib():
    """The loaded libhundcrc.so (ctypes.CDLL)."""
    return _lib()


# ---- buffer helpers --------------------------------------------------------
def _ro_ptr(data):
    """(address, length, keepalive) of a bytes-like object without copying."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        return a.ctypes.data, a.nbytes, a
    mv = memoryview(data).cast("B")
    if mv.readonly:
        a = np.frombuffer(mv, dtype=np.uint8)
        return a.ctypes.data, a.nbytes, a
    a = np.frombuffer(mv, dtype=np.uint8)
    return a.ctypes.data, a.nbytes, a


def _rw_ptr(data):
    if isinstance(data, np.ndarray):
        if not data.flags.c_contiguous or not data.flags.writeable:
            raise ValueError("need a writable contiguous array")
        return data.ctypes.data, data.nbytes, data
    mv = memoryview(data).cast("B")
    if mv.readonly:
        raise TypeError("need a writable buffer (bytearray / numpy array)")
    a = np.frombuffer(mv, dtype=np.uint8)
    return a.ctypes.data, a.nbytes, a


def _err(code: int) -> Optional[CRCError]:
    if code == HC_OK:
        return None
    if code > 0:
        return CRCError(code)
    raise HundCRCError(code)


# ---- drop-ins (crc_util.go) --------------------------------------------------
def GetCRC(data) -> int:
    """crc_util.go:15-17 — crc32.ChecksumIEEE(data)."""
    p, n, _k = _ro_ptr(data)
    return int(_lib().hc_crc32_ieee(p if n else None, n))


def AddCRCToBlockData(data):
    """crc_util.go:21-33 — stamps data[0:4] in place and returns the same object."""
    p, n, _k = _rw_ptr(data)
    rc = _lib().hc_add_crc_block(p if n else None, n)
    if rc < 0:
        raise HundCRCError(rc, "AddCRCToBlockData")
    return data


def AddCRCsToData(serialized) -> bytearray:
    """crc_util.go:41-64 — frame into 4096-byte blocks with 4092-byte payloads."""
    p, n, _k = _ro_ptr(serialized)
    L = _lib()
    out = bytearray(L.hc_add_crcs_size(n))
    if not out:
        return out
    op, on, _ok = _rw_ptr(out)
    wrote = L.hc_add_crcs(p, n, op, on)
    if wrote == ctypes.c_size_t(-1).value:
        raise HundCRCError(-1, "AddCRCsToData")
    return out


def SizeAfterAddingCRCs(n: int) -> int:
    """crc_util.go:69-74 (float64 ceil semantics)."""
    return int(_lib().hc_size_after_crcs(n))


def SizeWithoutCRCs(n: int) -> int:
    """crc_util.go:79-83 (float64 ceil, uint64 wrap)."""
    return int(_lib().hc_size_without_crcs(n))


def CheckBlockIntegrity(block) -> Optional[CRCError]:
    """crc_util.go:88-100 — None, or CRCError("invalid block data" | "CRC mismatch in block")."""
    p, n, _k = _ro_ptr(block)
    return _err(_lib().hc_check_block(p if n else None, n))


def FixLastBlockCRC(data) -> Optional[CRCError]:
    """crc_util.go:106-122 — restamp the last complete 4096-byte block in place."""
    p, n, _k = _rw_ptr(data)
    return _err(_lib().hc_fix_last_block(p if n else None, n))


def ReadFromDisk(blocks, block_size: int, start_offset: int, size: int, verified=None):
    """lsm/block_manager/block_manager.go:189-242 minus the file I/O (row f1).

    `blocks`: the blocks from index start_offset // block_size on, as read (bytes
    past its end read as zeros).  Every touched block is verified in one batch,
    except those whose bit is set in `verified` (uint32 numpy array of
    ceil(read_blocks_touched()/32) words: the block cache's verified bits); on
    return `verified` also holds the blocks this call verified clean.
    Returns (payload, final_offset, None) or (None, 0, CRCError) like the Go
    method; `last_bad_block()` gives the failing block's relative index and
    `last_hashed()` how many blocks were hashed."""
    global _LAST_BAD, _LAST_HASHED
    p, n, _k = _ro_ptr(blocks)
    out = ctypes.create_string_buffer(max(1, size))
    fo, bad, hashed = ctypes.c_uint64(0), ctypes.c_int64(-1), ctypes.c_uint64(0)
    if verified is not None:
        k = read_blocks_touched(block_size, start_offset, size)
        if not (isinstance(verified, np.ndarray) and verified.dtype == np.uint32 and verified.size >= (k + 31) // 32):
            raise ValueError(f"verified: uint32 array of >= {(k + 31) // 32} words")
    vp = None if verified is None else verified.ctypes.data
    rc = _lib().hc_read_from_disk_v(p if n else None, n, block_size, start_offset, size, vp, out,
                                    ctypes.byref(fo), ctypes.byref(bad), ctypes.byref(hashed))
    _LAST_BAD = bad.value
    _LAST_HASHED = hashed.value
    if rc < 0:
        raise HundCRCError(rc, "ReadFromDisk")
    if rc != HC_OK:
        return None, 0, CRCError(rc)
    return out.raw[:size], fo.value, None


_LAST_BAD = -1
_LAST_HASHED = 0


def last_bad_block() -> int:
    return _LAST_BAD


def last_hashed() -> int:
    """Blocks whose CRC the last ReadFromDisk computed (masked ones excluded)."""
    return _LAST_HASHED


def read_blocks_touched(block_size: int, start_offset: int, size: int) -> int:
    """Blocks the ReadFromDisk loop touches (block_manager.go:195-235)."""
    return int(_lib().hc_read_blocks_touched(block_size, start_offset, size))


def wal_replay(blocks, block_size: int = BLOCK_SIZE, start_block: int = 0, start_offset: int = CRC_SIZE,
               max_records: int = 0, buf_cap=None, slots=None, as_arrays=False, out=None, end_blocks=False):
    """WAL recovery (lsm/wal/wal.go:362-455, row f3): verify every written block in
    one batch, then parse FULL records and reassemble fragments.

    Returns (records, err, bad_block, (pos_block, pos_offset)): `records` is a
    list of the serialized record bytes (what record.Deserialize receives),
    `err` None or CRCError.  buf_cap/slots limit the output (resumable).
    end_blocks=True (hc_wal_replay_v) appends two items: the absolute block in
    which each record completes (memtable.IsFull resumes at that + 1), and the
    (block, offset) where fragments still pending at the end start (None if
    nothing is pending or the call stopped early) -- a windowed replay's next
    start."""
    p, n, _k = _ro_ptr(blocks)
    nb = n // block_size
    cap = nb * block_size if buf_cap is None else int(buf_cap)
    if slots is None:
        slots = nb * ((block_size - CRC_SIZE) // 17 + 1)
    buf = np.empty(max(1, cap), dtype=np.uint8) if out is None else out
    cap = min(cap, buf.nbytes)
    off = np.empty(max(1, slots), dtype=np.uint64)
    ln = np.empty(max(1, slots), dtype=np.uint64)
    cnt, pb, po, bad = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_int64(-1)
    ends = np.empty(max(1, slots), dtype=np.uint64) if end_blocks else None
    pend = np.zeros(2, dtype=np.uint64)
    rc = _lib().hc_wal_replay_v(p if n else None, nb, block_size, start_block, start_offset, max_records,
                                buf.ctypes.data, cap, off.ctypes.data, ln.ctypes.data,
                                None if ends is None else ends.ctypes.data, slots,
                                ctypes.byref(cnt), ctypes.byref(pb), ctypes.byref(po), ctypes.byref(bad),
                                pend.ctypes.data)
    if rc < 0:
        raise HundCRCError(rc, "wal_replay")
    if as_arrays:  # (record bytes back to back, offsets, lengths) without per-record copies
        recs = (buf, off[:cnt.value], ln[:cnt.value])
    else:
        mv = memoryview(buf)
        recs = [bytes(mv[int(off[i]):int(off[i]) + int(ln[i])]) for i in range(cnt.value)]
    res = (recs, (None if rc == HC_OK else CRCError(rc)), bad.value, (pb.value, po.value))
    if not end_blocks:
        return res
    pending = None if int(pend[0]) == 2**64 - 1 else (int(pend[0]), int(pend[1]))
    return res + (ends[:cnt.value].copy(), pending)


# ---- batched, host-resident (GPU) ---------------------------------------------
def _meta(off, lens):
    o = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    l = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint32)
    return o, l


def _nblocks(buf_len, off, lens, stride, ulen, nblocks):
    if nblocks is not None:
        return int(nblocks)
    if off is not None:
        return len(off)
    if lens is not None:
        return len(lens)
    if stride:
        return buf_len // stride
    raise ValueError("cannot infer the block count")


def crc32_blocks(buf, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE, nblocks=None) -> np.ndarray:
    """CRC of block[4:len] for every block (what CheckBlockIntegrity computes), on the GPU."""
    p, n, _k = _ro_ptr(buf)
    o, l = _meta(off, lens)
    nb = _nblocks(n, o, l, stride, ulen, nblocks)
    out = np.zeros(nb, dtype=np.uint32)
    rc = _lib().hc_crc32_blocks(p, None if o is None else o.ctypes.data,
                                None if l is None else l.ctypes.data, stride, ulen, nb, out.ctypes.data)
    if rc != HC_OK:
        raise HundCRCError(rc, "crc32_blocks")
    return out


def verify_blocks(buf, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE, nblocks=None):
    """Batched CheckBlockIntegrity: (err | None, bad_bitmap uint32[], first_bad int)."""
    p, n, _k = _ro_ptr(buf)
    o, l = _meta(off, lens)
    nb = _nblocks(n, o, l, stride, ulen, nblocks)
    bm = np.zeros((nb + 31) // 32, dtype=np.uint32)
    fb = ctypes.c_int64(-1)
    rc = _lib().hc_verify_blocks(p, None if o is None else o.ctypes.data,
                                 None if l is None else l.ctypes.data, stride, ulen, nb,
                                 bm.ctypes.data if nb else None, ctypes.addressof(fb))
    return _err(rc), bm, fb.value


def stamp_blocks(buf, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE, nblocks=None):
    """Batched AddCRCToBlockData (in place)."""
    p, n, _k = _rw_ptr(buf)
    o, l = _meta(off, lens)
    nb = _nblocks(n, o, l, stride, ulen, nblocks)
    rc = _lib().hc_stamp_blocks(p, None if o is None else o.ctypes.data,
                                None if l is None else l.ctypes.data, stride, ulen, nb)
    if rc != HC_OK:
        raise HundCRCError(rc, "stamp_blocks")
    return buf


# ---- several GPUs in one process (include/hundcrc.h hc_shard_plan, hc_multi_*) ----
def shard_plan(nblocks: int, ndev: int, lens=None) -> np.ndarray:
    """Block-index bounds (ndev+1) of a batch split over ndev GPUs: by count, or
    balanced by bytes when `lens` is given (the plan of shard.py)."""
    l = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint32)
    b = np.zeros(ndev + 1, dtype=np.uint64)
    rc = _lib().hc_shard_plan(int(nblocks), None if l is None else l.ctypes.data, int(ndev), b.ctypes.data)
    if rc != HC_OK:
        raise HundCRCError(rc, "shard_plan")
    return b


def _devs(devices, bounds):
    d = np.ascontiguousarray(devices, dtype=np.int32)
    b = None if bounds is None else np.ascontiguousarray(bounds, dtype=np.uint64)
    if b is not None and len(b) != len(d) + 1:
        raise ValueError("bounds needs len(devices) + 1 entries")
    return d, b


def multi_crc32_blocks(buf, devices, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE, nblocks=None,
                       bounds=None) -> np.ndarray:
    """crc32_blocks with shard d of the plan on devices[d] (one host pipeline and thread per shard)."""
    p, n, _k = _ro_ptr(buf)
    o, l = _meta(off, lens)
    nb = _nblocks(n, o, l, stride, ulen, nblocks)
    d, b = _devs(devices, bounds)
    out = np.zeros(nb, dtype=np.uint32)
    rc = _lib().hc_multi_crc32_blocks(p, None if o is None else o.ctypes.data, None if l is None else l.ctypes.data,
                                      stride, ulen, nb, out.ctypes.data, len(d), d.ctypes.data,
                                      None if b is None else b.ctypes.data)
    if rc != HC_OK:
        raise HundCRCError(rc, "multi_crc32_blocks")
    return out


def multi_verify_blocks(buf, devices, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE, nblocks=None,
                        bounds=None):
    """verify_blocks over several GPUs: (err | None, bad_bitmap uint32[], first_bad int)."""
    p, n, _k = _ro_ptr(buf)
    o, l = _meta(off, lens)
    nb = _nblocks(n, o, l, stride, ulen, nblocks)
    d, b = _devs(devices, bounds)
    bm = np.zeros((nb + 31) // 32, dtype=np.uint32)
    fb = ctypes.c_int64(-1)
    rc = _lib().hc_multi_verify_blocks(p, None if o is None else o.ctypes.data, None if l is None else l.ctypes.data,
                                       stride, ulen, nb, bm.ctypes.data if nb else None, ctypes.addressof(fb),
                                       len(d), d.ctypes.data, None if b is None else b.ctypes.data)
    if rc < 0:
        raise HundCRCError(rc, "multi_verify_blocks")
    return _err(rc), bm, fb.value


def multi_stamp_blocks(buf, devices, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE, nblocks=None,
                       bounds=None):
    """stamp_blocks over several GPUs (in place)."""
    p, n, _k = _rw_ptr(buf)
    o, l = _meta(off, lens)
    nb = _nblocks(n, o, l, stride, ulen, nblocks)
    d, b = _devs(devices, bounds)
    rc = _lib().hc_multi_stamp_blocks(p, None if o is None else o.ctypes.data, None if l is None else l.ctypes.data,
                                      stride, ulen, nb, len(d), d.ctypes.data, None if b is None else b.ctypes.data)
    if rc != HC_OK:
        raise HundCRCError(rc, "multi_stamp_blocks")
    return buf


def dev_multi_crc32_blocks(shards, flags=0):
    """hc_dev_multi_crc32_blocks: `shards` = dicts with device, buf (torch tensor on
    that device), out (int32 tensor or None), stride/ulen/nblocks, off/lens
    (device tensors or None), stream (or None); enqueued, not synchronised."""
    arr = (DevShard * len(shards))()
    for k, sh in enumerate(shards):
        buf = sh["buf"]
        arr[k].device = int(sh.get("device", buf.device.index or 0))
        arr[k].base = buf.data_ptr()
        arr[k].off = _tptr(sh.get("off"))
        arr[k].len = _tptr(sh.get("lens"))
        arr[k].stride = int(sh.get("stride", 0))
        arr[k].ulen = int(sh.get("ulen", 0))
        arr[k].nblocks = int(sh["nblocks"])
        arr[k].crc_out = _tptr(sh.get("out"))
        arr[k].bad_bitmap = _tptr(sh.get("bad_bitmap"))
        arr[k].first_bad = _tptr(sh.get("first_bad"))
        st = sh.get("stream")
        if st is None:
            import torch
            st = torch.cuda.current_stream(buf.device)
        arr[k].stream = st.cuda_stream
    rc = _lib().hc_dev_multi_crc32_blocks(arr, len(shards), int(flags))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_multi_crc32_blocks")


def crc32_messages(buf, off, lens) -> np.ndarray:
    """GetCRC of every variable-length message buf[off[i]:off[i]+lens[i]], on the GPU."""
    p, n, _k = _ro_ptr(buf)
    o, l = _meta(off, lens)
    out = np.zeros(len(o), dtype=np.uint32)
    rc = _lib().hc_crc32_messages(p, o.ctypes.data, l.ctypes.data, len(o), out.ctypes.data)
    if rc != HC_OK:
        raise HundCRCError(rc, "crc32_messages")
    return out


# ---- batched, device-resident (torch tensors as device memory only) ------------
def _tptr(t):
    return None if t is None else t.data_ptr()


def _stream_ptr(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def dev_crc32_blocks(buf, crc_out=None, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE,
                     nblocks=None, bad_bitmap=None, first_bad=None, flags=0, stream=None):
    """Enqueue the CRC kernel on device tensors (uint8 buf; uint64 off; int32/uint32 lens;
    int32 crc_out / bad_bitmap; int64 first_bad).  Asynchronous on `stream`."""
    nb = _nblocks(buf.numel(), off, lens, stride, ulen, nblocks)
    dev = buf.device.index if buf.device.index is not None else 0
    rc = _lib().hc_dev_crc32_blocks(dev, buf.data_ptr(), _tptr(off), _tptr(lens), stride, ulen, nb,
                                    _tptr(crc_out), _tptr(bad_bitmap), _tptr(first_bad), flags,
                                    _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_crc32_blocks")
    return crc_out


def dev_verify_prepare(bad_bitmap, first_bad, nblocks, stream=None):
    dev = first_bad.device.index or 0
    rc = _lib().hc_dev_verify_prepare(dev, _tptr(bad_bitmap), _tptr(first_bad), nblocks, _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_verify_prepare")


def dev_fill_blocks(buf, seed, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE, nblocks=None,
                    stream=None):
    nb = _nblocks(buf.numel(), off, lens, stride, ulen, nblocks)
    dev = buf.device.index if buf.device.index is not None else 0
    rc = _lib().hc_dev_fill_blocks(dev, buf.data_ptr(), _tptr(off), _tptr(lens), stride, ulen, nb,
                                   seed & ((1 << 64) - 1), _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_fill_blocks")


def dev_fill_range(buf, seed, first_block, nblocks, off=None, lens=None, stride=BLOCK_SIZE, ulen=BLOCK_SIZE,
                   stream=None):
    """Fill a rank's shard: buffer block i = global block first_block + i of the
    seeded synthetic batch (hc_dev_fill_range)."""
    dev = buf.device.index if buf.device.index is not None else 0
    rc = _lib().hc_dev_fill_range(dev, buf.data_ptr(), _tptr(off), _tptr(lens), stride, ulen, int(first_block),
                                  int(nblocks), seed & ((1 << 64) - 1), _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_fill_range")


def dev_add_crcs(src, dst=None, crc_out=None, n=None, stream=None):
    """Fused AddCRCsToData (crc_util.go:41-64) on device tensors: frame the first
    `n` bytes of uint8 `src` (default: all) into stamped 4096-byte blocks at `dst`
    (allocated when None).  Returns dst.  Asynchronous on `stream`."""
    import torch
    n = src.numel() if n is None else int(n)
    out = hc_add_crcs_size_py(n)
    if dst is None:
        dst = torch.empty(out, dtype=torch.uint8, device=src.device)
    if dst.numel() < out:
        raise HundCRCError(HC_E_ARG, "dev_add_crcs: dst too small")
    dev = src.device.index if src.device.index is not None else 0
    rc = _lib().hc_dev_add_crcs(dev, src.data_ptr(), n, dst.data_ptr(), _tptr(crc_out), _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_add_crcs")
    return dst


def dev_read_blocks(blocks, block_size=BLOCK_SIZE, out=None, crc_out=None, bad_bitmap=None, first_bad=None,
                    nblocks=None, stream=None):
    """Batched ReadFromDisk on device tensors (k_unframe): verify every block of the
    uint8 tensor `blocks` and write the payloads back to back into `out`
    (allocated when None).  Prepare bad_bitmap/first_bad with dev_verify_prepare."""
    import torch
    nb = blocks.numel() // block_size if nblocks is None else int(nblocks)
    if out is None:
        out = torch.empty(nb * (block_size - CRC_SIZE), dtype=torch.uint8, device=blocks.device)
    if out.numel() < nb * (block_size - CRC_SIZE):
        raise HundCRCError(HC_E_ARG, "dev_read_blocks: out too small")
    dev = blocks.device.index if blocks.device.index is not None else 0
    rc = _lib().hc_dev_read_blocks(dev, blocks.data_ptr(), nb, block_size, out.data_ptr(), _tptr(crc_out),
                                   _tptr(bad_bitmap), _tptr(first_bad), _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_read_blocks")
    return out


def hc_add_crcs_size_py(n: int) -> int:
    """Output size of AddCRCsToData: ceil(n/4092) * 4096 (crc_util.go:43-46)."""
    return (n + BLOCK_SIZE - CRC_SIZE - 1) // (BLOCK_SIZE - CRC_SIZE) * BLOCK_SIZE


def last_launch() -> dict:
    info = LaunchInfo()
    _lib().hc_last_launch(ctypes.byref(info))
    return {f: (getattr(info, f).decode() if f == "kernel" and getattr(info, f) else getattr(info, f))
            for f, _ in LaunchInfo._fields_}


def device_count() -> int:
    return int(_lib().hc_device_count())


def stats() -> dict:
    """hc_stats(): the library's process-wide event counters."""
    st = Stats()
    rc = _lib().hc_stats(ctypes.byref(st))
    if rc != HC_OK:
        raise HundCRCError(rc, "hc_stats")
    return {k: int(getattr(st, k)) for k, _ in Stats._fields_}


def stats_reset() -> None:
    _lib().hc_stats_reset()


def host_pipelines() -> int:
    """Host-batch pipelines alive in this process (bounded by HC_MAX_PIPES)."""
    return int(_lib().hc_host_pipelines())


def debug_set(name: str, value=None) -> None:
    """Change one of the library's HC_* settings after it has read them from
    the environment (hc_debug_set; None restores the compiled default)."""
    v = None if value is None else str(value).encode()
    r = int(_lib().hc_debug_set(name.encode(), v))
    if r != 0:
        raise HundCRCError(r, f"debug_set({name})")


def seg_path():
    """How this thread's last device batch of whole messages was hashed:
    "packed" (the packed-record stream over records back to back), "gapped"
    (the same stream over sorted records with gaps of at most 64 B, which the
    combine hashes itself), "gapped_wide" (sorted, wider gaps, zeroed in the
    stream), "fallback_grp" (the stream's fallback for aligned 4 KiB-multiple
    records: k_crc_grp) or "fallback" (k_crc_any, or not offered to the
    stream); "sorted_packed" / "sorted_gapped" / "sorted_gapped_wide" when the
    records were listed out of order and the stream ran over their sorted view
    (from HC_SEG_SORT_MIN records, round 6).  Synchronizes the device; tests
    and tools."""
    r = int(_lib().hc_debug_seg_taken())
    if r < 0:
        raise HundCRCError(r, "seg_taken")
    return {1: "packed", 2: "gapped_wide", 3: "fallback_grp", 4: "gapped",
            9: "sorted_packed", 10: "sorted_gapped_wide", 12: "sorted_gapped"}.get(r, "fallback")


def seg_prof():
    """The stream kernel's phase clock for this thread's last stream batch, in
    microseconds from its start (hc_debug_seg_prof; tools only)."""
    buf = np.zeros(16, dtype=np.uint64)
    r = int(_lib().hc_debug_seg_prof(buf.ctypes.data))
    if r != 0:
        raise HundCRCError(r, "seg_prof")
    return [(int(x) - int(buf[0])) / 100.0 for x in buf]


def seg_mode():
    """"packed" or "gapped" (either gap width) when the packed-record stream
    took this thread's last device batch of whole messages in the batch's own
    order, "sorted_packed" / "sorted_gapped" over its sorted view, else None
    (synchronizes the device)."""
    p = seg_path()
    return {"packed": "packed", "gapped": "gapped", "gapped_wide": "gapped", "sorted_packed": "sorted_packed",
            "sorted_gapped": "sorted_gapped", "sorted_gapped_wide": "sorted_gapped"}.get(p)


def seg_taken() -> bool:
    """Whether this thread's last device batch of whole messages was hashed by
    the packed-record stream (k_seg_*, packed or gapped) rather than a
    fallback (synchronizes the device; tests and tools)."""
    return seg_mode() is not None


def debug_tables() -> np.ndarray:
    L = _lib()
    size = L.hc_debug_tables(None, 0)
    buf = np.zeros(size // 4, dtype=np.uint32)
    assert L.hc_debug_tables(buf.ctypes.data, size) == 0
    return buf
