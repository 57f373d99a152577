"""Row f4: the Merkle/MD5 integrity check of SSTable data, mirroring
lsm/sstable/merkle_tree/merkle_tree.go and the core of
lsm/sstable/sstable.go:2287-2420 (CheckIntegrity) over libhundcrc.so.

Names follow the Go package (NewMerkleTree, Serialize, Deserialize, Validate,
Height, MaxNumOfNodes, MaxNumOfLeafs) so the parity tests read like
merkle_tree_test.go.  A built tree is kept as the library's level arrays
(hc_merkle_levels: the leaves, each odd level's zero padding node, the parents
up to the root); a deserialized tree as its stored DFS bytes.  The record
leaves are one GPU batch (hc_md5_messages); a handful of blocks are hashed on
the host (hc_md5).
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

import numpy as np

from .crc import HC_OK, HundCRCError, _lib, _ro_ptr, _stream_ptr, _tptr

_ZERO = bytes(16)


def md5_sum(data) -> bytes:
    """md5.Sum(data) on the host CPU."""
    p, n, _k = _ro_ptr(data)
    out = ctypes.create_string_buffer(16)
    _lib().hc_md5(p if n else None, n, out)
    return out.raw


def md5_records(buf, off, lens) -> np.ndarray:
    """md5.Sum of every record buf[off[i]:off[i]+lens[i]] in one GPU batch
    (sstable.go:2358's leaves).  Returns an (n, 16) uint8 array."""
    p, _n, _k = _ro_ptr(buf)
    o = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.empty((len(o), 16), dtype=np.uint8)
    if len(o):
        rc = _lib().hc_md5_messages(p, o.ctypes.data, ln.ctypes.data, len(o), out.ctypes.data)
        if rc != HC_OK:
            raise HundCRCError(rc, "md5_records")
    return out


def dev_md5_messages(buf, out16, off=None, lens=None, stride=0, ulen=0, n=None, workspace=None, stream=None):
    """Device form (k_md5): digests of base[off(i):+len(i)] into the
    uint8 tensor out16 (n*16 bytes).  Asynchronous on `stream`."""
    if n is None:
        n = off.numel() if off is not None else buf.numel() // max(1, stride)
    dev = buf.device.index if buf.device.index is not None else 0
    rc = _lib().hc_dev_md5_messages(dev, buf.data_ptr(), _tptr(off), _tptr(lens), stride, ulen, int(n),
                                    out16.data_ptr(), _tptr(workspace), _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_md5_messages")
    return out16


def md5_workspace_bytes(n: int) -> int:
    """Device workspace of dev_md5_messages for n messages (hc_md5_workspace_bytes)."""
    return int(_lib().hc_md5_workspace_bytes(n))


def merkle_nodes(n: int) -> int:
    """Entries of the level layout for n leaves (hc_merkle_nodes)."""
    return int(_lib().hc_merkle_nodes(n))


def dev_merkle_levels(levels, n: int, stream=None):
    """Device form (k_merkle_level per level): `levels` (uint8 tensor of
    merkle_nodes(n)*16 bytes) holds the n leaves first; fills the rest."""
    dev = levels.device.index if levels.device.index is not None else 0
    rc = _lib().hc_dev_merkle_levels(dev, levels.data_ptr(), int(n), _stream_ptr(stream))
    if rc != HC_OK:
        raise HundCRCError(rc, "dev_merkle_levels")
    return levels


def _layout(n: int):
    """(start, real count) per level, leaves first -- the hc_merkle_nodes layout."""
    c, s, out = (n if n else 1), 0, []
    while True:
        out.append((s, c))
        padded = c + (c & 1) if c > 1 else c
        s += padded
        if c <= 1:
            return out
        c = padded // 2


class MerkleTree:
    """merkle_tree.MerkleTree built by NewMerkleTree (merkle_tree.go:36-81)."""

    def __init__(self, levels: np.ndarray, n: int):
        self.levels = levels.reshape(-1, 16)
        self.n = n
        self._lay = _layout(n)

    # node helpers: (L, i) with L = 0 the leaves
    def _hash(self, L, i) -> bytes:
        return self.levels[self._lay[L][0] + i].tobytes()

    def _children(self, L, i):
        if L > 0 and i < self._lay[L][1]:
            return (L - 1, 2 * i), (L - 1, 2 * i + 1)
        return None, None

    @property
    def root(self) -> bytes:
        return self._hash(len(self._lay) - 1, 0)

    def GetRootHash(self) -> bytes:
        return self.root

    def Height(self) -> int:
        """merkle_tree.go:88-96: left-child steps from the root."""
        return len(self._lay) - 1

    def MaxNumOfNodes(self) -> int:
        return 2 ** (self.Height() + 1) - 1

    def MaxNumOfLeafs(self) -> int:
        return 2 ** self.Height()

    def Serialize(self) -> bytes:
        """merkle_tree.go:173-187 (DFS pre-order), by hc_merkle_serialize."""
        nb = ctypes.c_uint64(0)
        size = merkle_nodes(self.n) * 16
        out = ctypes.create_string_buffer(size)
        rc = _lib().hc_merkle_serialize(self.levels.ctypes.data, self.n, out, size, ctypes.byref(nb))
        if rc != HC_OK:
            raise HundCRCError(rc, "Serialize")
        return out.raw[:nb.value]

    def DFS(self) -> List[bytes]:
        """Node hashes in DFS pre-order (merkle_tree.go:161-171)."""
        return [self.Serialize()[k:k + 16] for k in range(0, merkle_nodes(self.n) * 16, 16)]

    def Validate(self, other) -> Tuple[bool, List[bytes], List[bytes]]:
        """merkle_tree.go:115-147.  `other` is a built MerkleTree or the result of
        Deserialize(); returns (same, mismatched leaves of self, of other)."""
        if isinstance(other, DeserializedTree):
            valid, mb, ms, nm = ctypes.c_int(0), ctypes.create_string_buffer(16), ctypes.create_string_buffer(16), \
                ctypes.c_uint64(0)
            rc = _lib().hc_merkle_validate(self.levels.ctypes.data, self.n, other.data, len(other.data),
                                           ctypes.byref(valid), mb, ms, ctypes.byref(nm))
            if rc != HC_OK:
                raise HundCRCError(rc, "Validate")
            return bool(valid.value), [mb.raw] * nm.value, [ms.raw] * nm.value
        if self.root == other.root:
            return True, [], []
        m1: List[bytes] = []
        m2: List[bytes] = []
        stack = [((len(self._lay) - 1, 0), (len(other._lay) - 1, 0))]
        while stack:  # DeepValidate (:129-147), iteratively, left before right
            a, b = stack.pop()
            if a is None or b is None:
                continue
            ha, hb = self._hash(*a), other._hash(*b)
            if ha == hb:
                continue
            al, ar = self._children(*a)
            bl, br = other._children(*b)
            if al is None and bl is None:
                m1.append(ha)
                m2.append(hb)
            elif ha != _ZERO or hb != _ZERO:
                stack.append((ar, br))
                stack.append((al, bl))
        return False, m1, m2


class DeserializedTree:
    """merkle_tree.Deserialize(data) (:192-226): every node takes its left child
    while bytes remain, so the stored tree is a left chain of its 16-byte nodes."""

    def __init__(self, data: bytes):
        self.data = bytes(data)

    def DFS(self) -> List[bytes]:
        return [self.data[k:k + 16] for k in range(0, len(self.data), 16)]

    def Serialize(self) -> bytes:
        return self.data

    def Height(self) -> int:
        return max(0, len(self.data) // 16 - 1)


def Deserialize(data: bytes) -> DeserializedTree:
    return DeserializedTree(data)


def NewMerkleTree(blocks: Sequence, hashed_already: bool = False) -> MerkleTree:
    """merkle_tree.go:36-81.  `blocks`: str/bytes items (hashed with md5.Sum
    unless hashed_already) or, hashed, an (n, 16) uint8 array of leaves."""
    if isinstance(blocks, np.ndarray) and hashed_already:
        leaves = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 16)
    else:
        items = [b.encode() if isinstance(b, str) else bytes(b) for b in blocks]
        if hashed_already:
            leaves = np.frombuffer(b"".join((x + _ZERO)[:16] for x in items), dtype=np.uint8).reshape(-1, 16)
        elif len(items) > 256:  # one GPU batch of leaves
            lens = np.array([len(x) for x in items], dtype=np.uint32)
            off = np.zeros(len(items), dtype=np.uint64)
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            leaves = md5_records(np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8), off, lens)
        else:
            leaves = np.frombuffer(b"".join(md5_sum(x) for x in items), dtype=np.uint8).reshape(-1, 16)
    n = leaves.shape[0]
    levels = np.empty((merkle_nodes(n), 16), dtype=np.uint8)
    rc = _lib().hc_merkle_levels(np.ascontiguousarray(leaves).ctypes.data if n else None, n, levels.ctypes.data)
    if rc != HC_OK:
        raise HundCRCError(rc, "NewMerkleTree")
    return MerkleTree(levels, n)


def check_integrity(buf, off, lens, stored: bytes):
    """The data half of CheckIntegrity (sstable.go:2352-2411) over records
    buf[off[i]:off[i]+lens[i]] already read and CRC-verified: md5.Sum leaves
    (one GPU batch), the tree, Validate against Deserialize(stored).  Returns
    (valid, indices of the records whose leaf DeepValidate reports) -- Go maps
    those hashes back to block offsets through hashToOffset (:2359)."""
    leaves = md5_records(buf, off, lens) if len(off) else np.frombuffer(md5_sum(b""), np.uint8).reshape(1, 16)
    tree = NewMerkleTree(leaves, hashed_already=True)
    valid, mism, _ = tree.Validate(Deserialize(stored))
    where = {leaves[i].tobytes(): i for i in range(len(off))}  # hashToOffset: the last record with the hash
    return valid, [where[h] for h in mism if h in where]
