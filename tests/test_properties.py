"""Property tests (CPU): the product's host paths in libhundcrc against the
oracle's restatement of utils/crc/crc_util.go:10-122 and
block_manager.go:189-242, on inputs drawn by hypothesis -- lengths, offsets,
block sizes, truncations, corruptions and verified masks the fixed fixtures do
not enumerate.  Batches stay under the 256-block GPU threshold, so every call
here runs the product's host code (hc_cpu.cpp), never a GPU; the GPU side of
the same entries is tests/test_gpu_parity.py.
"""
import ctypes
import zlib

import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

SETTINGS = settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@SETTINGS
@given(data=st.binary(max_size=20000), shift=st.integers(0, 15))
def test_getcrc_matches_zlib_and_oracle(hc, oracle, data, shift):
    """GetCRC (crc_util.go:15-17) = ChecksumIEEE at any length and alignment."""
    buf = bytearray(shift) + bytearray(data)
    view = memoryview(buf)[shift:]
    want = zlib.crc32(data)
    assert hc.GetCRC(view) == want == oracle.checksum(data)


@SETTINGS
@given(data=st.binary(max_size=9000), flip=st.integers(0, 2**31))
def test_stamp_then_check_detects_every_single_bit_flip(hc, oracle, data, flip):
    """AddCRCToBlockData (:21-33) stamps exactly what the oracle stamps;
    CheckBlockIntegrity (:88-100) accepts the stamped block and rejects it
    after any single-bit flip (CRC-32 detects every 1-bit error)."""
    b = bytearray(data)
    ref = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(bytes(b) + b"\0")
    hc.AddCRCToBlockData(b)
    oracle.lib().oc_add_crc_to_block_data(ref, len(b))
    assert bytes(b) == bytes(ref)[:len(b)]
    err = hc.CheckBlockIntegrity(bytes(b))
    if len(b) < 4:
        assert str(err) == "invalid block data"
        return
    assert err is None
    bit = flip % (8 * len(b))
    b[bit // 8] ^= 1 << (bit % 8)
    assert str(hc.CheckBlockIntegrity(bytes(b))) == "CRC mismatch in block"


@SETTINGS
@given(data=st.binary(max_size=4092 * 40 + 17))
def test_add_crcs_to_data_host_matches_oracle(hc, oracle, data):
    """AddCRCsToData (:41-64) below the GPU threshold: byte-exact framing."""
    got = hc.AddCRCsToData(data)
    want = np.zeros(int(hc.lib().hc_add_crcs_size(len(data))), dtype=np.uint8)
    m = oracle.lib().oc_add_crcs_to_data(data, len(data), want.ctypes.data)
    assert m == len(got) and bytes(got) == want.tobytes()


@SETTINGS
@given(data=st.binary(max_size=3 * 4096 + 100))
def test_fix_last_block_crc_matches_oracle(hc, oracle, data):
    """FixLastBlockCRC (:106-122): same error and the same bytes."""
    b = bytearray(data)
    ref = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(bytes(b) + b"\0")
    err = hc.FixLastBlockCRC(b)
    rc = oracle.lib().oc_fix_last_block_crc(ref, len(b))
    assert (0 if err is None else err.code) == rc
    assert bytes(b) == bytes(ref)[:len(b)]


@SETTINGS
@given(n=st.one_of(st.integers(0, 1 << 20), st.integers(0, 2**64 - 1),
                   st.integers(2**64 - 70000, 2**64 - 1)))
def test_size_helpers_match_oracle(hc, oracle, n):
    """SizeAfterAddingCRCs / SizeWithoutCRCs (:69-83): float64 ceil, uint64 wrap."""
    L = oracle.lib()
    assert hc.SizeAfterAddingCRCs(n) == L.oc_size_after_adding_crcs(n)
    assert hc.SizeWithoutCRCs(n) == L.oc_size_without_crcs(n)


def _image(oracle, seed, nblocks, B):
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 256, nblocks * B, dtype=np.uint8)
    crcs = oracle.crc32_blocks(raw, stride=B, ulen=B)
    for i in range(nblocks):
        raw[i * B:i * B + 4] = np.frombuffer(np.uint32(crcs[i]).tobytes(), dtype=np.uint8)
    return raw


@SETTINGS
@given(B=st.sampled_from([1024, 2048, 4096, 5000, 8192]), nblocks=st.integers(1, 24), seed=st.integers(0, 2**32),
       start_frac=st.floats(0, 1), size_frac=st.floats(0, 1.2), corrupt=st.one_of(st.none(), st.integers(0, 2**31)),
       cut=st.one_of(st.none(), st.integers(1, 3 * 8192)))
def test_read_from_disk_host_matches_oracle(hc, oracle, B, nblocks, seed, start_frac, size_frac, corrupt, cut):
    """ReadFromDisk (block_manager.go:189-242) on the host path: any block size,
    start offset (inside the CRC field too), size (past the image too), a
    truncated image (zero-extended short reads) and a corrupted byte."""
    img = _image(oracle, seed, nblocks, B)
    start = int(start_frac * (nblocks * B - 1))
    view = bytearray(img[(start // B) * B:].tobytes())
    size = int(size_frac * len(view))
    if corrupt is not None:
        view[corrupt % len(view)] ^= 0x20
    if cut is not None and cut < len(view):
        view = view[:len(view) - cut]
    got, fo, err = hc.ReadFromDisk(bytes(view), B, start, size)
    want, wfo, wrc, wbad = oracle.read_from_disk(bytes(view), B, start, size)
    assert (0 if err is None else err.code) == wrc
    if wrc == 0:
        assert got == want and fo == wfo
    else:
        assert hc.last_bad_block() == wbad


@SETTINGS
@given(B=st.sampled_from([1024, 4096, 8192]), nblocks=st.integers(1, 24), seed=st.integers(0, 2**32),
       mask_seed=st.integers(0, 2**32), start_frac=st.floats(0, 1))
def test_read_from_disk_verified_mask_properties(hc, oracle, B, nblocks, seed, mask_seed, start_frac):
    """The block cache's verified bits (hc_read_from_disk_v): masked blocks are
    not hashed, every touched block ends up marked, and the data is the
    oracle's."""
    img = _image(oracle, seed, nblocks, B)
    start = int(start_frac * (nblocks * B - 1))
    view = img[(start // B) * B:].tobytes()
    # exactly the view's payload: the first block from max(start % B, 4), the rest from 4
    size = (B - max(start % B, 4)) + (len(view) // B - 1) * (B - 4)
    k = hc.read_blocks_touched(B, start, size)
    assert k == len(view) // B
    words = (k + 31) // 32
    rng = np.random.default_rng(mask_seed)
    bits = rng.integers(0, 2, k).astype(bool)
    mask = np.zeros(words, dtype=np.uint32)
    for i in np.nonzero(bits)[0]:
        mask[i >> 5] |= np.uint32(1 << (int(i) & 31))
    got, fo, err = hc.ReadFromDisk(view, B, start, size, verified=mask)
    want, wfo, wrc, _ = oracle.read_from_disk(view, B, start, size)
    assert err is None and wrc == 0 and got == want and fo == wfo
    assert hc.last_hashed() == int((~bits).sum())
    marked = np.unpackbits(mask.view(np.uint8), bitorder="little")[:k]
    assert marked.all()
