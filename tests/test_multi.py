"""Several GPUs in one process (include/hundcrc.h hc_shard_plan, hc_multi_*,
SURVEY.md 8b "multi-GPU variants take a shard plan", 8e): the C-ABI plan equals
hunddb_amd/shard.py's, arguments are checked, and without a gfx950 the multi
entries fail like the one-GPU batches (no CPU fallback).  GPU parity:
tests/test_gpu_multi.py."""
import numpy as np
import pytest

from hunddb_amd import shard


@pytest.mark.parametrize("ndev", [1, 2, 3, 4, 7, 8])
def test_shard_plan_by_count_equals_shard_py(hc, ndev):
    for n in [0, 1, ndev - 1, ndev, 1000, 16_000_000, 2**40 + 3]:
        b = hc.shard_plan(n, ndev)
        want = [shard.index_range(n, ndev, r)[0] for r in range(ndev)] + [n]
        assert b.tolist() == want, (n, ndev)


@pytest.mark.parametrize("ndev", [1, 2, 3, 4, 8])
def test_shard_plan_by_bytes_equals_shard_py(hc, ndev):
    rng = np.random.default_rng(ndev)
    cases = [rng.choice([4096, 8192, 16384], 5000).astype(np.uint32),   # configs[2]
             rng.integers(0, 65536, 3001).astype(np.uint32),            # record sizes, zero-length ones
             np.array([1 << 31, 1, 1, 1 << 31, 5], dtype=np.uint32),    # a few huge blocks
             np.zeros(10, dtype=np.uint32), np.array([7], dtype=np.uint32)]
    for lens in cases:
        got = hc.shard_plan(len(lens), ndev, lens)
        want = shard.byte_balanced_bounds(lens, ndev)
        assert got.tolist() == want.tolist(), (lens[:8], ndev)
        assert got[0] == 0 and got[-1] == len(lens) and (np.diff(got.astype(np.int64)) >= 0).all()


def test_shard_plan_rejects_bad_arguments(hc):
    L = hc.lib()
    b = np.zeros(3, dtype=np.uint64)
    assert L.hc_shard_plan(10, None, 0, b.ctypes.data) == hc.HC_E_ARG
    assert L.hc_shard_plan(10, None, 2, None) == hc.HC_E_ARG
    assert L.hc_shard_plan(10, None, 65, b.ctypes.data) == hc.HC_E_ARG


def test_multi_entries_check_the_plan(hc):
    """A plan that does not cover [0, n) in order is refused before any device work."""
    L = hc.lib()
    buf = np.zeros(4096 * 10, dtype=np.uint8)
    out = np.zeros(10, dtype=np.uint32)
    devs = np.zeros(2, dtype=np.int32)
    for bad in ([0, 5, 9], [1, 5, 10], [0, 6, 5]):
        b = np.array(bad, dtype=np.uint64)
        rc = L.hc_multi_crc32_blocks(buf.ctypes.data, None, None, 4096, 4096, 10, out.ctypes.data, 2,
                                     devs.ctypes.data, b.ctypes.data)
        assert rc == hc.HC_E_ARG, bad
    assert L.hc_multi_crc32_blocks(buf.ctypes.data, None, None, 4096, 4096, 10, out.ctypes.data, 0,
                                   devs.ctypes.data, None) == hc.HC_E_ARG
    assert L.hc_multi_crc32_blocks(buf.ctypes.data, None, None, 4096, 4096, 10, out.ctypes.data, 2,
                                   None, None) == hc.HC_E_ARG
    assert L.hc_dev_multi_crc32_blocks(None, 1, 0) == hc.HC_E_ARG
    assert L.hc_dev_multi_crc32_blocks(None, 0, 0) == hc.HC_OK


def test_multi_entries_fail_loudly_without_gpu(hc):
    if hc.device_count() > 0:
        pytest.skip("a gfx950 device is present")
    buf = np.zeros(4096 * 8, dtype=np.uint8)
    for fn in (hc.multi_crc32_blocks, hc.multi_stamp_blocks):
        with pytest.raises(hc.HundCRCError) as ei:
            fn(buf, [0, 0])
        assert ei.value.code == hc.HC_E_NODEV
    with pytest.raises(hc.HundCRCError) as ei:
        hc.multi_verify_blocks(buf, [0])
    assert ei.value.code == hc.HC_E_NODEV
