"""The CPU oracle (oracle/hc_oracle.c) against the golden fixtures.

Pins every restated form of Go's hash/crc32 (bit-serial definition, Sarwate,
slicing-by-8, amd64 CLMUL) and every utils/crc function (crc_util.go:10-122)
to the zlib-derived vectors in tests/golden/golden.json.
"""
import ctypes
import hashlib

import numpy as np
import pytest

ALGOS = ["oc_crc32_bitwise", "oc_crc32_sarwate", "oc_crc32_slicing8", "oc_crc32_go_amd64"]


def _vec_bytes(oracle, v):
    if v["hex"] is not None:
        return bytes.fromhex(v["hex"])
    seed, blk = v["seed_fill"]
    buf, _, _ = oracle.fill_blocks(seed, 0, sizes=[(v["len"] + 7) // 8 * 8])
    # fill_blocks numbers blocks from 0; regenerate block index `blk` explicitly
    n8 = (v["len"] + 7) // 8 * 8
    out = np.zeros(n8, dtype=np.uint8)
    oracle.lib().oc_fill_block(seed, blk, out.ctypes.data, n8)
    return out.tobytes()[: v["len"]]


def test_known_answers(oracle, golden):
    L = oracle.lib()
    k = golden["known"]
    assert oracle.checksum(b"123456789") == k["check_123456789"] == 0xCBF43926
    assert oracle.checksum(b"") == k["empty"] == 0
    for B, c in k["zero_payload"].items():
        assert oracle.checksum(bytes(int(B) - 4)) == c
    for v in k["vectors"]:
        b = _vec_bytes(oracle, v)
        for a in ALGOS:
            assert getattr(L, a)(0, b, len(b)) == v["crc"], (a, v["len"])


@pytest.mark.parametrize("algo", ALGOS)
def test_algorithms_agree_incremental(oracle, algo):
    """Update(crc, p) chaining (Go's crc32.Update) matches one-shot for every form."""
    L = oracle.lib()
    rng = np.random.default_rng(1)
    for n in [0, 1, 15, 16, 17, 63, 64, 65, 200, 4096, 10007]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        whole = L.oc_crc32_bitwise(0, b, n)
        cut = n // 3
        part = getattr(L, algo)(getattr(L, algo)(0, b[:cut], cut), b[cut:], n - cut)
        assert part == whole


def test_pclmul_path_used(oracle):
    # the cpu_baseline restates Go's amd64 path; it needs PCLMULQDQ on the host
    assert oracle.lib().oc_have_pclmul() in (0, 1)


def test_add_crc_to_block_data(oracle, golden):
    for c in golden["functions"]["add_crc_to_block_data"]:
        b = bytearray.fromhex(c["in"])
        a = np.frombuffer(b, dtype=np.uint8)
        oracle.lib().oc_add_crc_to_block_data(a.ctypes.data if len(b) else None, len(b))
        assert b.hex() == c["out"]


def test_check_block_integrity(oracle, golden):
    L = oracle.lib()
    for c in golden["functions"]["check_block_integrity"]:
        b = bytes.fromhex(c["in"])
        code = L.oc_check_block_integrity(b if b else None, len(b))
        got = None if code == 0 else L.oc_strerror(code).decode()
        assert got == c["err"]


def test_add_crcs_to_data(oracle, golden):
    L = oracle.lib()
    for c in golden["functions"]["add_crcs_to_data"]:
        if c["in"] is not None:
            src = bytes.fromhex(c["in"])
        else:
            seed, n = c["seed_fill"]
            n8 = (n + 7) // 8 * 8
            a = np.zeros(n8, dtype=np.uint8)
            L.oc_fill_block(seed, n, a.ctypes.data, n8)
            src = a.tobytes()[:n]
        out = np.zeros(max(c["len_out"], 1), dtype=np.uint8)
        n_out = L.oc_add_crcs_to_data(src if src else None, len(src), out.ctypes.data)
        assert n_out == c["len_out"]
        assert hashlib.sha256(out[:n_out].tobytes()).hexdigest() == c["sha256"]


def test_fix_last_block_crc(oracle, golden):
    L = oracle.lib()
    for c in golden["functions"]["fix_last_block_crc"]:
        b = bytearray.fromhex(c["in"])
        a = np.frombuffer(b, dtype=np.uint8)
        code = L.oc_fix_last_block_crc(a.ctypes.data if len(b) else None, len(b))
        assert (None if code == 0 else L.oc_strerror(code).decode()) == c["err"]
        assert hashlib.sha256(bytes(b)).hexdigest() == c["sha256"]


def test_size_helpers(oracle, golden):
    L = oracle.lib()
    for n, want in golden["functions"]["size_after_adding_crcs"]:
        assert L.oc_size_after_adding_crcs(n) == want, n
    for n, want in golden["functions"]["size_without_crcs"]:
        assert L.oc_size_without_crcs(n) == want, n


def test_config1_batch(oracle, golden):
    c = golden["config1"]
    buf, _, _ = oracle.fill_blocks(c["seed"], c["n"], c["block"])
    assert hashlib.sha256(buf.tobytes()).hexdigest() == c["sha256_inputs"]
    got = oracle.crc32_blocks(buf, stride=c["block"], ulen=c["block"])
    assert got.tolist() == c["crcs"]


def test_mixed_batch(oracle, golden):
    m = golden["mixed"]
    sizes = oracle.mixed_sizes(m["seed"], m["n"])
    assert sizes.tolist() == m["sizes"]
    buf, off, lens = oracle.fill_blocks(m["seed"], m["n"], sizes=sizes)
    assert oracle.crc32_blocks(buf, off=off, lens=lens).tolist() == m["crcs"]


def test_wal_framing(oracle, golden):
    for name, w in golden["wal"].items():
        b, st, _ = oracle.wal_frame(w["seed"], w["record_sizes"])
        blocks = [b[i:i + 4096].tobytes() for i in range(0, len(b), 4096)]
        assert [hashlib.sha256(x).hexdigest() for x in blocks] == w["sha256"], name
        assert st.refused == w["refused"], name
        # every flushed WAL block verifies (wal.go:383)
        for x in blocks:
            assert oracle.lib().oc_check_block_integrity(x, len(x)) == 0


def test_global_key_dict_header(oracle, golden):
    h = golden["global_key_dict_header"]
    blk = bytearray(4096)
    blk[4:12] = h["count"].to_bytes(8, "little")
    assert oracle.checksum(bytes(blk[4:])) == h["crc"]


def test_read_from_disk(oracle, golden):
    """oc_read_from_disk (block_manager.go:189-242) against the zlib-derived fixtures."""
    g = golden["read_from_disk"]
    for c in g["cases"]:
        B = c["block_size"]
        img = bytearray.fromhex(g["image_hex"][str(B)])
        if c["image"] == "bad3":
            img[3 * B + 1000] ^= 0x04
        start_blk = 0  # fixtures index the image from block 0
        got, fo, rc, bad = oracle.read_from_disk(bytes(img[start_blk * B:]), B, c["start"], c["size"])
        want_rc = {None: 0, "CRC mismatch in block": 2}[c["err"]]
        assert rc == want_rc, c
        if rc == 0:
            assert hashlib.sha256(got).hexdigest() == c["sha256"] and fo == c["final_offset"], c
        else:
            assert bad == c["bad_block"], c


def _replay_case_blocks(oracle, golden, c):
    if "block_hex" in c:
        return bytes.fromhex(c["block_hex"])
    w = golden["wal"][c["fixture"]]
    b, _, _ = oracle.wal_frame(w["seed"], w["record_sizes"])
    b = bytearray(b.tobytes())
    if "corrupt" in c:
        blk, off, bit = c["corrupt"]
        b[blk * 4096 + off] ^= bit
    return bytes(b)


ERRS = {None: 0, "CRC mismatch in block": 2, "unknown fragment type": 4, "truncated": 5}


def test_wal_replay(oracle, golden):
    """oc_wal_replay (wal.go:362-455) against the zlib-derived replay fixtures."""
    for name, c in golden["wal_replay"].items():
        blocks = _replay_case_blocks(oracle, golden, c)
        recs, rc, bad, pos = oracle.wal_replay(blocks, 4096, max_records=c["max_records"])
        assert rc == ERRS[c["err"]], name
        assert [len(r) for r in recs] == c["lens"], name
        assert [hashlib.sha256(r).hexdigest() for r in recs] == c["sha256"], name
        assert list(pos) == c["pos"], name
        assert bad == c["bad_block"], name
