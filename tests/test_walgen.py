"""The config-5 WAL image generator (tools/walgen.c) reproduces the oracle's
sequential restatement of lsm/wal/wal.go:177-283 byte for byte."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("case", ["loguniform", "edges", "golden"])
def test_walgen_matches_oracle(oracle, golden, case):
    import walgen
    if case == "loguniform":
        seed = 0xC0FFEE
        plan = walgen.WalPlan(seed, nrec=3000)
        sizes = plan.sizes
        assert sizes.min() >= 64 and sizes.max() <= 65536
    elif case == "edges":
        seed = 7
        sizes = np.array([64, 4075, 4076, 4071, 100, 8150, 8151, 4075 * 3, 3958, 100, 4092 - 17, 64,
                          4076, 4076, 25 + 39, 65536, 64] * 3, dtype=np.uint32)
        plan = walgen.WalPlan(seed, sizes=sizes)
    else:
        w = golden["wal"]["mixed_small"]
        seed, sizes = w["seed"], np.array(w["record_sizes"], dtype=np.uint32)
        plan = walgen.WalPlan(seed, sizes=sizes)
    img, st, _ = oracle.wal_frame(seed, sizes)
    assert plan.nblocks == st.blocks and plan.refused == st.refused
    for threads in (1, 5):
        got = plan.render(0, plan.nblocks, threads=threads)
        assert np.array_equal(got, img)
    # any sub-range renders identically (the streaming producer renders slots)
    a = plan.nblocks // 3
    b = min(a + 7, plan.nblocks)
    assert np.array_equal(plan.render(a, b), img[a * 4096:b * 4096])


def test_walgen_sizes_match_oracle(oracle):
    import walgen
    plan = walgen.WalPlan(3, nrec=1000)
    L = oracle.lib()
    assert plan.sizes.tolist() == [L.oc_wal_record_size(3, i, 64, 65536) for i in range(1000)]
