"""N>1 path on CPU: world_size-2 (and 3) gloo process groups.

Each rank owns a contiguous block-index shard (hunddb_amd.shard), computes
its CRC words (here with the oracle, standing in for the per-GPU kernel),
gathers them to rank 0 and the job clock is max-reduced -- exactly the
bench.py --gpus N flow minus the device.  Rank 0 checks against the
single-process result.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, B, mixed, q):
    import torch
    import torch.distributed as dist

    from hunddb_amd import shard
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if mixed:
            sizes = O.mixed_sizes(0x4D495845, n)
            bounds = shard.byte_balanced_bounds(sizes, world)
            lo, hi = int(bounds[rank]), int(bounds[rank + 1])
            counts = [int(bounds[r + 1] - bounds[r]) for r in range(world)]
        else:
            sizes = np.full(n, B, dtype=np.uint32)
            lo, hi = shard.index_range(n, world, rank)
            counts = [shard.index_range(n, world, r)[1] - shard.index_range(n, world, r)[0] for r in range(world)]
        # the rank's resident shard: blocks lo..hi of the global batch
        buf = np.zeros(int(sizes[lo:hi].sum()), dtype=np.uint8)
        off = np.zeros(hi - lo, dtype=np.uint64)
        off[1:] = np.cumsum(sizes[lo:hi - 1], dtype=np.uint64) if hi - lo > 1 else off[1:]
        for j, i in enumerate(range(lo, hi)):
            O.lib().oc_fill_block(0x77, i, buf.ctypes.data + int(off[j]), int(sizes[i]))
        local = O.crc32_blocks(buf, off=off, lens=sizes[lo:hi])
        got = shard.gather_crcs(torch.from_numpy(local.view(np.int32)), counts)
        wall, kern, tot = shard.job_timing(0.5 + rank, 0.1 * (rank + 1), float(buf.size))
        if rank == 0:
            q.put((got.numpy().view(np.uint32).copy(), wall, kern, tot, counts))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mixed", [(2, False), (2, True), (3, True)])
def test_sharded_crcs_match_single_process(world, mixed, oracle):
    n, B = 3001, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, B, mixed, q)) for r in range(world)]
    [p.start() for p in procs]
    got, wall, kern, tot, counts = q.get(timeout=120)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    sizes = oracle.mixed_sizes(0x4D495845, n) if mixed else np.full(n, B, dtype=np.uint32)
    full = np.zeros(int(sizes.sum()), dtype=np.uint8)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    for i in range(n):
        oracle.lib().oc_fill_block(0x77, i, full.ctypes.data + int(off[i]), int(sizes[i]))
    want = oracle.crc32_blocks(full, off=off, lens=sizes)
    assert np.array_equal(got, want)
    assert wall == 0.5 + (world - 1) and abs(kern - 0.1 * world) < 1e-12
    assert tot == float(sizes.sum())
    assert sum(counts) == n


def _gather_worker(rank, world, port, n, q):
    import torch
    import torch.distributed as dist

    from hunddb_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard.index_range(n, world, rank)
        counts = [shard.index_range(n, world, r)[1] - shard.index_range(n, world, r)[0] for r in range(world)]
        # a stand-in word per global block index (the CRC kernel's output on the GPUs)
        local = _word_of(np.arange(lo, hi, dtype=np.uint64))
        got = shard.gather_crcs(torch.from_numpy(local.view(np.int32)), counts)
        wall, kern, tot = shard.job_timing(1.0 + rank, 0.5, float(hi - lo))
        ids = shard.gather_identities(shard.rank_identity(None, 0.1 * (rank + 1)))
        proof = shard.device_proof(ids, "gloo")
        if rank == 0:
            got = got.numpy().view(np.uint32)
            want = _word_of(np.arange(n, dtype=np.uint64))
            q.put((counts, bool(np.array_equal(got, want)), int(got.size), wall, tot,
                   [i["rank"] for i in proof["ranks"]], proof["comm_world_size"]))
    finally:
        dist.destroy_process_group()


def _word_of(i):
    return ((i * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(32)).astype(np.uint32)


@pytest.mark.parametrize("world", [8, 3])
def test_gather_configs3_counts(world):
    """configs[3]'s 16M blocks split by index over 8 ranks (the driver's scaling
    run) and over 3 (uneven counts): the all-gather path of shard.gather_crcs
    returns every one of the 16M words in global order, the job clock is the
    max over ranks, and the device table has one row per rank."""
    n = 16_000_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, n, q)) for r in range(world)]
    [p.start() for p in procs]
    counts, same, size, wall, tot, ranks, cws = q.get(timeout=300)
    [p.join(timeout=120) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert sum(counts) == n and size == n and same
    assert max(counts) - min(counts) <= 1 and (world != 3 or len(set(counts)) == 2)
    assert wall == float(world) and tot == float(n)
    assert ranks == list(range(world)) and cws == world


def test_byte_balance():
    from hunddb_amd import shard
    rng = np.random.default_rng(0)
    lens = (4096 << rng.integers(0, 3, 100000)).astype(np.uint32)
    for world in (2, 4, 8):
        b = shard.byte_balanced_bounds(lens, world)
        sums = [int(lens[b[r]:b[r + 1]].sum()) for r in range(world)]
        assert b[0] == 0 and b[-1] == len(lens) and sum(sums) == int(lens.sum())
        assert max(sums) - min(sums) <= 2 * 16384


def test_index_range_covers():
    from hunddb_amd import shard
    for n in (0, 1, 7, 16_000_000):
        for w in (1, 2, 3, 8):
            r = [shard.index_range(n, w, k) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n and all(r[k][1] == r[k + 1][0] for k in range(w - 1))


def _scatter_worker(rank, world, port, nbytes, q):
    import torch
    import torch.distributed as dist

    from hunddb_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bounds = [shard.index_range(nbytes, world, r)[0] for r in range(world)] + [nbytes]
        full = None
        if rank == 0:
            full = torch.from_numpy(np.random.default_rng(9).integers(0, 256, nbytes, dtype=np.uint8))
        mine = shard.scatter_from_root(full, bounds)
        got = shard.gather_crcs(torch.from_numpy(np.frombuffer(mine.numpy().tobytes() + b"\0" * (-mine.numel() % 4),
                                                                dtype=np.int32).copy()),
                                [(bounds[r + 1] - bounds[r] + 3) // 4 for r in range(world)])
        if rank == 0:
            q.put((bounds, got.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_from_root(world):
    """bench.py --input scatter: rank 0 holds the batch, every rank receives its
    byte range (gloo here, RCCL send/recv on the GPUs)."""
    nbytes = 4096 * 1001 + 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, nbytes, q)) for r in range(world)]
    [p.start() for p in procs]
    bounds, got = q.get(timeout=120)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    full = np.random.default_rng(9).integers(0, 256, nbytes, dtype=np.uint8)
    words = got.view(np.uint8)
    pos = 0
    for r in range(world):  # each rank's range came back as whole int32 words, zero-padded
        n = bounds[r + 1] - bounds[r]
        assert np.array_equal(words[pos:pos + n], full[bounds[r]:bounds[r + 1]])
        pos += (n + 3) // 4 * 4
