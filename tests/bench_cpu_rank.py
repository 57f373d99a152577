"""One rank of bench.py's N>1 flow on the CPU, for tests/test_bench_launch.py.

TEST INFRASTRUCTURE: started by bench.self_launch (the same launcher
`bench.py --gpus N` uses) with the torch.distributed.run environment.  The
per-GPU CRC kernel is replaced by the oracle (the checker), because the CPU
container has no GPU; everything around it is bench.py's: argument parsing,
the strong-scaling shard of one global batch (hunddb_amd.shard.index_range),
the global-index fill, the gloo gather of the words to rank 0, the
max-over-ranks clock, the per-rank device table (bench.py's multi_gpu proof
fields), and one JSON line printed by rank 0 with the gathered words' check
against a single-process run of the whole batch.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    from hunddb_amd import shard
    from oracle import oracle as O

    import datetime
    args = bench.parse(sys.argv[1:])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    bench.phase("init")
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=args.rank_timeout))
    bench.phase("fill")
    n, B = args.blocks, 4096
    lo, hi = shard.index_range(n, world, rank)
    counts = [shard.index_range(n, world, r)[1] - shard.index_range(n, world, r)[0] for r in range(world)]
    L = O.lib()
    buf = np.empty((hi - lo) * B, dtype=np.uint8)
    for j, i in enumerate(range(lo, hi)):  # global block index, as hc_dev_fill_range
        L.oc_fill_block(bench.SEED, i, buf.ctypes.data + j * B, B)
    bench.phase("timed")
    dist.barrier()
    t0 = time.perf_counter()
    local = O.crc32_blocks(buf, stride=B, ulen=B)
    dt = time.perf_counter() - t0
    bench.phase("gather")
    proof = shard.device_proof(shard.gather_identities(shard.rank_identity(None, dt * 1e3)), "gloo")
    dt, _, tot = shard.job_timing(dt, dt, float(buf.size))
    got = shard.gather_crcs(torch.from_numpy(local.view(np.int32)), counts)
    if rank == 0:
        full = np.empty(n * B, dtype=np.uint8)
        for i in range(n):
            L.oc_fill_block(bench.SEED, i, full.ctypes.data + i * B, B)
        want = O.crc32_blocks(full, stride=B, ulen=B)
        same = bool(np.array_equal(got.numpy().view(np.uint32), want))
        print(json.dumps({"n_gpus": world, "scaling": "strong", "blocks_total": n, "counts": counts,
                          "bytes": tot, "words_match_1proc": same, "value": tot / dt / 2**30,
                          "multi_gpu": proof}), flush=True)
    bench.phase("done")
    dist.destroy_process_group()


if __name__ == "__main__":
    import bench as _b
    _b.main = main  # bench._run's error handling around this rank's flow
    _b._run()
