"""Child process of tests/test_gpu_rccl.py: one rank of a "nccl" (RCCL) process
group on cuda:0.  It hashes its shard of a global batch with the HIP path,
all-gathers the words with shard.gather_crcs, runs the float64 MAX/SUM
all-reduces that shard.job_timing issues at N > 1 and the device-identity
all-gather of bench.py's multi_gpu proof, then prints one JSON line.
On a one-GPU box the group has one rank: no xGMI traffic, but every RCCL call
bench.py makes at N > 1 runs (communicator init, all_gather, all_reduce)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from hunddb_amd import crc, shard

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    nblk, B, seed = int(sys.argv[1]), 8192, 0x5EED
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    lo, hi = shard.index_range(nblk, world, rank)
    buf = torch.empty((hi - lo) * B, dtype=torch.uint8, device=dev)
    crc.dev_fill_range(buf, seed, lo, hi - lo, stride=B, ulen=B)
    out = torch.empty(hi - lo, dtype=torch.int32, device=dev)
    crc.dev_crc32_blocks(buf, out, stride=B, ulen=B, nblocks=hi - lo)
    counts = [shard.index_range(nblk, world, r)[1] - shard.index_range(nblk, world, r)[0] for r in range(world)]
    got = shard.gather_crcs(out, counts)
    t = torch.tensor([1.5 + rank, 2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    b = torch.tensor([float(hi - lo)], dtype=torch.float64, device=dev)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    # bench.py's multi_gpu proof fields over RCCL (object all-gather on the device)
    proof = shard.device_proof(shard.gather_identities(shard.rank_identity(dev, 1.25)), "nccl")
    res = {"backend": dist.get_backend(), "world": world, "kernel": crc.last_launch()["kernel"],
           "max": t.cpu().tolist(), "sum": float(b.item()), "proof": proof}
    if rank == 0:
        res["words"] = got.cpu().numpy().view(np.uint32).tolist()
        res["gathered_device"] = str(got.device)
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
