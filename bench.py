#!/usr/bin/env python3
"""Benchmark of the batched block-checksum hot path (BASELINE.json metric).

One "step" = CRC-32/IEEE of every block of one device-resident batch (what
HundDB's utils/crc CheckBlockIntegrity computes per block,
/root/reference/utils/crc/crc_util.go:88-100), through the C ABI
(hc_dev_crc32_blocks) into the hand-written gfx950 streaming kernel.

Default workload (N=1): the north star, 1M x 8 KiB blocks (8.192 GB) resident
in HBM, synthetic splitmix64 data.  With N ranks each rank owns its own 1M-block
shard (partition by block index, no data-path collective): weak scaling.
`--workload config4` runs 16M x 8 KiB split across the ranks (strong scaling).

Prints ONE JSON line (rank 0) with value = whole-job GiB/s (all ranks' bytes /
max-over-ranks wall time), the roofline of the dominant kernel (algorithmic
bytes per launch / mean HIP-event launch time vs 8 TB/s) and the CPU
baseline (the oracle's restatement of Go's crc32.ChecksumIEEE on host cores).
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
WORKLOADS = {
    # name: (blocks per rank or total, block bytes or "mixed", scaling)
    "northstar": (1_000_000, 8192, "weak"),
    "config2": (1_000_000, 4096, "weak"),
    "config3": (1_000_000, "mixed", "weak"),
    "config4": (16_000_000, 8192, "strong"),
    "16k": (500_000, 16384, "weak"),
    # f2: fused AddCRCsToData (k_frame): 1M output blocks = 4092 MB payload read
    # from an unaligned address, 4096 MB framed blocks written
    "frame": (1_000_000, "frame", "weak"),
    # f1: batched ReadFromDisk (k_unframe): verify 1M x 4 KiB blocks and strip
    # the CRC words (4096 MB read, 4092 MB payload written)
    "unframe": (1_000_000, "unframe", "weak"),
    # config2's blocks described by off/len arrays (the per-block metadata path)
    "offlen4k": (1_000_000, "offlen4k", "weak"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="northstar", choices=sorted(WORKLOADS))
    ap.add_argument("--blocks", type=int, default=0, help="override the block count")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--pmc", choices=["auto", "on", "off"], default="auto",
                    help="collect FETCH_SIZE/WRITE_SIZE in rocprofv3 child runs (N=1 only)")
    ap.add_argument("--settle", type=float, default=0.5, help="untimed clock-settle seconds before warmup")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--json-out", default="")
    return ap.parse_args()


# --------------------------------------------------------------------------
# PMC traffic via rocprofv3 child runs (started before this process touches
# the GPU; one counter group per pass as MI355X_MICROARCH.md prescribes).
def pmc_traffic(args):
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    out = {}
    # the streaming kernel: k_crc_uni (uniform 4/8/16 KiB blocks) or k_crc_fast
    kern = {"frame": "k_frame", "unframe": "k_unframe"}.get(WORKLOADS[args.workload][1], "k_crc_(uni|fast)")
    tmp = tempfile.mkdtemp(prefix="hc_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.abspath(__file__), "--child", "--steps", "3", "--warmup", "1",
             "--workload", args.workload, "--cpu-seconds", "0", "--pmc", "off"]
    if args.blocks:
        child += ["--blocks", str(args.blocks)]
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(tmp, ctr)
        cmd = [exe, "--pmc", ctr, "--kernel-include-regex", kern, "--output-format", "csv",
               "-d", d, "-o", "run", "--"] + child
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300,
                               cwd=tmp, env=dict(os.environ, TMPDIR=tmp))
        except subprocess.TimeoutExpired:
            return None, f"rocprofv3 {ctr} pass timed out"
        if r.returncode != 0:
            return None, f"rocprofv3 {ctr} pass failed rc={r.returncode}: {r.stdout[-400:].decode(errors='replace')}"
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        vals = []
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if re.search(kern, row.get("Kernel_Name", "")) and row.get("Counter_Name") == ctr:
                        vals.append(float(row["Counter_Value"]))
        if not vals:
            return None, f"no {ctr} rows"
        out[ctr] = vals
    shutil.rmtree(tmp, ignore_errors=True)
    # units: KiB; gfx950 FETCH_SIZE reports half the bytes of 16-B/lane streaming
    # reads (MI355X_MICROARCH.md "HBM") -> x2.  Skip the first (warmup) dispatch.
    f = out["FETCH_SIZE"][1:] or out["FETCH_SIZE"]
    w = out["WRITE_SIZE"][1:] or out["WRITE_SIZE"]
    fetch = 2.0 * 1024.0 * sum(f) / len(f)
    write = 1024.0 * sum(w) / len(w)
    return {"fetch_bytes": fetch, "write_bytes": write, "bytes": fetch + write,
            "raw_fetch_kib": sum(f) / len(f), "raw_write_kib": sum(w) / len(w)}, None


def mixed_sizes(seed, lo, n):
    """Config-3 block sizes: 4096 << (splitmix64(seed ^ 0x5A.., i, 2^21-1) % 3),
    the same draw as tests/golden/gen_golden.py."""
    import numpy as np
    i = np.arange(lo, lo + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed ^ 0x5A5A5A5A5A5A5A5A) + ((i << np.uint64(21)) + np.uint64((1 << 21) - 1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (np.uint32(4096) << (z % np.uint64(3)).astype(np.uint32)).astype(np.uint32)


# --------------------------------------------------------------------------
def cpu_baseline_framing(kind, dev_src, budget_s):
    """One host thread running the oracle's restatement of the reference loop
    (Go runs each AddCRCsToData / ReadFromDisk call on one goroutine) over a
    256 MB sample of the same data; bytes counted as in the GPU line (read +
    written)."""
    import ctypes
    import numpy as np
    from oracle import oracle as O
    L = O.lib()
    nblk = (256 << 20) // 4096
    if kind == "frame":  # crc_util.go:41-64
        src = dev_src[: nblk * 4092].cpu().numpy()
        dst = np.empty(nblk * 4096, dtype=np.uint8)
        run = lambda: L.oc_add_crcs_to_data(src.ctypes.data, src.size, dst.ctypes.data)  # noqa: E731
        per = src.size + dst.size
        what = f"oc_add_crcs_to_data over {src.size} B of payload (crc_util.go:41-64)"
    else:  # block_manager.go:189-242
        blocks = dev_src[: nblk * 4096].cpu().numpy()
        out = np.empty(nblk * 4092, dtype=np.uint8)
        fo, bad = ctypes.c_uint64(0), ctypes.c_int64(0)
        run = lambda: L.oc_read_from_disk(blocks.ctypes.data, blocks.size, 4096, 0, out.size,  # noqa: E731
                                          out.ctypes.data, ctypes.byref(fo), ctypes.byref(bad))
        per = blocks.size + out.size
        what = f"oc_read_from_disk over {nblk} stamped 4096-B blocks (block_manager.go:189-242)"
    run()
    t0, passes = time.perf_counter(), 0
    while True:
        run()
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(passes * per / dt / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{what}, {passes} passes in {dt:.1f} s, read+written bytes"}


def cpu_baseline(host_sample, block, threads, budget_s):
    """The oracle's restatement of Go's amd64 crc32.ChecksumIEEE (CLMUL +
    slicing-by-8) over the same blocks, on `threads` host threads."""
    from oracle import oracle as O
    n = host_sample.size // block
    O.crc32_blocks(host_sample, stride=block, ulen=block, threads=threads)  # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        O.crc32_blocks(host_sample, stride=block, ulen=block, threads=threads)
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    gib = passes * n * block / dt / 2**30
    return {"value": round(gib, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{n} x {block} B blocks copied from the GPU batch, {passes} passes in {dt:.1f} s; "
                      f"oracle/hc_oracle.c oc_crc32_go_amd64 (restates Go 1.23 hash/crc32 amd64: "
                      f"PCLMULQDQ fold + slicing-by-8), pclmul={O.lib().oc_have_pclmul()}"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        args.gpus = world

    traffic, pmc_note = None, "off"
    if not args.child and rank == 0 and world == 1 and args.pmc != "off":
        traffic, pmc_note = pmc_traffic(args)
        if traffic is None and args.pmc == "on":
            print(f"[bench] PMC collection failed: {pmc_note}", file=sys.stderr)

    import numpy as np
    import torch
    import torch.distributed as dist

    from hunddb_amd import crc, shard

    ndev = torch.cuda.device_count()
    local_dev = local % max(1, ndev)  # (rehearsal: ranks may share a GPU)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        # RCCL (backend "nccl") over xGMI; HC_DIST_BACKEND=gloo rehearses the
        # N>1 path with several ranks sharing one GPU.
        backend = os.environ.get("HC_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    nblk, bsize, scaling = WORKLOADS[args.workload]
    if args.blocks:
        nblk = args.blocks
    if scaling == "strong":  # one global batch, partitioned by block index
        lo, hi = shard.index_range(nblk, world, rank)
        my = hi - lo
    else:  # every rank owns its own full-size shard (blocks rank*n .. rank*n+n-1)
        lo, my = nblk * rank, nblk
    stream = torch.cuda.current_stream()
    seed = 0x48756E64

    if bsize == "mixed":
        sizes = mixed_sizes(seed, lo, my)
        off = np.zeros(my, dtype=np.uint64)
        off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
        total = int(off[-1]) + int(sizes[-1])
        doff = torch.from_numpy(off.view(np.int64)).to(dev)
        dlen = torch.from_numpy(sizes.view(np.int32)).to(dev)
        buf = torch.empty(total, dtype=torch.uint8, device=dev)
        crc.dev_fill_blocks(buf, seed ^ rank, off=doff, lens=dlen, nblocks=my)
        kw = dict(off=doff, lens=dlen, nblocks=my)
        step_bytes = total
        block_desc = "mixed 4/8/16 KiB"
    elif bsize == "offlen4k":
        buf = torch.empty(my * 4096, dtype=torch.uint8, device=dev)
        crc.dev_fill_blocks(buf, seed ^ rank, stride=4096, ulen=4096, nblocks=my)
        doff = torch.arange(my, dtype=torch.int64, device=dev) * 4096
        dlen = torch.full((my,), 4096, dtype=torch.int32, device=dev)
        kw = dict(off=doff, lens=dlen, nblocks=my)
        step_bytes = my * 4096
        block_desc = "4096 B via off/len arrays"
    elif bsize == "frame":
        npay = my * 4092 - 1000  # ragged last block
        raw = torch.empty(npay + 1, dtype=torch.uint8, device=dev)
        crc.dev_fill_blocks(raw, seed ^ rank, stride=npay + 1, ulen=npay + 1, nblocks=1)
        buf = raw[1:]  # payload at an odd address
        dst = torch.empty(my * 4096, dtype=torch.uint8, device=dev)
        kw = None
        step_bytes = npay + my * 4096  # one read of the payload + one write of the blocks
        block_desc = "AddCRCsToData: 4092-B payload slices -> 4096-B stamped blocks"
    elif bsize == "unframe":
        buf = torch.empty(my * 4096, dtype=torch.uint8, device=dev)
        crc.dev_fill_blocks(buf, seed ^ rank, stride=4096, ulen=4096, nblocks=my)
        crc.dev_crc32_blocks(buf, None, stride=4096, ulen=4096, nblocks=my, flags=crc.HC_F_STAMP)
        dst = torch.empty(my * 4092, dtype=torch.uint8, device=dev)
        bitmap = torch.empty((my + 31) // 32, dtype=torch.int32, device=dev)
        first_bad = torch.empty(1, dtype=torch.int64, device=dev)
        crc.dev_verify_prepare(bitmap, first_bad, my)
        kw = "unframe"
        step_bytes = my * 4096 + my * 4092  # one read of the blocks + one write of the payload
        block_desc = "ReadFromDisk: verify 4096-B blocks + strip CRCs"
    else:
        buf = torch.empty(my * bsize, dtype=torch.uint8, device=dev)
        crc.dev_fill_blocks(buf, seed ^ rank, stride=bsize, ulen=bsize, nblocks=my)
        kw = dict(stride=bsize, ulen=bsize, nblocks=my)
        step_bytes = my * bsize
        block_desc = f"{bsize} B"
    out = torch.empty(my, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def step():
        if kw is None:
            crc.dev_add_crcs(buf, dst, crc_out=out, stream=stream)
        elif kw == "unframe":
            crc.dev_read_blocks(buf, 4096, out=dst, bad_bitmap=bitmap, first_bad=first_bad, stream=stream)
        else:
            crc.dev_crc32_blocks(buf, out, stream=stream, **kw)

    # Clock settle (untimed): memory-bound launches of ~1 ms right after the fill
    # run below the sustained clock; issue launches for >= args.settle seconds
    # before the W warmup steps (MI355X_MICROARCH.md "DVFS give-back").
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    info = crc.last_launch()

    # per-launch HIP events on the launch stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    mean_kern_s = sum(kern_ms) / len(kern_ms) / 1e3

    # max-over-ranks clock, summed bytes (RCCL all-reduce of 3 scalars, after the timed region)
    dt, mean_kern_s, all_bytes = shard.job_timing(dt, mean_kern_s, float(step_bytes), device=dev)
    job_bytes = all_bytes * args.steps

    if args.child:
        if world > 1:
            dist.destroy_process_group()
        return

    if rank == 0:
        gib_s = job_bytes / dt / 2**30
        achieved = step_bytes / mean_kern_s / 1e9  # algorithmic bytes per launch / launch time
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else round(traffic["bytes"]),
                "kernel": info["kernel"], "bytes_per_launch": step_bytes,
                "mean_launch_ms": round(mean_kern_s * 1e3, 4),
                "traffic_note": (f"PMC FETCH_SIZE*2*1024 + WRITE_SIZE*1024 per launch "
                                 f"(fetch {traffic['fetch_bytes']:.4g} B, write {traffic['write_bytes']:.4g} B)"
                                 if traffic else f"null: {pmc_note}")}
        cpu = None
        if world == 1 and args.cpu_seconds > 0 and bsize in ("frame", "unframe"):
            cpu = cpu_baseline_framing(bsize, buf, args.cpu_seconds)
        elif world == 1 and args.cpu_seconds > 0 and bsize not in ("mixed", "offlen4k"):
            sample_blocks = min(my, (512 << 20) // bsize)
            host = buf[: sample_blocks * bsize].cpu().numpy()
            cpu = cpu_baseline(host, bsize, args.cpu_threads, args.cpu_seconds)
        res = {
            "metric": "GiB/s CRC32 over device-resident batched 4/8/16 KB blocks; % HBM peak",
            "value": round(gib_s, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 keyed by block index, generated in HBM)",
            "config": {"workload": args.workload, "blocks_per_gpu": my, "block_bytes": block_desc,
                       "bytes_per_gpu_step": step_bytes, "parallelism": f"shard-by-block-index x{world}",
                       "hbm_frac_of_8TBps": round(job_bytes / dt / world / 1e12 / 8.0, 4)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
