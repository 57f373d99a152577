#!/usr/bin/env python3
"""Secondary benchmarks (DESIGN.md numbers; bench.py is the headline):

  --mode host8k   1M x 8 KiB blocks resident in HOST memory, CRC'd through
                  hc_crc32_blocks: pinned staging / direct DMA, H2D + kernel +
                  D2H of the CRC words overlapped on side streams.  The
                  PCIe-inclusive rate BASELINE.json asks for.
  --mode config5  WAL replay (BASELINE config 5): 10M records 64 B..64 KiB
                  (log-uniform), framed into 4 KiB WAL blocks exactly as
                  lsm/wal/wal.go:177-283 (tools/walgen.c), image in host memory,
                  every block verified (hc_verify_blocks = recoverMemtable's
                  CheckBlockIntegrity, wal.go:383) through the streamed pipeline.
  --mode config5b GetCRC over each variable-length record, device-resident
                  (hc_dev_crc32_blocks with HC_F_MESSAGES).
  --mode replay   row f3 end to end: the config-5 image (--records, default
                  2M) through hc_wal_replay = one GPU verify batch + parallel
                  block scan + fragment reassembly + record copy-out
                  (wal.go:362-455); rate = WAL image bytes / wall time.

--mem pinned|pageable chooses where the host image lives (pinned = as if the
segment files were read into hipHostMalloc'd buffers).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def host_array(nbytes, mem):
    import torch
    if mem == "pinned":
        t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        return t.numpy(), t
    a = np.empty(nbytes, dtype=np.uint8)
    return a, a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["host8k", "config5", "config5b", "replay", "addcrcs", "readdisk"],
                    default="host8k")
    ap.add_argument("--mem", choices=["pinned", "pageable"], default="pinned")
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--blocks", type=int, default=1_000_000)
    ap.add_argument("--bsize", type=int, default=8192, help="host8k: block bytes")
    ap.add_argument("--verify", type=int, default=0, help="host8k: hc_verify_blocks instead of hc_crc32_blocks")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--check", type=int, default=1, help="spot-check results against a CPU CRC")
    args = ap.parse_args()

    import torch
    from hunddb_amd import crc
    torch.cuda.set_device(0)
    import bench
    res = {"mode": args.mode, "mem": args.mem, "lib": os.environ.get("HUNDCRC_LIB", "in-tree"),
           "copy_threads": os.environ.get("HC_COPY_THREADS", "8 (default)")}
    thr0 = bench.cgroup_throttled_us()

    if args.mode == "host8k":
        B, n = args.bsize, args.blocks
        res.update(bsize=B, blocks=n, verify=args.verify, chunk_mb=int(os.environ.get("HC_CHUNK_MB", "64")))
        host, keep = host_array(n * B, args.mem)
        dev = torch.empty(n * B, dtype=torch.uint8, device="cuda")
        crc.dev_fill_blocks(dev, 0x48756E64, stride=B, ulen=B, nblocks=n)
        torch.cuda.synchronize()
        t = time.perf_counter()
        host[:] = dev.cpu().numpy()
        res["fill_s"] = time.perf_counter() - t
        want = torch.empty(n, dtype=torch.int32, device="cuda")
        crc.dev_crc32_blocks(dev, want, stride=B, ulen=B, nblocks=n)
        torch.cuda.synchronize()
        want = want.cpu().numpy().view(np.uint32)
        del dev
        crc.crc32_blocks(host, stride=B, ulen=B, nblocks=min(n, 1000))  # warm the pipeline
        times = []
        if args.verify:  # stamp the host copy so that every block verifies clean
            wv = want.view(np.uint8).reshape(n, 4)
            host.reshape(n, B)[:, :4] = wv
        for step_i in range(args.steps + 1):  # the first, untimed: the GPU pipeline's warm-up at full size
            t = time.perf_counter()
            if args.verify:
                err, bm, fb = crc.verify_blocks(host, stride=B, ulen=B, nblocks=n)
            else:
                got = crc.crc32_blocks(host, stride=B, ulen=B, nblocks=n)
            if step_i:
                times.append(time.perf_counter() - t)
        if args.verify:
            assert err is None and fb == -1, (err, fb)
        else:
            assert np.array_equal(got, want), "host-path CRCs differ from the device-resident path"
        bytes_ = n * B
    elif args.mode == "addcrcs":
        # AddCRCsToData (crc_util.go:41-64) over a host payload: --blocks output
        # blocks, a ragged last one; rate = payload bytes / wall time
        import ctypes
        L = crc._lib()
        n = args.blocks * 4092 - 1000
        src, keep = host_array(n + 1, args.mem)
        src = src[1:]  # odd address
        src[:] = np.arange(n, dtype=np.uint64).astype(np.uint8) ^ 0x5A
        cap = int(L.hc_add_crcs_size(n))
        dst = np.empty(cap, dtype=np.uint8)
        dst[::4096] = 1  # fault the output pages in once, outside the timed region
        sp, dp = src.ctypes.data, dst.ctypes.data
        L.hc_add_crcs(sp, 4092 * 300, dp, cap)  # warm
        times = []
        for step_i in range(args.steps + 1):  # the first, untimed: the GPU pipeline's warm-up at full size
            t = time.perf_counter()
            wrote = L.hc_add_crcs(sp, n, dp, cap)
            if step_i:
                times.append(time.perf_counter() - t)
            assert wrote == cap, wrote
        rng = np.random.default_rng(3)
        for b in list(rng.choice(cap // 4096, 300, replace=False)) + [cap // 4096 - 1]:
            blk = dst[b * 4096:(b + 1) * 4096]
            assert crc.CheckBlockIntegrity(blk) is None, b
            pay = src[b * 4092:min(n, (b + 1) * 4092)]
            assert np.array_equal(blk[4:4 + len(pay)], pay), b
        res.update(blocks=cap // 4096, payload=n)
        bytes_ = n
    elif args.mode == "readdisk":
        # ReadFromDisk (block_manager.go:189-242 minus the file I/O) over --blocks
        # stamped 4 KiB blocks from offset 4: verify every touched block, append
        # each block's payload; rate = block bytes / wall time
        import ctypes
        L = crc._lib()
        B, n = 4096, args.blocks
        host, keep = host_array(n * B, args.mem)
        dev = torch.empty(n * B, dtype=torch.uint8, device="cuda")
        crc.dev_fill_blocks(dev, 0x5EED, stride=B, ulen=B, nblocks=n)
        words = torch.empty(n, dtype=torch.int32, device="cuda")
        crc.dev_crc32_blocks(dev, words, stride=B, ulen=B, nblocks=n, flags=crc.HC_F_STAMP)
        torch.cuda.synchronize()
        host[:] = dev.cpu().numpy()
        del dev
        size = n * (B - 4) - 1000
        out = np.empty(size, dtype=np.uint8)
        out[::4096] = 0  # fault the output pages in once, outside the timed region
        fo, bad, hashed = ctypes.c_uint64(0), ctypes.c_int64(-1), ctypes.c_uint64(0)
        args_ = (host.ctypes.data, n * B, B, 4, size, None, out.ctypes.data,
                 ctypes.byref(fo), ctypes.byref(bad), ctypes.byref(hashed))
        L.hc_read_from_disk_v(host.ctypes.data, 300 * B, B, 4, 300 * (B - 4) - 10, None, out.ctypes.data,
                              ctypes.byref(fo), ctypes.byref(bad), ctypes.byref(hashed))  # warm
        times = []
        for step_i in range(args.steps + 1):  # the first, untimed: the GPU pipeline's warm-up at full size
            t = time.perf_counter()
            rc = L.hc_read_from_disk_v(*args_)
            if step_i:
                times.append(time.perf_counter() - t)
            assert rc == 0 and bad.value == -1 and hashed.value == n, (rc, bad.value, hashed.value)
        hv = host.reshape(n, B)
        for b in list(np.random.default_rng(4).choice(n - 1, 300, replace=False)) + [n - 1]:
            want = hv[b, 4:] if b < n - 1 else hv[b, 4:4 + size - (n - 1) * (B - 4)]
            assert np.array_equal(out[b * (B - 4):b * (B - 4) + len(want)], want), b
        victim = n // 3  # a corrupted block is found at its index
        host[victim * B + 100] ^= 1
        rc = L.hc_read_from_disk_v(*args_)
        host[victim * B + 100] ^= 1
        assert rc == 2 and bad.value == victim, (rc, bad.value)
        res.update(blocks=n, payload=size)
        bytes_ = n * B
    elif args.mode == "config5":
        import walgen
        t = time.perf_counter()
        plan = walgen.WalPlan(0x57414C, nrec=args.records)
        res["plan_s"] = time.perf_counter() - t
        nb = plan.nblocks
        host, keep = host_array(nb * 4096, args.mem)
        t = time.perf_counter()
        step = 1 << 18
        for b0 in range(0, nb, step):
            plan.render(b0, min(nb, b0 + step), out=host[b0 * 4096:min(nb, b0 + step) * 4096], threads=args.threads)
        res["render_s"] = time.perf_counter() - t
        res.update(records=args.records, blocks=nb, refused=plan.refused,
                   blocks_per_record=round(nb / args.records, 3), image_gib=round(nb * 4096 / 2**30, 2))
        if args.check:  # every rendered block carries a valid CRC (host CPU, sampled)
            idx = np.random.default_rng(1).choice(nb, 2000, replace=False)
            for b in idx:
                assert crc.CheckBlockIntegrity(host[b * 4096:(b + 1) * 4096]) is None
        crc.verify_blocks(host, stride=4096, ulen=4096, nblocks=min(nb, 1000))  # warm
        times = []
        for step_i in range(args.steps + 1):  # the first, untimed: the GPU pipeline's warm-up at full size
            t = time.perf_counter()
            err, bm, fb = crc.verify_blocks(host, stride=4096, ulen=4096, nblocks=nb)
            if step_i:
                times.append(time.perf_counter() - t)
            assert err is None and fb == -1, (err, fb)
        # a corrupted fragment is found (TestWAL_CorruptionDetection, asserted)
        victim = nb // 2
        host[victim * 4096 + 4 + 17 + 10] ^= 1
        err, bm, fb = crc.verify_blocks(host, stride=4096, ulen=4096, nblocks=nb)
        host[victim * 4096 + 4 + 17 + 10] ^= 1
        assert str(err) == "CRC mismatch in block" and fb == victim
        bytes_ = nb * 4096
    elif args.mode == "replay":
        import walgen
        nrec = args.records if args.records != 10_000_000 else 2_000_000
        plan = walgen.WalPlan(0x57414C, nrec=nrec)
        nb = plan.nblocks
        host, keep = host_array(nb * 4096, args.mem)
        for b0 in range(0, nb, 1 << 18):
            plan.render(b0, min(nb, b0 + (1 << 18)), out=host[b0 * 4096:min(nb, b0 + (1 << 18)) * 4096],
                        threads=args.threads)
        kept = plan.sizes[~((plan.sizes + 17 > 4092) & (plan.sizes + 17 <= 4096))]
        res.update(records=nrec, blocks=nb, refused=plan.refused, image_gib=round(nb * 4096 / 2**30, 2))
        crc.wal_replay(host[: 64 * 4096], 4096)  # warm
        rec_out = np.empty(nb * 4096, dtype=np.uint8)
        rec_out[::4096] = 0  # fault the output pages in once, outside the timed region
        times = []
        for step_i in range(args.steps + 1):  # the first, untimed: the GPU pipeline's warm-up at full size
            t = time.perf_counter()
            (rbuf, roff, rlen), err, bad, pos = crc.wal_replay(host, 4096, slots=nrec + 16, as_arrays=True,
                                                                out=rec_out)
            if step_i:
                times.append(time.perf_counter() - t)
            assert err is None and pos == (nb, 4), (err, pos)
            assert np.array_equal(rlen, kept.astype(np.uint64)), "record lengths differ from the writer's"
        bytes_ = nb * 4096
    else:  # config5b: per-record GetCRC, device-resident
        import walgen
        sizes = walgen.WalPlan(0x57414C, nrec=1).sizes  # noqa: F841 (lib init)
        sizes = np.zeros(args.records, dtype=np.uint32)
        walgen.lib().wg_record_sizes(0x57414C, args.records, 64, 65536, sizes.ctypes.data)
        off = np.zeros(args.records, dtype=np.uint64)
        off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
        total = int(off[-1]) + int(sizes[-1])
        buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        doff = torch.from_numpy(off.view(np.int64)).cuda()
        dlen = torch.from_numpy(sizes.view(np.int32)).cuda()
        crc.dev_fill_blocks(buf, 0x57414C, off=doff, lens=dlen, nblocks=args.records)
        out = torch.empty(args.records, dtype=torch.int32, device="cuda")
        kw = dict(off=doff, lens=dlen, nblocks=args.records, flags=crc.HC_F_MESSAGES)
        crc.dev_crc32_blocks(buf, out, **kw)
        torch.cuda.synchronize()
        times = []
        for step_i in range(args.steps + 1):  # the first, untimed: the GPU pipeline's warm-up at full size
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            crc.dev_crc32_blocks(buf, out, **kw)
            e.record()
            torch.cuda.synchronize()
            if step_i:
                times.append(s.elapsed_time(e) / 1e3)
        if args.check:
            got = out.cpu().numpy().view(np.uint32)
            idx = np.random.default_rng(2).choice(args.records, 2000, replace=False)
            hb = buf.cpu().numpy()
            for i in idx:
                assert got[i] == crc.GetCRC(hb[int(off[i]):int(off[i]) + int(sizes[i])])
        res.update(records=args.records, mean_record_bytes=round(total / args.records, 1))
        res["launch"] = crc.last_launch()
        bytes_ = total
    best = min(times)
    thr1 = bench.cgroup_throttled_us()
    # time the cgroup's CPU quota held the process back over the whole run
    # (fills and warm-up included): a host path with more busy threads than the
    # quota's CPUs is throttled in whole 100 ms periods
    res["cgroup_throttled_ms"] = None if thr0 is None or thr1 is None else round((thr1 - thr0) / 1e3, 1)
    res["cgroup_cpu_quota"] = bench.cgroup_cpu_quota()
    res.update(bytes=bytes_, seconds=[round(x, 4) for x in times], gib_s=round(bytes_ / best / 2**30, 2),
               gb_s=round(bytes_ / best / 1e9, 2), pcie_gen5_x16_frac=round(bytes_ / best / 63e9, 3)
               if args.mode not in ("config5b",) else None)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
