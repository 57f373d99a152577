#!/usr/bin/env python3
"""Row f4 benchmarks: the Merkle/MD5 data half of
CheckIntegrity (lsm/sstable/sstable.go:2352-2411) on device-resident records.

  leaves   md5.Sum of every record (k_md5, hc_dev_md5_messages):
           --records records, serialized sizes log-uniform 64 B .. 64 KiB
           (config 5's record sizes) packed back to back, unaligned; and
           4096-B records (uniform stride).  Rate = record bytes / launch time.
  levels   NewMerkleTree(leaves, true) parents (k_merkle_level per level) over
           --leaves leaves.  Rate = leaves / s.
  host     --host-records log-uniform records in pinned HOST memory through
           hc_md5_messages (PCIe-inclusive).
  cpu      hashlib.md5 (OpenSSL) on one host core over a sample of the
           record workload.

HIP events on the launch stream; one JSON line per measurement.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def timed(torch, fn, steps, warmup):
    s = torch.cuda.current_stream()
    for _ in range(warmup):
        fn(s)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record(s)
        fn(s)
        b.record(s)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    return ms[len(ms) // 2], sum(ms) / len(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=2_000_000)
    ap.add_argument("--leaves", type=int, default=16_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--only", default="", help="run only this part: loguniform | 4096 | levels | host")
    ap.add_argument("--host-records", type=int, default=500_000)
    args = ap.parse_args()

    import torch

    from hunddb_amd import crc, merkle as M

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0x4D4435)
    if args.only in ("", "loguniform"):
        leaves_loguniform(args, torch, crc, M, dev, rng)
    if args.only in ("", "4096"):
        leaves_4096(args, torch, crc, M, dev)
    if args.only in ("", "levels"):
        levels(args, torch, crc, M, dev, rng)
    if args.only in ("", "host"):
        host_records(args, torch, M, rng)


def host_records(args, torch, M, rng):
    """CheckIntegrity from host memory: records in pinned host memory through
    hc_md5_messages (span DMA or pinned staging, H2D, k_md5, D2H of the
    digests, overlapped).  PCIe-inclusive rate = record bytes / wall time."""
    n = args.host_records
    lens = np.minimum(np.exp(rng.uniform(np.log(64), np.log(65536), n)), 65536).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(off[-1] + lens[-1])
    t = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    buf = t.numpy()
    buf[:] = rng.integers(0, 256, total, dtype=np.uint8)
    M.md5_records(buf, off[:1000], lens[:1000])  # warm the pipeline
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        out = M.md5_records(buf, off, lens)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    for i in rng.integers(0, n, 500):
        assert out[i].tobytes() == hashlib.md5(buf[int(off[i]):int(off[i]) + int(lens[i])]).digest()
    print(json.dumps({"bench": "md5_host_pinned", "records": n, "bytes": total, "best_s": round(best, 4),
                      "GBps": round(total / best / 1e9, 2)}), flush=True)


def leaves_loguniform(args, torch, crc, M, dev, rng):
    n = args.records
    lens = np.minimum(np.exp(rng.uniform(np.log(64), np.log(65536), n)), 65536).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    off += 3  # unaligned record starts
    total = (int(off[-1] + lens[-1]) + 16 + (1 << 20) - 1) >> 20 << 20
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    crc.dev_fill_blocks(buf, 0x5EED, stride=1 << 20, ulen=1 << 20, nblocks=total >> 20)
    doff = torch.from_numpy(off.view(np.int64)).to(dev)
    dlen = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.empty(M.md5_workspace_bytes(n), dtype=torch.uint8, device=dev)
    rec_bytes = int(lens.astype(np.uint64).sum())

    def leaves(s):
        M.dev_md5_messages(buf, out, off=doff, lens=dlen, n=n, workspace=ws, stream=s)

    med, mean = timed(torch, leaves, args.steps, args.warmup)
    res = {"bench": "md5_leaves_loguniform", "records": n, "bytes": rec_bytes, "median_ms": round(med, 3),
           "GBps": round(rec_bytes / med / 1e6, 1), "Mrec_s": round(n / med / 1e3, 1)}
    # spot-check against the oracle on a sample (the GPU tests check everything)
    host = buf.cpu().numpy()
    got = out.cpu().numpy().reshape(-1, 16)
    idx = rng.integers(0, n, 2000)
    for i in idx:
        assert got[i].tobytes() == hashlib.md5(host[int(off[i]):int(off[i]) + int(lens[i])].tobytes()).digest()
    # CPU: hashlib (OpenSSL MD5) on one core, and the oracle, over a sample
    t0, done, k = time.perf_counter(), 0, 0
    mv = memoryview(host)
    while time.perf_counter() - t0 < args.cpu_seconds and k < n:
        o, ln = int(off[k]), int(lens[k])
        hashlib.md5(mv[o:o + ln]).digest()
        done += ln
        k += 1
    res["cpu_hashlib_1core_GBps"] = round(done / (time.perf_counter() - t0) / 1e9, 3)
    res["cpu_sample_records"] = k
    print(json.dumps(res), flush=True)
    del buf, ws, out, doff, dlen
    torch.cuda.empty_cache()


def leaves_4096(args, torch, crc, M, dev):
    """4096-B records, uniform stride (SSTable-block-sized records)."""
    nb = 2_000_000
    b4 = torch.empty(nb * 4096, dtype=torch.uint8, device=dev)
    crc.dev_fill_blocks(b4, 7, stride=4096, ulen=4096, nblocks=nb)
    o4 = torch.empty(nb * 16, dtype=torch.uint8, device=dev)
    w4 = torch.empty(M.md5_workspace_bytes(nb), dtype=torch.uint8, device=dev)

    def uni(s):
        M.dev_md5_messages(b4, o4, stride=4096, ulen=4096, n=nb, workspace=w4, stream=s)

    med, mean = timed(torch, uni, args.steps, args.warmup)
    print(json.dumps({"bench": "md5_leaves_4096", "records": nb, "bytes": nb * 4096, "median_ms": round(med, 3),
                      "GBps": round(nb * 4096 / med / 1e6, 1)}), flush=True)
    del b4, o4, w4
    torch.cuda.empty_cache()


def levels(args, torch, crc, M, dev, rng):
    """NewMerkleTree parents over --leaves leaves."""
    nl = args.leaves
    total_nodes = M.merkle_nodes(nl)
    lv = torch.empty(total_nodes * 16, dtype=torch.uint8, device=dev)
    crc.dev_fill_blocks(lv[:nl * 16], 9, stride=16, ulen=16, nblocks=nl)

    def run(s):
        M.dev_merkle_levels(lv, nl, stream=s)

    med, mean = timed(torch, run, args.steps, args.warmup)
    # spot-check parents at every level with hashlib (the GPU tests check the
    # whole tree against the oracle)
    lay = M._layout(nl)
    host = lv.cpu().numpy().reshape(-1, 16)
    for L in range(1, len(lay)):
        s0, c = lay[L]
        c0 = lay[L - 1][0]
        for i in set(rng.integers(0, c, 50).tolist()) | {c - 1}:
            want = hashlib.md5(host[c0 + 2 * i].tobytes() + host[c0 + 2 * i + 1].tobytes()).digest()
            assert host[s0 + i].tobytes() == want, (L, i)
    print(json.dumps({"bench": "merkle_levels", "leaves": nl, "nodes": total_nodes, "median_ms": round(med, 3),
                      "Mleaves_s": round(nl / med / 1e3, 1),
                      "parent_GBps": round((total_nodes - nl) * 48 / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
