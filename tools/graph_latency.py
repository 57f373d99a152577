#!/usr/bin/env python3
"""Small batches: per-call time of the device entries called eagerly (one C-ABI
call per batch, the launches enqueued each time) against the same batch
captured once in a HIP graph (torch.cuda.CUDAGraph) and replayed.  Back-to-back
calls, timed over many iterations with HIP events on the calling stream; the
words of both forms are compared.  One JSON line per case.

  python tools/graph_latency.py [--iters 2000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    args = ap.parse_args()
    import numpy as np
    import torch

    from hunddb_amd import crc

    torch.cuda.set_device(0)
    s = torch.cuda.Stream()

    def timed(fn, iters):
        with torch.cuda.stream(s):
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(iters):
                fn()
            b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / iters  # us per call

    cases = []
    for nb in (16, 64, 256, 1024):  # WAL segments (16 blocks by default) .. components
        buf = torch.empty(nb * 4096, dtype=torch.uint8, device="cuda")
        crc.dev_fill_blocks(buf, 7, stride=4096, ulen=4096, nblocks=nb)
        out = torch.empty(nb, dtype=torch.int32, device="cuda")
        cases.append((f"{nb} x 4 KiB blocks (k_crc_grp)", nb * 4096,
                      lambda buf=buf, out=out, nb=nb: crc.dev_crc32_blocks(buf, out, stride=4096, ulen=4096,
                                                                            nblocks=nb, stream=s), out))
    for nb in (16, 256):
        n = nb * 4092 - 100
        src = torch.empty(n + 1, dtype=torch.uint8, device="cuda")[1:]
        dst = torch.empty(nb * 4096, dtype=torch.uint8, device="cuda")
        w = torch.empty(nb, dtype=torch.int32, device="cuda")
        cases.append((f"AddCRCsToData {n} B (k_frame_edges + k_frame)", n,
                      lambda src=src, dst=dst, w=w, n=n: crc.dev_add_crcs(src, dst, crc_out=w, n=n, stream=s), w))
    for nb in (16, 256):
        blk = torch.empty(nb * 4096, dtype=torch.uint8, device="cuda")
        crc.dev_fill_blocks(blk, 9, stride=4096, ulen=4096, nblocks=nb)
        pay = torch.empty(nb * 4092, dtype=torch.uint8, device="cuda")
        w = torch.empty(nb, dtype=torch.int32, device="cuda")
        cases.append((f"ReadFromDisk {nb} x 4 KiB (k_unframe)", nb * 4096,
                      lambda blk=blk, pay=pay, w=w: crc.dev_read_blocks(blk, 4096, out=pay, crc_out=w, stream=s), w))
    for line in cases:
        name, nbytes, fn, out = line
        eager = timed(fn, args.iters)
        ref = out.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            fn()
        out.zero_()
        replay = timed(g.replay, args.iters)
        same = bool(torch.equal(out, ref))
        print(json.dumps({"case": name, "bytes": nbytes, "eager_us": round(eager, 2), "graph_us": round(replay, 2),
                          "speedup": round(eager / replay, 2), "words_equal": same}), flush=True)
        assert same


if __name__ == "__main__":
    main()
