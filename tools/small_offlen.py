"""Per-call time of small device block batches by layout: uniform (stride/ulen,
one k_crc_grp launch), the same blocks through off/len arrays (k_crc_grp +
the k_crc_any sweep), and off/len blocks the streaming kernel cannot take
(1 KiB lengths: all left to the sweep).  One JSON line per (layout, n);
words checked against the uniform call.  DESIGN.md 4.1a / 4.2.

  python tools/small_offlen.py [--ns 16,256,4096,65536] [--calls 50]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="16,256,4096,65536")
    ap.add_argument("--calls", type=int, default=50)
    args = ap.parse_args()
    import torch

    from hunddb_amd import crc as hc

    ns = [int(x) for x in args.ns.split(",")]
    B = 4096
    nmax = max(ns)
    buf = torch.empty(nmax * B, dtype=torch.uint8, device="cuda")
    hc.dev_fill_blocks(buf, 0x99, stride=B, ulen=B, nblocks=nmax)

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.calls):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.calls

    for n in ns:
        ref = torch.zeros(n, dtype=torch.int32, device="cuda")
        t_uni = timed(lambda: hc.dev_crc32_blocks(buf, ref, stride=B, ulen=B, nblocks=n))
        k_uni = hc.last_launch()["kernel"]
        off = torch.from_numpy((np.arange(n, dtype=np.uint64) * B).view(np.int64)).cuda()
        lens = torch.full((n,), B, dtype=torch.int32, device="cuda")
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        t_ol = timed(lambda: hc.dev_crc32_blocks(buf, out, off=off, lens=lens, nblocks=n))
        k_ol = hc.last_launch()["kernel"]
        same = bool(torch.equal(out, ref))
        lens1 = torch.full((n,), 1024, dtype=torch.int32, device="cuda")
        out1 = torch.zeros(n, dtype=torch.int32, device="cuda")
        t_nc = timed(lambda: hc.dev_crc32_blocks(buf, out1, off=off, lens=lens1, nblocks=n))
        k_nc = hc.last_launch()["kernel"]
        print(json.dumps({"n": n, "uniform_us": round(t_uni, 2), "uniform_kernel": k_uni, "offlen_us": round(t_ol, 2),
                          "offlen_kernel": k_ol, "offlen_words_equal": same, "nonconforming_1k_us": round(t_nc, 2),
                          "nonconforming_kernel": k_nc}), flush=True)
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
