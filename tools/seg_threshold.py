"""Where the packed-record stream (k_seg_*) starts to beat k_crc_any: device
batches of n packed records (config 5's law: log-uniform 64 B - 64 KiB, at an
odd address; and equal 1 KiB records), timed per call on each path in one
process (HC_SEG_MIN_MSGS is read per call), words compared between the paths.
Prints one JSON line per (law, n).  DESIGN.md 4.2a "Routing".

  python tools/seg_threshold.py [--ns 4096,8192,...] [--calls 40]
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
    ap.add_argument("--ns", default="4096,8192,16384,32768,65536,131072,262144")
    ap.add_argument("--calls", type=int, default=40)
    ap.add_argument("--laws", default="loguniform,1k")
    args = ap.parse_args()
    import torch

    from hunddb_amd import crc as hc

    ns = [int(x) for x in args.ns.split(",")]
    rng = np.random.default_rng(5)
    nmax = max(ns)
    laws = {
        "loguniform": (64.0 * np.exp(rng.random(nmax) * np.log(1024.0))).astype(np.uint64),
        "1k": np.full(nmax, 1024, dtype=np.uint64),
    }
    total = int(max(l.sum() for l in laws.values())) + (2 << 20)
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    hc.dev_fill_range(buf, 0x77, 0, total >> 20, stride=1 << 20, ulen=1 << 20)
    for law in args.laws.split(","):
        lens_all = laws[law]
        for n in ns:
            lens = lens_all[:n]
            off = np.zeros(n, dtype=np.uint64)
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            off += np.uint64(1)
            doff = torch.from_numpy(off.view(np.int64)).cuda()
            dlen = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).cuda()
            res = {}
            for path, env in (("seg", "1"), ("any", str(1 << 40))):
                # the library reads HC_* once at first use: hc_debug_set, not os.environ
                hc.debug_set("HC_SEG_MIN_MSGS", env)
                out = torch.zeros(n, dtype=torch.int32, device="cuda")

                def call():
                    hc.dev_crc32_blocks(buf, out, nblocks=n, off=doff, lens=dlen, flags=hc.HC_F_MESSAGES)

                for _ in range(5):
                    call()
                torch.cuda.synchronize()
                kern = hc.last_launch()["kernel"]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.calls):
                    call()
                e1.record()
                torch.cuda.synchronize()
                res[path] = (e0.elapsed_time(e1) * 1e3 / args.calls, out.clone(), kern, hc.seg_taken())
            same = bool(torch.equal(res["seg"][1], res["any"][1]))
            nbytes = int(lens.sum())
            print(json.dumps({"law": law, "n": n, "bytes": nbytes, "seg_us": round(res["seg"][0], 2),
                              "any_us": round(res["any"][0], 2), "seg_taken": res["seg"][3],
                              "any_kernel": res["any"][2], "words_equal": same,
                              "seg_speedup": round(res["any"][0] / res["seg"][0], 3)}), flush=True)
            if not same:
                sys.exit(1)
    hc.debug_set("HC_SEG_MIN_MSGS", None)


if __name__ == "__main__":
    main()
