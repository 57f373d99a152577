"""Whole-message batches of 16-B aligned 4 KiB-multiple records (k_crc_grp's
block shape) in the layouts the packed-record stream takes: which path wins,
the stream's mode or the k_crc_grp fallback.  One JSON
line per layout: GB/s (HIP events around K launches), seg_path, words against
a k_crc_any run of the same batch (HC_SEG_MIN_MSGS above n).  Run it with
HUNDCRC_LIB set to compare two builds.

  python tools/seg_aligned_probe.py [--records 1000000]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch

    from hunddb_amd import crc

    n = a.records
    rng = np.random.default_rng(7)
    four = np.full(n, 4096, np.uint32)
    mixed = rng.choice(np.array([4096, 8192, 16384], np.uint32), n // 3)
    layouts = {  # name: (lens, gap after each record)
        "packed4k": (four, 0),
        "gap16_4k": (four, 16),
        "gap1k_4k": (four, 1024),
        "packed_mixed": (mixed, 0),
        "gap16_mixed": (mixed, 16),
    }
    for name, (lens, gap) in layouts.items():
        m = len(lens)
        off = np.zeros(m, dtype=np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(gap))
        total = int(off[-1]) + int(lens[-1]) + 4096
        buf = torch.empty(total, dtype=torch.uint8, device="cuda")
        crc.dev_fill_blocks(buf, 0x5EED, stride=4096, ulen=4096, nblocks=total // 4096)
        doff = torch.from_numpy(off.view(np.int64)).cuda()
        dlen = torch.from_numpy(lens.view(np.int32)).cuda()
        out = torch.empty(m, dtype=torch.int32, device="cuda")
        ref = torch.empty(m, dtype=torch.int32, device="cuda")
        crc.debug_set("HC_SEG_MIN_MSGS", 1 << 40)
        crc.dev_crc32_blocks(buf, ref, off=doff, lens=dlen, nblocks=m, flags=crc.HC_F_MESSAGES)
        crc.debug_set("HC_SEG_MIN_MSGS", None)
        s = torch.cuda.current_stream()
        for _ in range(3):
            crc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=m, flags=crc.HC_F_MESSAGES, stream=s)
        torch.cuda.synchronize()
        path = crc.seg_path()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.steps):
            crc.dev_crc32_blocks(buf, out, off=doff, lens=dlen, nblocks=m, flags=crc.HC_F_MESSAGES, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        byts = int(lens.astype(np.uint64).sum())
        print(json.dumps({"layout": name, "records": m, "GBps": round(byts / ms / 1e6, 1), "ms": round(ms, 4),
                          "seg_path": path, "words_match": bool(torch.equal(out, ref))}), flush=True)
        del buf, doff, dlen, out, ref


if __name__ == "__main__":
    main()
