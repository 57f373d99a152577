"""The sorted view's phase clock: config 5's records back to
back, listed in a permuted order, through dev_crc32_blocks; per call the
stream kernel's workgroup-0 stamps (hc_debug_seg_prof, microseconds from the
kernel's start, each phase's END): prologue, key range + residency check, A1
coarse histograms, A2 their scan, A3 the coarse scatter, B the per-bucket unit
sort, P5 the plan of the sorted view, P6, the sorted stream body; and the words
against an in-order run.

  python tools/sort_phase_probe.py [--records 2000000] [--calls 3]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sort_route_probe import record_sizes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", default="2000000")
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    import torch

    from hunddb_amd import crc

    stamps_at = {"prologue": 1, "range_resident": 2, "A1_hist": 3, "A2_scan": 4, "A3_scatter": 5,
                 "B1_count_wg0": 8, "B2_scan_wg0": 9, "B3_scatter_wg0": 11, "B4_rank_wg0": 12, "B_buckets": 6,
                 "P5_plan": 7, "P6_mode": 10, "body_start": 14, "body_end": 15}
    for n in [int(x) for x in a.records.split(",")]:
        lens = record_sizes(n)
        off = np.zeros(n, dtype=np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64), dtype=np.uint64)
        off += np.uint64(1)
        total = (int(off[-1]) + int(lens[-1]) + 64 + (1 << 20) - 1) >> 20 << 20
        buf = torch.empty(total, dtype=torch.uint8, device="cuda")
        crc.dev_fill_range(buf, 0x5EED, 0, total >> 20, stride=1 << 20, ulen=1 << 20)
        perm = np.random.default_rng(7).permutation(n)
        ref = torch.zeros(n, dtype=torch.int32, device="cuda")
        crc.dev_crc32_blocks(buf, ref, off=torch.from_numpy(off.view(np.int64)).cuda(),
                             lens=torch.from_numpy(lens.view(np.int32)).cuda(), nblocks=n, flags=crc.HC_F_MESSAGES)
        poff = torch.from_numpy(off[perm].view(np.int64)).cuda()
        plen = torch.from_numpy(lens[perm].view(np.int32)).cuda()
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        for c in range(a.calls):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            crc.dev_crc32_blocks(buf, out, off=poff, lens=plen, nblocks=n, flags=crc.HC_F_MESSAGES)
            e1.record()
            torch.cuda.synchronize()
            path = crc.seg_path()
            prof = crc.seg_prof()
            stamps = {k: round(prof[i], 1) for k, i in stamps_at.items()}
            same = bool(torch.equal(out.cpu(), ref.cpu()[torch.from_numpy(perm)]))
            print(json.dumps({"records": n, "call": c, "dispatch_ms": round(e0.elapsed_time(e1), 4), "path": path,
                              "stamps_us": stamps, "words_equal": same}), flush=True)
            if not same:
                sys.exit(1)
        del buf


if __name__ == "__main__":
    main()
