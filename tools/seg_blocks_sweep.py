"""Uniform block batches that k_crc_grp refuses: k_crc_any against the message
stream (launch_seg_blocks) per block length and alignment, same buffers, same
process, alternating routes (HC_SEG_MIN_BLOCKS through hc_debug_set).  One JSON
line per case: GB/s of each route (HIP events around K launches on the launch
stream), the words of both routes compared.  Sets HC_SEG_MIN_BLOCKS's default.

  python tools/seg_blocks_sweep.py [--gib 4] [--steps 10] [--out file.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hunddb_amd import crc  # noqa: E402

CASES = [  # (block bytes, address offset)
    (1020, 0), (2044, 0), (4092, 0), (4092, 1), (4096, 1), (6000, 0), (8188, 0), (8192, 3),
    (12000, 0), (16380, 0), (16384, 5), (65532, 0),
]


def rate(buf, out, n, B, steps, route):
    crc.debug_set("HC_SEG_MIN_BLOCKS", 1 if route == "seg" else 1 << 40)
    s = torch.cuda.current_stream()
    for _ in range(3):
        crc.dev_crc32_blocks(buf, out, stride=B, ulen=B, nblocks=n, stream=s)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(steps):
        crc.dev_crc32_blocks(buf, out, stride=B, ulen=B, nblocks=n, stream=s)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / steps
    path = crc.seg_path() if route == "seg" else "k_crc_any"
    return n * B / ms / 1e6, ms, path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    total = int(a.gib * (1 << 30))
    raw = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    crc.dev_fill_range(raw, 0x48756E64, 0, (total + 64) >> 20, stride=1 << 20, ulen=1 << 20)
    fh = open(a.out, "a") if a.out else None
    for B, lead in CASES:
        n = (total - lead) // B
        buf = raw[lead:lead + n * B]
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        res = {"block_bytes": B, "lead": lead, "n": n}
        words = {}
        for r in range(a.rounds):
            for route in (("any", "seg") if r % 2 == 0 else ("seg", "any")):
                gbs, ms, path = rate(buf, out, n, B, a.steps, route)
                res.setdefault(route + "_gbs", []).append(round(gbs, 1))
                res[route + "_path"] = path
                words[route] = out.clone()
        res["words_match"] = bool(torch.equal(words["any"], words["seg"]))
        line = json.dumps(res)
        print(line, flush=True)
        if fh:
            fh.write(line + "\n")
        del out, words
    crc.debug_set("HC_SEG_MIN_BLOCKS", None)


if __name__ == "__main__":
    main()
