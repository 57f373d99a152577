"""VERDICT r5 item 4, route (a) priced before it is built: config 5's records
(log-uniform 64 B - 64 KiB, back to back from an odd address) listed in a
permuted order, which the packed-record stream refuses (k_crc_any's work in the
combine).  Times, with HIP events around K iterations, each on the same buffer:

  shuffled   dev_crc32_blocks on the permuted off/len (today's fallback)
  sorted     dev_crc32_blocks on the same records in offset order (the stream)
  sort_route torch.sort of the offsets (rocPRIM radix sort) + gather of the
             lengths + the stream on the sorted view + scatter of the words back
             through the permutation

and checks that every route's words agree.  One JSON line per record count.

  python tools/sort_route_probe.py [--records 2000000] [--steps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def record_sizes(n):  # bench.py's record law (configs[4]): log-uniform 64 B - 64 KiB
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(0x5B) + (i << np.uint64(21)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) / 9007199254740992.0
    return (64.0 * np.exp(u * np.log(1024.0))).astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", default="2000000")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch

    from hunddb_amd import crc

    for n in [int(x) for x in a.records.split(",")]:
        lens = record_sizes(n)
        off = np.zeros(n, dtype=np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64), dtype=np.uint64)
        off += np.uint64(1)
        total = (int(off[-1]) + int(lens[-1]) + 64 + (1 << 20) - 1) >> 20 << 20
        buf = torch.empty(total, dtype=torch.uint8, device="cuda")
        crc.dev_fill_range(buf, 0x5EED, 0, total >> 20, stride=1 << 20, ulen=1 << 20)
        perm = np.random.default_rng(7).permutation(n)
        soff = torch.from_numpy(off.view(np.int64)).cuda()
        slen = torch.from_numpy(lens.view(np.int32)).cuda()
        poff = torch.from_numpy(off[perm].view(np.int64)).cuda()
        plen = torch.from_numpy(lens[perm].view(np.int32)).cuda()
        nbytes = int(lens.sum(dtype=np.uint64)) + 4 * n
        outs = {k: torch.zeros(n, dtype=torch.int32, device="cuda") for k in ("shuffled", "sorted", "sort_route")}
        tmp = torch.zeros(n, dtype=torch.int32, device="cuda")

        def shuffled():
            crc.dev_crc32_blocks(buf, outs["shuffled"], off=poff, lens=plen, nblocks=n, flags=crc.HC_F_MESSAGES)

        def sorted_():
            crc.dev_crc32_blocks(buf, outs["sorted"], off=soff, lens=slen, nblocks=n, flags=crc.HC_F_MESSAGES)

        def sort_route():
            so, idx = torch.sort(poff)
            sl = plen[idx]
            crc.dev_crc32_blocks(buf, tmp, off=so, lens=sl, nblocks=n, flags=crc.HC_F_MESSAGES)
            outs["sort_route"][idx] = tmp

        res = {"records": n, "bytes": nbytes}
        for name, fn in (("shuffled", shuffled), ("sorted", sorted_), ("sort_route", sort_route)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            res[name + "_ms"] = round(ms, 4)
            res[name + "_frac_8tbs"] = round(nbytes / (ms * 1e-3) / 8e12, 4)
            res[name + "_path"] = crc.seg_path()
        # the sort alone (no CRC): what route (a) pays on top of the stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            so, idx = torch.sort(poff)
            sl = plen[idx]
            outs["sort_route"][idx] = tmp
        e1.record()
        torch.cuda.synchronize()
        res["sort_gather_scatter_ms"] = round(e0.elapsed_time(e1) / a.steps, 4)
        want = outs["sorted"].cpu().numpy()[perm]  # entry i of the permuted batch is sorted record perm[i]
        res["shuffled_words_equal"] = bool(np.array_equal(outs["shuffled"].cpu().numpy(), want))
        res["sort_route_words_equal"] = bool(np.array_equal(outs["sort_route"].cpu().numpy(), want))
        print(json.dumps(res), flush=True)
        if not (res["shuffled_words_equal"] and res["sort_route_words_equal"]):
            sys.exit(1)
        del buf


if __name__ == "__main__":
    main()
