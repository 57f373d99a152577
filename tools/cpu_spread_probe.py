"""where the CPU baseline's slice spread comes from.  The
oracle's Go amd64 restatement (bench.py's cpu_baseline port) on 16 pinned
threads over 8 KiB blocks, timed in slices of ~1 s, every call 512 MiB of
blocks whose offsets cycle over a region of R MiB: R = 512 streams from DRAM
(bench.py's north-star sample), a few MiB stays cache-resident (the reference
CRCs each block right after reading it into a fresh buffer:
block_manager.go:203-235, wal.go:261).  Regions interleaved slice by slice, so
a burst of another tenant on the shared host lands on every region alike.  One
JSON line per region: median GiB/s, the min/max spread of its slices, and per
slice the share of threads x wall time the process was on a CPU (busy).

  python tools/cpu_spread_probe.py [--sizes-mib 512,16,4] [--slices 11] [--slice-s 1.0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mib", default="512,16,4")
    ap.add_argument("--slices", type=int, default=11)
    ap.add_argument("--slice-s", type=float, default=1.0)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import bench
    from oracle import oracle as O

    sizes = [int(x) for x in a.sizes_mib.split(",")]
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, max(sizes) << 20, dtype=np.uint8)
    runs = {}
    n = (512 << 20) // 8192
    for s in sizes:
        off = (np.arange(n, dtype=np.uint64) % np.uint64((s << 20) // 8192)) * np.uint64(8192)
        lens = np.full(n, 8192, np.uint32)
        runs[s] = (off, lens, int(lens.sum(dtype=np.uint64)))
    res = {s: [] for s in sizes}
    busy = {s: [] for s in sizes}  # process CPU time / (wall x threads) per slice
    with bench.pinned(a.threads) as pin:
        for s in sizes:  # warm every size once
            off, lens, nb = runs[s]
            bench._rate(lambda: O.crc32_blocks(data, off=off, lens=lens, threads=a.threads), nb, a.slice_s)
        for _ in range(a.slices):
            for s in sizes:
                off, lens, nb = runs[s]
                c0, w0 = time.process_time(), time.perf_counter()
                r = bench._rate(lambda: O.crc32_blocks(data, off=off, lens=lens, threads=a.threads), nb, a.slice_s)
                res[s].append(r)
                busy[s].append((time.process_time() - c0) / (time.perf_counter() - w0) / a.threads)
                time.sleep(0.1)
        info = pin.info()
    for s in sizes:
        v = np.array(res[s])
        med = float(np.median(v))
        print(json.dumps({"region_mib": s, "call_mib": 512, "threads": a.threads, "median_gib_s": round(med, 2),
                          "spread_pct": [round(100 * (v.min() / med - 1), 1), round(100 * (v.max() / med - 1), 1)],
                          "slices": [round(float(x), 1) for x in v],
                          "busy": [round(x, 3) for x in busy[s]], "pinned_cpus": info["pinned_cpus"]}), flush=True)


if __name__ == "__main__":
    main()
