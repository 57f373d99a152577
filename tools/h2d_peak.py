"""The host link's practical ceiling: pinned host -> device copies (hipMemcpyAsync
through torch) of a 16 GiB buffer in 64 / 256 MiB chunks on 1-3 streams, the
shapes the host pipelines use (hc_api.cpp: 64 MiB staging slots, 256 MiB span
buffers, three slots).  Not part of the product.

    python tools/h2d_peak.py [--gib 16] [--json-out f]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=16)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    total = a.gib << 30
    src = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    src.fill_(0x5A)
    dst = [torch.empty(256 << 20, dtype=torch.uint8, device="cuda") for _ in range(3)]
    res = {}
    for chunk_mib in (64, 256):
        chunk = chunk_mib << 20
        for nstreams in (1, 2, 3):
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            best = 0.0
            for _rep in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k, o in enumerate(range(0, total, chunk)):
                    s = streams[k % nstreams]
                    with torch.cuda.stream(s):
                        dst[k % 3][:chunk].copy_(src[o:o + chunk], non_blocking=True)
                torch.cuda.synchronize()
                best = max(best, total / (time.perf_counter() - t0) / 1e9)
            res[f"h2d_{chunk_mib}MiB_{nstreams}streams_GBps"] = round(best, 2)
            print(f"H2D {chunk_mib:4d} MiB chunks, {nstreams} streams: {best:6.2f} GB/s", flush=True)
    # device -> host of the same volume (the CRC words' direction, for reference)
    dsrc = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    hdst = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(total // (256 << 20)):
        hdst.copy_(dsrc, non_blocking=True)
    torch.cuda.synchronize()
    res["d2h_256MiB_GBps"] = round(total / (time.perf_counter() - t0) / 1e9, 2)
    print(f"D2H 256 MiB chunks: {res['d2h_256MiB_GBps']:.2f} GB/s")
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
