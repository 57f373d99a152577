"""Where k_md5 loses on log-uniform records against 4096-B ones: the same
kernel over 2M records of several shapes (off/len arrays throughout), one JSON
line each with GB/s and compressions per second.

  python tools/md5_probe.py [--records 2000000]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=2_000_000)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    import torch

    from hunddb_amd import crc, merkle as M

    n = a.records
    rng = np.random.default_rng(0x4D4435)
    logu = np.minimum(np.exp(rng.uniform(np.log(64), np.log(65536), n)), 65536).astype(np.uint32)
    shapes = {
        "loguniform_unaligned": (logu, 3),
        "loguniform_aligned_start": (logu, 0),
        "loguniform_len64": (((logu + 63) // 64 * 64).astype(np.uint32), 0),
        "loguniform_len64_minus9": (((logu + 63) // 64 * 64 - 9).astype(np.uint32), 0),
        "4096_offlen": (np.full(n, 4096, np.uint32), 0),
        "4096_offlen_unaligned": (np.full(n, 4096, np.uint32), 3),
        "4096_shuffled_lens": (np.where(rng.random(n) < 0.5, 2048, 6144).astype(np.uint32), 0),
    }
    for name, (lens, pad) in shapes.items():
        off = np.zeros(n, dtype=np.uint64)
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        off += np.uint64(pad)
        total = (int(off[-1] + lens[-1]) + 16 + (1 << 20) - 1) >> 20 << 20
        buf = torch.empty(total, dtype=torch.uint8, device="cuda")
        crc.dev_fill_blocks(buf, 0x5EED, stride=1 << 20, ulen=1 << 20, nblocks=total >> 20)
        doff = torch.from_numpy(off.view(np.int64)).cuda()
        dlen = torch.from_numpy(lens.view(np.int32)).cuda()
        out = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        ws = torch.empty(max(16, M.md5_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream()
        for _ in range(2):
            M.dev_md5_messages(buf, out, off=doff, lens=dlen, n=n, workspace=ws, stream=s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.steps):
            M.dev_md5_messages(buf, out, off=doff, lens=dlen, n=n, workspace=ws, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        byts = int(lens.astype(np.uint64).sum())
        comp = int((lens.astype(np.uint64) // 64 + np.where(lens % 64 < 56, 1, 2)).sum())
        print(json.dumps({"shape": name, "ms": round(ms, 3), "GBps": round(byts / ms / 1e6, 1),
                          "Gcomp_s": round(comp / ms / 1e6, 2), "comp_per_rec": round(comp / n, 1)}), flush=True)
        del buf, doff, dlen, out, ws


if __name__ == "__main__":
    main()
