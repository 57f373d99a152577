#!/usr/bin/env python3
"""Where the host-resident MD5 batch (hc_md5_messages) spends its time: the
same pinned records through hc_crc32_messages (same pipeline, CRC kernel) and
hc_md5_messages, with the staging chunk size varied (HC_CHUNK_MB is read when
a thread's pipeline is created, so each size runs in a child process)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(n):
    import numpy as np
    import torch

    from hunddb_amd import crc, merkle as M
    rng = np.random.default_rng(5)
    lens = np.minimum(np.exp(rng.uniform(np.log(64), np.log(65536), n)), 65536).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(off[-1] + lens[-1])
    t = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    buf = t.numpy()
    buf[:] = 7
    res = {"chunk_mb": int(os.environ.get("HC_CHUNK_MB", "64")), "bytes": total}
    for name, fn in (("crc32_messages", lambda: crc.crc32_messages(buf, off, lens)),
                     ("md5_records", lambda: M.md5_records(buf, off, lens))):
        fn()
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        res[name + "_GBps"] = round(total / best / 1e9, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(int(sys.argv[2]))
    else:
        for mb in (64, 256, 1024):
            env = dict(os.environ, HC_CHUNK_MB=str(mb))
            subprocess.run([sys.executable, __file__, "child", "500000"], env=env, check=True)
