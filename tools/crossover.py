"""GPU/host crossover of the host-resident entries (Next 3).

For hc_add_crcs (AddCRCsToData), hc_read_from_disk_v (ReadFromDisk),
hc_verify_blocks (the batched CheckBlockIntegrity) and hc_wal_replay (WAL
recovery), on pageable and pinned host buffers of 16 .. 4096 x 4 KiB blocks:
microseconds per call on the GPU path and on the host path, from 1 caller and
from 4 concurrent callers (SSTable flushes run on a pool of 4 workers,
flush_worker.go:41-48).  Each path is forced with the entry's own
HC_*_GPU_MIN_BLOCKS (set through hc_debug_set: the library reads its
settings from the environment once); the batched verify's host path is the
per-block CheckBlockIntegrity loop it replaces (tools/xover_host.c).

    python tools/crossover.py [--seconds 0.25] [--json-out F] [--sizes 16,64,...]

Prints one JSON object per measurement and a markdown table per entry with
the crossover (smallest size at which the GPU path is faster).  Measurement
tooling; needs a GPU."""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

ENV = {"add_crcs": "HC_ADD_CRCS_GPU_MIN_BLOCKS", "read_from_disk": "HC_READ_GPU_MIN_BLOCKS",
       "wal_replay": "HC_WAL_GPU_MIN_BLOCKS"}
B = 4096
MAXT = 4


def xover_lib():
    path = os.path.join(ROOT, "tools", "libxover.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools"), "libxover.so"])
    L = ctypes.CDLL(path)
    L.xo_check_loop.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
    L.xo_check_loop.restype = ctypes.c_int64
    return L


def alloc(nbytes, pinned, torch):
    if pinned:
        t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        return t.numpy(), t
    a = np.empty(nbytes, dtype=np.uint8)
    return a, a


class Buffers:
    """One caller's buffers for the largest size (every size uses a prefix)."""

    def __init__(self, nmax, pinned, torch, hc, wal_img, seed):
        rng = np.random.default_rng(seed)
        self.keep = []
        self.src, k = alloc(nmax * 4092, pinned, torch)
        self.keep.append(k)
        self.src[:] = rng.integers(0, 256, self.src.size, dtype=np.uint8)
        self.dst = np.empty(nmax * B, dtype=np.uint8)
        self.blocks, k = alloc(nmax * B, pinned, torch)
        self.keep.append(k)
        self.blocks[:] = rng.integers(0, 256, self.blocks.size, dtype=np.uint8)
        for i in range(nmax):  # stamp on the host path
            hc.AddCRCToBlockData(self.blocks[i * B:(i + 1) * B])
        self.payload = np.empty(nmax * B, dtype=np.uint8)
        self.verified = np.zeros((nmax + 31) // 32 + 1, dtype=np.uint32)
        self.wal, k = alloc(nmax * B, pinned, torch)
        self.keep.append(k)
        self.wal[:] = wal_img[:nmax * B]
        slots = nmax * 64
        self.rec_buf = np.empty(nmax * B, dtype=np.uint8)
        self.rec_off = np.empty(slots, dtype=np.uint64)
        self.rec_len = np.empty(slots, dtype=np.uint64)
        self.slots = slots
        self.u64 = (ctypes.c_uint64 * 4)()
        self.i64 = (ctypes.c_int64 * 2)()


def call(entry, path, L, X, b, nb):
    """One call of `entry` over nb blocks; checks the result."""
    if entry == "add_crcs":
        n = nb * 4092
        w = L.hc_add_crcs(b.src.ctypes.data, n, b.dst.ctypes.data, b.dst.nbytes)
        assert w == nb * B, w
    elif entry == "read_from_disk":
        size = nb * (B - 4)
        u, i = b.u64, b.i64
        rc = L.hc_read_from_disk_v(b.blocks.ctypes.data, nb * B, B, 4, size, None, b.payload.ctypes.data,
                                   ctypes.byref(u, 0), ctypes.byref(i, 0), ctypes.byref(u, 8))
        assert rc == 0 and u[1] == nb, (rc, u[1])
    elif entry == "verify_blocks":
        if path == "gpu":
            rc = L.hc_verify_blocks(b.blocks.ctypes.data, None, None, B, B, nb, None, ctypes.byref(b.i64, 0))
            assert rc == 0 and b.i64[0] == -1, rc
        else:
            assert X.xo_check_loop(b.blocks.ctypes.data, nb, B) == -1
    elif entry == "wal_replay":
        u, i = b.u64, b.i64
        rc = L.hc_wal_replay(b.wal.ctypes.data, nb, B, 0, 4, 0, b.rec_buf.ctypes.data, b.rec_buf.nbytes,
                             b.rec_off.ctypes.data, b.rec_len.ctypes.data, b.slots, ctypes.byref(u, 0),
                             ctypes.byref(u, 8), ctypes.byref(u, 16), ctypes.byref(i, 0))
        assert rc == 0 and i[0] == -1, rc


def measure(entry, path, L, X, bufs, nb, threads, seconds):
    """(median us per call, calls, aggregate GB/s of block bytes)."""
    if entry in ENV:
        from hunddb_amd import crc
        crc.debug_set(ENV[entry], "1" if path == "gpu" else str(1 << 30))
    for t in range(threads):  # warm: pipelines, page faults
        for _ in range(3):
            call(entry, path, L, X, bufs[t], nb)
    times = [[] for _ in range(threads)]
    start = threading.Barrier(threads)

    def run(t):
        start.wait()
        t_end = time.perf_counter() + seconds
        ts = times[t]
        while True:
            t0 = time.perf_counter()
            call(entry, path, L, X, bufs[t], nb)
            t1 = time.perf_counter()
            ts.append(t1 - t0)
            if t1 > t_end and len(ts) >= 10:
                break

    w0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    [x.start() for x in th]
    [x.join() for x in th]
    wall = time.perf_counter() - w0
    allt = [x for ts in times for x in ts]
    calls = len(allt)
    return statistics.median(allt) * 1e6, calls, calls * nb * B / wall / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=0.25)
    ap.add_argument("--sizes", default="16,64,256,1024,4096")
    ap.add_argument("--entries", default="add_crcs,read_from_disk,verify_blocks,wal_replay")
    ap.add_argument("--mem", default="pageable,pinned")
    ap.add_argument("--threads", default="1,4")
    ap.add_argument("--json-out")
    a = ap.parse_args()
    import torch

    import walgen
    from hunddb_amd import crc as hc
    assert torch.cuda.is_available() and hc.device_count() > 0, "crossover needs a gfx950 GPU"
    L, X = hc.lib(), xover_lib()
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    plan = walgen.WalPlan(0x57414C, nrec=nmax)  # ~2.5 blocks per record: enough blocks
    assert plan.nblocks >= nmax
    wal_img = plan.render(0, nmax)
    res = []
    out = open(a.json_out, "w") if a.json_out else None
    for mem in a.mem.split(","):
        bufs = [Buffers(nmax, mem == "pinned", torch, hc, wal_img, 100 + t) for t in range(MAXT)]
        for entry in a.entries.split(","):
            for nb in sizes:
                for threads in [int(x) for x in a.threads.split(",")]:
                    row = {"entry": entry, "mem": mem, "blocks": nb, "threads": threads}
                    for path in ("host", "gpu"):
                        us, calls, gbs = measure(entry, path, L, X, bufs, nb, threads, a.seconds)
                        row[f"{path}_us"] = round(us, 1)
                        row[f"{path}_gb_s"] = round(gbs, 2)
                        row[f"{path}_calls"] = calls
                    row["gpu_faster"] = row["gpu_us"] < row["host_us"]
                    print(json.dumps(row), flush=True)
                    if out:
                        out.write(json.dumps(row) + "\n")
                        out.flush()
                    res.append(row)
        del bufs
    for k in ENV:
        hc.debug_set(ENV[k], None)
    # tables
    for entry in a.entries.split(","):
        print(f"\n### {entry}\n")
        print("| mem | callers | " + " | ".join(f"{n} blk host / GPU us" for n in sizes) + " | crossover |")
        print("|---|---|" + "---|" * len(sizes) + "---|")
        for mem in a.mem.split(","):
            for threads in [int(x) for x in a.threads.split(",")]:
                rows = [r for r in res if r["entry"] == entry and r["mem"] == mem and r["threads"] == threads]
                rows.sort(key=lambda r: r["blocks"])
                cross = next((r["blocks"] for r in rows if r["gpu_faster"]), None)
                print(f"| {mem} | {threads} | " + " | ".join(f"{r['host_us']} / {r['gpu_us']}" for r in rows)
                      + f" | {cross if cross is not None else '> ' + str(sizes[-1])} |")


if __name__ == "__main__":
    main()
