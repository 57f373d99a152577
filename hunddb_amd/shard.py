"""Multi-GPU partition of a block batch: one process per GPU, shard by block index.

CRCs of independent blocks are independent, so nothing is exchanged while
computing.  The only collectives are outside the data path:
gathering the 4-byte CRC words to a root (``gather_crcs``) and reducing the
benchmark clock (``job_timing``).  With the "nccl" backend these are RCCL
collectives over xGMI; the same code runs on "gloo" for the CPU tests.
"""
from __future__ import annotations

import os

import numpy as np


def index_range(nblocks: int, world: int, rank: int):
    """Contiguous block-index range [lo, hi) of `rank` (sizes differ by <= 1)."""
    return nblocks * rank // world, nblocks * (rank + 1) // world


def byte_balanced_bounds(lens, world: int) -> np.ndarray:
    """Split boundaries (world+1 indices) balancing the sum of block bytes per
    rank for mixed 4/8/16 KiB batches, using prefix sums."""
    lens = np.asarray(lens, dtype=np.uint64)
    csum = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)])
    total = int(csum[-1])
    targets = [total * r // world for r in range(world + 1)]
    b = np.searchsorted(csum, targets, side="left").astype(np.int64)
    b[0], b[-1] = 0, len(lens)
    return np.maximum.accumulate(b)


def gather_crcs(local, counts, dst: int = 0, group=None):
    """Gather every rank's CRC words (torch int32 tensor) to `dst`, in rank order.

    `counts[r]` = number of blocks of rank r.  Returns the concatenated tensor on
    `dst` and None elsewhere.  Variable sizes are padded to max(counts).  RCCL
    (backend "nccl") all-gathers device tensors over xGMI; gloo gathers host
    copies (CPU tests, one-GPU rehearsals).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    m = max(counts)
    nccl = dist.get_backend(group) == "nccl"
    dev = local.device if nccl else torch.device("cpu")
    pad = torch.zeros(m, dtype=local.dtype, device=dev)
    pad[: local.numel()] = local.to(dev)
    if nccl:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
    else:
        bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
        dist.gather(pad, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def scatter_from_root(full, bounds_bytes, device=None, root: int = 0, group=None):
    """The batch starts on one GPU (reported separately from the
    device-resident numbers): `root` holds the whole uint8 tensor `full` and
    sends every other rank its byte range [bounds_bytes[r], bounds_bytes[r+1])
    by point-to-point transfers (RCCL send/recv over xGMI, batched into one
    group; gloo on CPU tests).  Returns the rank's shard: on the root a view of
    `full`, elsewhere a new tensor on `device`."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    nccl = dist.get_backend(group) == "nccl"
    lo, hi = int(bounds_bytes[rank]), int(bounds_bytes[rank + 1])
    if rank == root:
        # (gloo moves host copies: a one-GPU rehearsal of the RCCL path)
        ops = [dist.P2POp(dist.isend, full[int(bounds_bytes[r]):int(bounds_bytes[r + 1])].contiguous()
                          if nccl else full[int(bounds_bytes[r]):int(bounds_bytes[r + 1])].cpu(), r, group)
               for r in range(world) if r != root and bounds_bytes[r + 1] > bounds_bytes[r]]
        mine = full[lo:hi]
    else:
        mine = torch.empty(hi - lo, dtype=torch.uint8, device=device if nccl else "cpu")
        ops = [dist.P2POp(dist.irecv, mine, root, group)] if hi > lo else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != root and not nccl and device is not None:
        mine = mine.to(device)
    return mine


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


PHASE_ENV = "HC_RANK_PHASE_DIR"  # set by launch_ranks: where each rank records its phase


def report_phase(phase: str, error=None) -> None:
    """Rank side: record this rank's current phase (and, on failure, its error)
    in $HC_RANK_PHASE_DIR/rank<RANK>.json, so the launching parent can name
    the phase a hung or failed rank was in.  A no-op outside launch_ranks."""
    import json
    import time

    d = os.environ.get(PHASE_ENV)
    if not d:
        return
    r = int(os.environ.get("RANK", "0"))
    path = os.path.join(d, f"rank{r}.json")
    with open(path + ".tmp", "w") as f:
        json.dump({"rank": r, "phase": phase, "t": time.time(), "pid": os.getpid(), "error": error}, f)
    os.replace(path + ".tmp", path)  # the parent never reads a half-written file


def _read_phases(d, nproc):
    import json

    out = {}
    for r in range(nproc):
        try:
            with open(os.path.join(d, f"rank{r}.json")) as f:
                out[r] = json.load(f)
        except (OSError, ValueError):
            out[r] = None
    return out


def launch_ranks(cmd, nproc: int, port: int = 0, env=None, timeout=None, grace: float = 5.0):
    """Start `nproc` copies of `cmd` (argv list), one per GPU, with the
    torch.distributed.run environment (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) plus
    HC_RANK_PHASE_DIR, and wait for them -- at most `timeout` seconds.

    The caller must not have touched the GPU (children are started with
    subprocess, never by exec).  When a rank exits non-zero, or the deadline
    passes, every rank still running is terminated (killed after `grace`
    seconds).  Returns (rc, report): rc 0, the first failing rank's exit
    status, or 124 at the deadline; report None on success, else {"reason":
    "rank_failed" | "timeout", "failed": [{rank, rc, phase, error}], "alive":
    [{rank, phase, phase_age_s}] (the ranks still running when it ended),
    "elapsed_s"}."""
    import shutil
    import subprocess
    import tempfile
    import time

    port = port or free_port()
    base = dict(os.environ if env is None else env)
    pdir = tempfile.mkdtemp(prefix="hc_ranks_")
    procs = []
    for r in range(nproc):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **{PHASE_ENV: pdir})
        procs.append(subprocess.Popen(cmd, env=e))
    t0, rc, reason = time.monotonic(), 0, None
    failed, alive = [], []
    live = dict(enumerate(procs))
    try:
        while live:
            for r, p in list(live.items()):
                code = p.poll()
                if code is None:
                    continue
                del live[r]
                if code != 0:
                    failed.append((r, code))
            if failed and live:
                reason = "rank_failed"
            elif timeout is not None and live and time.monotonic() - t0 > timeout:
                reason = "timeout"
            if reason and live:  # name the survivors' phases, then end them
                now = time.time()
                ph = _read_phases(pdir, nproc)
                alive = [{"rank": r, "phase": (ph[r] or {}).get("phase"),
                          "phase_age_s": None if not ph[r] else round(now - ph[r]["t"], 1)} for r in sorted(live)]
                for p in live.values():
                    p.terminate()
                t1 = time.monotonic()
                while any(p.poll() is None for p in live.values()) and time.monotonic() - t1 < grace:
                    time.sleep(0.05)
                for p in live.values():
                    if p.poll() is None:
                        p.kill()
                    p.wait()
                live = {}
                break
            time.sleep(0.05)
        if failed and reason is None:
            reason = "rank_failed"
        if reason is None:
            return 0, None
        ph = _read_phases(pdir, nproc)
        # the first rank to fail is usually the cause (its peers then fail on the
        # closed connection): order by the time each recorded its last phase
        failed.sort(key=lambda rc_: (ph[rc_[0]] or {}).get("t", float("inf")))
        rc = failed[0][1] if failed and reason == "rank_failed" else 124
        return rc, {"reason": reason, "elapsed_s": round(time.monotonic() - t0, 1),
                    "failed": [{"rank": r, "rc": c, "phase": (ph[r] or {}).get("phase"),
                                "error": (ph[r] or {}).get("error")} for r, c in failed],
                    "alive": alive}
    finally:
        for p in procs:  # (an exception in the parent: no orphaned ranks)
            if p.poll() is None:
                p.kill()
                p.wait()
        shutil.rmtree(pdir, ignore_errors=True)


def spawn_ranks(cmd, nproc: int, port: int = 0, env=None, timeout=None) -> int:
    """launch_ranks without the report: 0, the first failing rank's exit
    status, or 124 at the deadline."""
    return launch_ranks(cmd, nproc, port=port, env=env, timeout=timeout)[0]


def rank_identity(device=None, kernel_ms=None) -> dict:
    """What this rank ran on, for a multi-GPU result that proves itself: host,
    pid, the GPU's PCI address and UUID as the HIP runtime reports them, the
    number of GPUs the process sees and how many of them libhundcrc accepts
    (gfx950), and the rank's own mean kernel time.  device=None: a CPU rank."""
    import socket

    import torch
    import torch.distributed as dist

    ident = {"rank": dist.get_rank() if dist.is_initialized() else 0, "host": socket.gethostname(),
             "pid": os.getpid()}
    if device is not None and torch.cuda.is_available():
        from . import crc
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        p = torch.cuda.get_device_properties(idx)
        ident.update({"device": idx, "name": p.name,
                      "bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
                      "uuid": str(p.uuid), "visible_devices": torch.cuda.device_count(),
                      "hc_devices": crc.device_count()})
    else:
        ident.update({"device": "cpu", "name": "cpu", "bus_id": "cpu", "uuid": None,
                      "visible_devices": 0, "hc_devices": 0})
    ident["kernel_ms"] = None if kernel_ms is None else round(float(kernel_ms), 4)
    return ident


def gather_identities(ident: dict, group=None) -> list:
    """Every rank's rank_identity(), in rank order, on every rank."""
    import torch.distributed as dist

    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, ident, group=group)
    return out


def device_proof(idents: list, backend: str, group=None) -> dict:
    """The multi_gpu fields that show which devices the ranks really used:
    the per-rank table, the number of distinct (host, PCI address) pairs, the
    communicator size, the RCCL version and the spread of per-rank kernel
    times.  `rehearsal` is true when ranks share a device (a one-GPU gloo run):
    such a line is not an N-GPU measurement."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else len(idents)
    distinct = len({(i["host"], i["bus_id"]) for i in idents})
    ks = [i["kernel_ms"] for i in idents if i.get("kernel_ms") is not None]
    ver = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            ver = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception as e:  # noqa: BLE001 (reported, not hidden)
            ver = f"unknown ({e})"
    out = {"ranks": idents, "distinct_devices": distinct, "comm_world_size": world, "backend": backend,
           "rccl_version": ver,
           "kernel_ms_max": max(ks) if ks else None, "kernel_ms_min": min(ks) if ks else None,
           "rehearsal": distinct != world}
    if out["rehearsal"]:
        out["rehearsal_note"] = (f"{world} ranks on {distinct} distinct device(s): a rehearsal of the N-GPU path, "
                                 "not an N-GPU measurement")
    return out


def job_timing(wall_s: float, kernel_s: float, local_bytes: float, device=None, group=None):
    """Whole-job numbers for the benchmark: (max wall over ranks, max mean
    kernel time over ranks, sum of bytes over ranks)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return wall_s, kernel_s, local_bytes
    if dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor([wall_s, kernel_s], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    b = torch.tensor([local_bytes], dtype=torch.float64, device=device)
    dist.all_reduce(b, op=dist.ReduceOp.SUM, group=group)
    return float(t[0]), float(t[1]), float(b[0])
