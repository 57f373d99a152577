#!/usr/bin/env python3
"""Benchmark of the batched block-checksum hot path (BASELINE.json metric).

One "step" = CRC-32/IEEE of every block of one device-resident batch (what
HundDB's utils/crc CheckBlockIntegrity computes per block,
/root/reference/utils/crc/crc_util.go:88-100), through the C ABI
(hc_dev_crc32_blocks) into the hand-written gfx950 streaming kernel.

Workloads (synthetic splitmix64 data keyed by GLOBAL block index, generated in HBM):
  N = 1, default   the north star, 1M x 8 KiB (8.192 GB), BASELINE.json's target config.
  N > 1, default   configs[3] strong scaling: ONE global batch of 16M x 8 KiB
                   (131 GB) split by block index (hunddb_amd.shard.index_range),
                   rank r fills and hashes blocks [lo_r, hi_r) of it.  After the
                   timed region the CRC words are all-gathered over RCCL and rank 0
                   re-runs the WHOLE batch alone: `speedup_vs_1gpu` is that 1-GPU
                   step time / the N-GPU step time on the same batch, and the
                   gathered words must equal the 1-GPU words.
  --workload       any of WORKLOADS below (configs[1], configs[2], 16 KiB, the
                   framing kernels f1/f2, off/len metadata path).

`python bench.py --gpus N` with no WORLD_SIZE in the environment starts its N
ranks itself (subprocesses with the torch.distributed.run environment, started
before this process touches the GPU); under torch.distributed.run it is one rank.

Prints ONE JSON line (rank 0): value = whole-job GiB/s (all ranks' bytes / the
max-over-ranks wall time of the K timed steps), the roofline of the dominant
kernel (algorithmic bytes per launch / mean HIP-event launch time vs 8 TB/s, PMC
traffic from rocprofv3 child runs at N=1) and, at N=1, the CPU baseline (the
oracle's restatement of Go's crc32.ChecksumIEEE on the host cores, 1 thread and
all threads with the run-to-run spread, and system zlib's crc32 as a second,
independent point).
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
COPY_CEILING_GBS = 6290.0  # MI355X_MICROARCH.md: measured float4 copy (SURVEY 8(d) asks for both)
SEED = 0x48756E64
WORKLOADS = {
    # name: (blocks per rank (weak) or in total (strong), block bytes or kind, scaling)
    "northstar": (1_000_000, 8192, "weak"),
    "config2": (1_000_000, 4096, "weak"),
    "config3": (1_000_000, "mixed", "weak"),
    "config4": (16_000_000, 8192, "strong"),
    "16k": (500_000, 16384, "weak"),
    # f2: fused AddCRCsToData (k_frame): 1M output blocks = 4092 MB payload read
    # from an unaligned address, 4096 MB framed blocks written
    "frame": (1_000_000, "frame", "weak"),
    # f1: batched ReadFromDisk (k_unframe): verify 1M x 4 KiB blocks and strip
    # the CRC words (4096 MB read, 4092 MB payload written)
    "unframe": (1_000_000, "unframe", "weak"),
    # the same at HundDB's other block sizes (config.go:137, README.md:191,255):
    # 0.5M x 8 KiB and 0.25M x 16 KiB (4 GB each way)
    "unframe8k": (500_000, "unframe8k", "weak"),
    "unframe16k": (250_000, "unframe16k", "weak"),
    # config2's blocks described by off/len arrays (the per-block metadata path)
    "offlen4k": (1_000_000, "offlen4k", "weak"),
    # verify mode (CheckBlockIntegrity over the north-star batch, stamped): read B,
    # compare, write the 4-B word + bitmap bits; SURVEY 8(d) counts B + 4 per block
    "verify": (1_000_000, "verify", "weak"),
    # configs[4]'s per-record variant on the device (SURVEY 8(d) config 5 notes):
    # GetCRC of 2M records, log-uniform 64 B - 64 KiB, back to back at an odd
    # address (18.9 GB) -> the packed-record stream (k_seg_*); bytes = record
    # bytes read + 4-B words written
    "records": (2_000_000, "records", "weak"),
    # the same records with a 17-B gap before each (the WAL header between
    # payloads, /root/reference/lsm/wal/wal_header.go:5-23): the stream over the
    # 2n record boundaries (round 5); bytes = record bytes + 4-B words (the gap
    # bytes the stream also reads are not counted)
    "records_gapped": (2_000_000, "records_gapped", "weak"),
    # GetCRC of 1M aligned 4 KiB records in shuffled order: the
    # stream refuses them; its fallback runs k_crc_grp's body inside the combine
    "records4k_shuffled": (1_000_000, "records4k_shuffled", "weak"),
    # config 5's records (log-uniform 64 B - 64 KiB, back to back from an odd
    # address) with their off/len arrays in a permuted order:
    # the plan finds them unsorted, so the stream refuses them
    "records_shuffled": (2_000_000, "records_shuffled", "weak"),
    # uniform blocks k_crc_grp refuses (config.go:241 allows any BlockSize >= 1024): 1M x 4092 B
    # and 0.5M x 8188 B, their messages block[4:] on the stream's small-gap mode
    # (launch_seg_blocks; round 5; 4-B aligned 2-8 KiB blocks stayed on k_crc_any until round 6)
    "blocks4092": (1_000_000, 4092, "weak"),
    "blocks8188": (500_000, 8188, "weak"),
}
# PMC passes count every kernel a dispatch launches (plan, stream, combine, the
# gated k_crc_grp / k_crc_any fallbacks, the block-route helpers), not one
# kernel: the traffic of a multi-kernel dispatch is their sum
PMC_KERNELS = r"k_(crc|seg|frame|unframe)"
PMC_EXCLUDE = ("k_fill", "k_verify_prepare")
SEG_WORKLOADS = ("records", "records_gapped", "records4k_shuffled", "records_shuffled", "blocks4092", "blocks8188")  # on k_seg_*: stream_mode
UNFRAME_B = {"unframe": 4096, "unframe8k": 8192, "unframe16k": 16384}  # f1 block sizes


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: northstar at N=1, config4 (strong scaling) at N>1")
    ap.add_argument("--blocks", type=int, default=0, help="override the block count")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = the CPUs this process may run on, capped by the cgroup quota)")
    ap.add_argument("--pmc", choices=["auto", "on", "off"], default="auto",
                    help="collect FETCH_SIZE/WRITE_SIZE in rocprofv3 child runs (N=1 only)")
    ap.add_argument("--ref1", choices=["auto", "on", "off"], default="auto",
                    help="strong scaling: rank 0 re-runs the whole batch alone (speedup + word check)")
    ap.add_argument("--settle", type=float, default=0.5, help="untimed clock-settle seconds before warmup")
    # bracket: one event pair on the launch stream around the K launches (the mean
    # launch time then includes the ~1.5 us gaps between launches: conservative);
    # step: a pair around every launch, whose recording costs the wall clock
    # ~0.5 % (profiles/r2/bench_events/)
    ap.add_argument("--kernel-events", choices=["step", "bracket"], default="bracket",
                    help="HIP events around the K launches (bracket) or around every launch (step)")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--input", choices=["resident", "scatter"], default="resident",
                    help="N>1 strong scaling: each rank fills its shard in HBM (resident), or rank 0 holds the "
                         "whole batch and sends the shards over RCCL first (scatter; timed and reported "
                         "separately, SURVEY.md 8e)")
    ap.add_argument("--host-leg", choices=["auto", "on", "off"], default="auto",
                    help="N=1: the host-inclusive leg (blocks in host memory, PCIe included; auto = northstar only)")
    ap.add_argument("--rank-timeout", type=float, default=900.0,
                    help="N>1: seconds the self-launcher waits for its ranks (then kills them and prints one JSON "
                         "error line naming the ranks still alive and their phase); also the process-group timeout")
    ap.add_argument("--json-out", default="")
    return ap.parse_args(argv)


METRIC = "GiB/s CRC32 over device-resident batched 4/8/16 KB blocks; % HBM peak"
WORKLOAD_NOTE = ("with no --workload, N = 1 runs northstar (1M x 8 KiB, the target config, scaling weak) and N > 1 "
                 "runs config4 (configs[3]: one 16M x 8 KiB batch split by block index, scaling strong): the value "
                 "column therefore changes batch between N = 1 and N > 1; multi_gpu.speedup_vs_1gpu (rank 0's "
                 "1-GPU run of the same 16M-block batch) is the like-for-like number")


def phase(name):
    """Record this rank's phase for the self-launcher (hunddb_amd.shard.report_phase);
    HC_BENCH_STALL=rank:phase:seconds / HC_BENCH_FAIL=rank:phase make a rank
    sleep in, or fail at, a phase (the launcher's deadline and failure tests)."""
    from hunddb_amd import shard
    shard.report_phase(name)
    rank = os.environ.get("RANK", "0")
    st = os.environ.get("HC_BENCH_STALL", "").split(":")
    if len(st) == 3 and st[0] == rank and st[1] == name:
        time.sleep(float(st[2]))
    fl = os.environ.get("HC_BENCH_FAIL", "").split(":")
    if len(fl) == 2 and fl[0] == rank and fl[1] == name:
        raise RuntimeError(f"HC_BENCH_FAIL at {name}")


# --------------------------------------------------------------------------
# PMC traffic via rocprofv3 child runs (started before this process touches
# the GPU; one counter group per pass as MI355X_MICROARCH.md prescribes).
def pmc_traffic(args):
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    out = {}
    steps = 3
    tmp = tempfile.mkdtemp(prefix="hc_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.abspath(__file__), "--child", "--steps", str(steps), "--warmup", "1",
             "--workload", args.workload, "--cpu-seconds", "0", "--pmc", "off", "--settle", "0"]
    if args.blocks:
        child += ["--blocks", str(args.blocks)]
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(tmp, ctr)
        cmd = [exe, "--pmc", ctr, "--kernel-include-regex", PMC_KERNELS, "--output-format", "csv",
               "-d", d, "-o", "run", "--"] + child
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300,
                               cwd=tmp, env=dict(os.environ, TMPDIR=tmp))
        except subprocess.TimeoutExpired:
            return None, f"rocprofv3 {ctr} pass timed out"
        if r.returncode != 0:
            return None, f"rocprofv3 {ctr} pass failed rc={r.returncode}: {r.stdout[-400:].decode(errors='replace')}"
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                rows += [row for row in csv.DictReader(fh) if row.get("Counter_Name") == ctr]
        out[ctr] = dispatch_traffic(rows, steps)
        if not out[ctr]:
            return None, f"no {ctr} rows"
    shutil.rmtree(tmp, ignore_errors=True)
    # units: KiB; gfx950 FETCH_SIZE reports half the bytes of 16-B/lane streaming
    # reads (MI355X_MICROARCH.md "HBM") -> x2
    by_kernel = {k: 2.0 * 1024.0 * out["FETCH_SIZE"].get(k, 0.0) + 1024.0 * out["WRITE_SIZE"].get(k, 0.0)
                 for k in sorted(set(out["FETCH_SIZE"]) | set(out["WRITE_SIZE"]))}
    fetch = 2.0 * 1024.0 * sum(out["FETCH_SIZE"].values())
    write = 1024.0 * sum(out["WRITE_SIZE"].values())
    return {"fetch_bytes": fetch, "write_bytes": write, "bytes": fetch + write,
            "by_kernel": {k: round(v) for k, v in by_kernel.items()},
            "raw_fetch_kib": sum(out["FETCH_SIZE"].values()), "raw_write_kib": sum(out["WRITE_SIZE"].values())}, None


def dispatch_traffic(rows, steps):
    """Per-dispatch counter value of every kernel the timed dispatches launch:
    rows are rocprofv3 counter_collection rows of one counter, in dispatch
    order.  A kernel belongs to the dispatch when it ran at least `steps` + 1
    times (warmup + timed); its value is the mean of its last `steps` rows (a
    kernel the workload's setup also launched -- the stamp before verify --
    keeps only the timed ones).  Returns {short kernel name: mean value}."""
    per = {}
    for row in rows:
        m = re.search(r"\b(k_[a-z0-9_]+)(<[^>]*>)?", row.get("Kernel_Name", ""))
        if not m or m.group(1) in PMC_EXCLUDE:
            continue
        per.setdefault(m.group(0), []).append(float(row["Counter_Value"]))  # one entry per template instance
    return {k: sum(v[-steps:]) / steps for k, v in per.items() if len(v) >= steps + 1}


def bytes_kernel(dispatch, seg_mode):
    """The kernel that moved the bytes of a dispatch: the stream's mode word says
    which of the packed-record path's kernels did the work."""
    if seg_mode in (False, None) or not dispatch.startswith("k_seg_plan"):
        return dispatch
    if seg_mode.startswith("sorted_"):  # the sort's phases ran in k_seg_stream too
        return "k_seg_stream"
    return {"packed": "k_seg_stream", "gapped": "k_seg_stream", "gapped_wide": "k_seg_stream",
            "fallback_grp": "k_crc_grp", "fallback": "k_seg_combine"}.get(seg_mode, dispatch)


def mixed_sizes(seed, lo, n):
    """Config-3 block sizes of global blocks lo .. lo+n-1: 4096 << (splitmix64(seed
    ^ 0x5A.., i, 2^21-1) % 3), the same draw as tests/golden/gen_golden.py."""
    import numpy as np
    i = np.arange(lo, lo + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed ^ 0x5A5A5A5A5A5A5A5A) + ((i << np.uint64(21)) + np.uint64((1 << 21) - 1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (np.uint32(4096) << (z % np.uint64(3)).astype(np.uint32)).astype(np.uint32)


# --------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the reference's CPU path timed on the host cores
def _rate(fn, nbytes, seconds):
    """GiB/s of fn() (nbytes per call) run back to back for >= seconds."""
    return _rate_cpu(fn, nbytes, seconds, 1)[0]


def _rate_cpu(fn, nbytes, seconds, threads):
    """fn() (nbytes per call) run back to back for >= seconds: (wall-clock
    GiB/s, GiB/s per `threads` CPUs of the process's CPU time, busy = CPU time
    / (threads x wall)).  The host is shared: a slice's wall time also holds
    the time other tenants' threads ran on the pinned CPUs (round 6,
    tools/cpu_spread_probe.py: 16 threads were on a CPU 67-85 % of each slice,
    and the wall-clock rate followed), which the process's CPU time leaves out."""
    fn()
    t0, c0, k = time.perf_counter(), time.process_time(), 0
    while True:
        fn()
        k += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            ct = time.process_time() - c0
            gib = k * nbytes / 2**30
            return gib / dt, gib / (ct / threads) if ct > 0 else float("nan"), ct / (threads * dt)


def cgroup_cpu_quota():
    """CPUs the cgroup lets this process use (cgroup v2 cpu.max, v1
    cfs_quota/period), or None when unlimited or not readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = float(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cores_available():
    """Threads the CPU baseline can actually run at once: the CPUs in this
    process's affinity set, capped by the cgroup quota."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    return max(1, min(n, int(q))) if q else n


N_SLICES = 7
_AFFINITY0 = os.sched_getaffinity(0)  # the process's own set (the baseline pins itself inside it)


def _cpu_idle():
    """Per logical CPU idle + iowait jiffies (/proc/stat), or {} if unreadable."""
    out = {}
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    v = line.split()
                    out[int(v[0][3:])] = int(v[4]) + int(v[5])
    except (OSError, ValueError, IndexError):
        pass
    return out


def quiet_cores(n, sample_s=0.3):
    """n logical CPUs of this process's affinity set on n distinct physical
    cores (no two on SMT siblings), the most idle ones over sample_s seconds
    (both siblings' idle time counted); None when the topology is not readable.
    The host is shared (16 of 256 logical CPUs by quota): unpinned, the CPU
    baseline's 16 threads land on busy cores and on each other's siblings, and
    its slices spread -13 / +25 % (round 6's first run)."""
    allowed = sorted(os.sched_getaffinity(0))
    core = {}
    try:
        for c in allowed:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "physical_package_id") as f:
                pk = int(f.read())
            with open(base + "core_id") as f:
                core.setdefault((pk, int(f.read())), []).append(c)
    except (OSError, ValueError):
        return None
    if len(core) < n:
        return None
    a = _cpu_idle()
    time.sleep(sample_s)
    b = _cpu_idle()
    idle = lambda cpus: sum(b.get(c, 0) - a.get(c, 0) for c in cpus)  # noqa: E731
    best = sorted(core.values(), key=lambda cpus: (-idle(cpus), cpus[0]))[:n]
    return sorted(c[0] for c in best)


class pinned:
    """Within the block, this thread (and the threads it starts) run on
    quiet_cores(n); restores the previous affinity after."""

    def __init__(self, n):
        self.n, self.cpus, self.prev = n, None, None

    def __enter__(self):
        self.prev = os.sched_getaffinity(0)
        self.cpus = quiet_cores(self.n)
        if self.cpus:
            os.sched_setaffinity(0, self.cpus)
        return self

    def __exit__(self, *exc):
        os.sched_setaffinity(0, self.prev)
        return False

    def info(self):
        return {"pinned_cpus": self.cpus,
                "pinning": ("one logical CPU per physical core, the most idle cores of the affinity set over 0.3 s "
                            "(/proc/stat), for the whole CPU-baseline leg" if self.cpus else
                            "none (topology not readable or too few cores)")}


def cgroup_throttled_us():
    """Microseconds the cgroup's CPU quota has held this process's threads back
    so far (cgroup v2 cpu.stat throttled_usec), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                if k == "throttled_usec":
                    return int(v)
    except (OSError, ValueError):
        pass
    return None


CPU_REGION = 16 << 20  # the CPU baseline's timed set: the sample's first 16 MiB (cpu_baseline)
CPU_CALL = 1 << 30     # ... listed over and over to 1 GiB a call
WARM_AGREE = 0.05   # warm-up ends when two consecutive warm-up slices agree within 5 %
WARM_CAP_S = 6.0    # ... or after this long (1.8 s did not reach steady state)


def _slices(fn, nbytes, budget_s, threads):
    """N_SLICES timed slices of fn (0.08 of the budget each), separated by idle
    gaps of 0.1 s so that one burst of another tenant on the host lands in one
    slice rather than in all of them; the median is the reported value.  Each
    slice's rate is taken against the process's CPU time (_rate_cpu), its
    wall-clock rate kept beside it.  Before them an untimed warm-up of slices of
    the same length, until two consecutive ones agree within WARM_AGREE (at most
    WARM_CAP_S): the host's cores ramp up over seconds (round 5's first slices
    read 113-139 GiB/s, the rest 162-169).  Also returns how long the cgroup's
    CPU quota throttled the process in each slice (the quota covers every thread
    of the container, not only the timed ones), and the warm-up's slices."""
    out, wall, busy, thr, warm = [], [], [], [], []
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < WARM_CAP_S:
        warm.append(_rate_cpu(fn, nbytes, 0.08 * budget_s, threads)[1])
        if len(warm) >= 2 and abs(warm[-1] / warm[-2] - 1.0) <= WARM_AGREE:
            break
    warm_s = time.perf_counter() - t_warm
    for k in range(N_SLICES):
        if k:
            time.sleep(0.1)
        t0 = cgroup_throttled_us()
        w, c, b = _rate_cpu(fn, nbytes, 0.08 * budget_s, threads)
        out.append(c)
        wall.append(w)
        busy.append(b)
        t1 = cgroup_throttled_us()
        thr.append(None if t0 is None or t1 is None else round((t1 - t0) / 1e3, 1))
    return out, thr, {"warmup_s": round(warm_s, 2), "warmup_slices": [round(x, 2) for x in warm],
                      "warmup_converged": len(warm) >= 2 and abs(warm[-1] / warm[-2] - 1.0) <= WARM_AGREE,
                      "wall": wall, "busy": busy}


def _spread(sl, budget_s, threads):
    import numpy as np
    slices, thr, info = sl
    info = dict(info)
    wall, busy = info.pop("wall"), info.pop("busy")
    med, wmed = float(np.median(slices)), float(np.median(wall))
    return {"spread": [round(min(slices), 3), round(max(slices), 3)],
            "spread_pct": [round(100.0 * (min(slices) / med - 1.0), 1), round(100.0 * (max(slices) / med - 1.0), 1)],
            "slices": [round(x, 2) for x in slices],
            "slices_busy": [round(x, 3) for x in busy],
            "wall_clock": {"value": round(wmed, 3),
                           "spread_pct": [round(100.0 * (min(wall) / wmed - 1.0), 1),
                                          round(100.0 * (max(wall) / wmed - 1.0), 1)],
                           "slices": [round(x, 2) for x in wall]},
            "slices_throttled_ms": thr,
            **info,
            "rate_note": f"value and slices: GiB per {threads} CPUs of the process's CPU time (bytes / (CPU s / "
                         f"{threads})), what {threads} cores of its own would do; the host is shared and "
                         f"slices_busy (CPU time / ({threads} x wall)) shows the share of each slice the pinned "
                         f"threads were on a CPU (round 6: 0.67-0.85, tools/cpu_spread_probe.py); wall_clock: the "
                         f"same slices by the wall clock",
            "spread_note": f"min/max of {len(slices)} slices of {0.08 * budget_s:.2f} s on {threads} threads after "
                           f"an untimed warm-up of slices of the same length until two consecutive ones agreed "
                           f"within {100 * WARM_AGREE:.0f} % (cap {WARM_CAP_S:.0f} s; warmup_s, warmup_slices), "
                           f"0.1 s idle between slices, work handed to the threads in 64-block chunks; "
                           f"slices_throttled_ms: time the cgroup CPU quota (cgroup_cpu_quota CPUs for the "
                           f"whole container) stalled the process during each slice"}


def cpu_host():
    """The host's CPU model and the CPU counts (SURVEY 8(d) asks for the core
    count): logical CPUs of the machine, the affinity set, the cgroup quota."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    q = cgroup_cpu_quota()
    return {"cpu_model": model, "logical_cpus": os.cpu_count(), "affinity_cpus": len(_AFFINITY0),
            "cgroup_cpu_quota": None if q is None else round(q, 2), "cores_available": cores_available()}


def record_sizes(n):
    """configs[4]'s record law: log-uniform in [64, 65536] B (u = splitmix64(0x5B,
    i, 0) >> 11 / 2^53, tools/kbench2.hip's draw)."""
    import numpy as np
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(0x5B) + (i << np.uint64(21)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) / 9007199254740992.0
    return (64.0 * np.exp(u * np.log(1024.0))).astype(np.uint32)


def cpu_baseline(sample, off, lens, threads, budget_s, what, gpu_words=None, messages=False):
    """Go's crc32.ChecksumIEEE over block[4:len] of every sample block
    (crc_util.go:16,94; with messages: over each whole record, GetCRC
    crc_util.go:15-17), three ways: the oracle's restatement of Go's amd64
    algorithm (oracle/hc_oracle.c oc_crc32_go_amd64: PCLMULQDQ fold + slicing-by-8)
    on `threads` threads (5 slices: median and spread) and on 1 thread, and
    system zlib's crc32 (Python zlib, an independent implementation) on 1 thread.
    The oracle's words for the sample are also compared with the GPU's."""
    import zlib

    import numpy as np

    from oracle import oracle as O

    def runner(o, ln):
        if messages:
            return lambda t: O.crc32_messages(sample, o, ln, threads=t)
        return lambda t: O.crc32_blocks(sample, off=o, lens=ln, threads=t)
    words = runner(off, lens)(threads)  # every word of the sample, against the GPU's
    # The timed set: the sample's blocks (records) inside its first CPU_REGION
    # bytes, listed over and over to CPU_CALL bytes a call -- cache-resident, as
    # the reference's CRC runs on a block it has just read into a fresh buffer
    # (block_manager.go:203-235) or just serialized (wal.go:261) -- and long
    # enough a call to bury the port's per-call thread start.
    o0 = int(off.min()) if len(off) else 0
    inr = np.nonzero(off.astype(np.uint64) + lens.astype(np.uint64) <= np.uint64(o0 + CPU_REGION))[0]
    rb = int(lens[inr].sum(dtype=np.uint64))
    reps = max(1, -(-CPU_CALL // max(rb, 1)))
    toff, tlen = np.tile(off[inr], reps), np.tile(lens[inr], reps)
    nbytes = rb * reps
    port = runner(toff, tlen)
    mv = memoryview(sample)
    skip = 0 if messages else 4
    pairs = list(zip(off[inr].tolist(), lens[inr].tolist()))

    def zl():
        for o, n_ in pairs:
            zlib.crc32(mv[o + skip:o + n_])
    zl_ok = all(zlib.crc32(mv[o + skip:o + n_]) == int(words[inr[k]]) for k, (o, n_) in enumerate(pairs[:200]))
    slices = _slices(lambda: port(threads), nbytes, budget_s, threads)
    one = _rate_cpu(lambda: port(1), nbytes, 0.2 * budget_s, 1)[1]
    zrate = _rate_cpu(zl, rb, 0.2 * budget_s, 1)[1]
    nsb = int(lens.sum(dtype=np.uint64))
    unit = "records" if messages else "blocks"
    res = {"value": round(float(np.median(slices[0])), 3), "unit": "GiB/s", "cores": threads, "kind": "port",
           "sample": f"{what}: {len(off)} {unit}, {nsb / 2**20:.0f} MiB copied from the GPU batch (every word "
                     f"checked against the GPU's); timed: its {len(inr)} {unit} in the first "
                     f"{CPU_REGION >> 20} MiB ({rb / 2**20:.1f} MiB, cache-resident) listed {reps} times a call; "
                     f"oracle/hc_oracle.c oc_crc32_go_amd64 restates Go 1.23 hash/crc32 amd64 "
                     f"(PCLMULQDQ fold + slicing-by-8), pclmul={O.lib().oc_have_pclmul()}",
           **_spread(slices, budget_s, threads),
           "single_thread": round(one, 3),
           "zlib_single_thread": round(zrate, 3),
           "zlib_note": f"system zlib {zlib.ZLIB_RUNTIME_VERSION} crc32 via Python, 1 thread, the timed region once "
                        f"a call (both single-thread rates per CPU second); same words as the oracle on the "
                        f"first 200 {unit}: {zl_ok}"}
    if gpu_words is not None:
        res["matches_gpu"] = bool(np.array_equal(words, gpu_words))
    res.update(cpu_host())
    return res


def cpu_baseline_framing(kind, dev_src, threads, budget_s, B=4096):
    """The oracle's restatement of the reference loop over a 256 MB sample of
    the same data (Go runs each AddCRCsToData / ReadFromDisk call on one
    goroutine): 1 thread, and `threads` threads on disjoint slices; bytes
    counted as in the GPU line (read + written)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    from oracle import oracle as O
    L = O.lib()
    nblk = (256 << 20) // B
    per_t = nblk // threads
    P = B - 4  # payload bytes per block
    if kind == "frame":  # crc_util.go:41-64 (B = 4096: the function's constant framing)
        src = dev_src[: nblk * P].cpu().numpy()
        dst = np.empty(nblk * B, dtype=np.uint8)

        def run(a, b):
            L.oc_add_crcs_to_data(src.ctypes.data + a * P, (b - a) * P, dst.ctypes.data + a * B)
        what = f"oc_add_crcs_to_data over {src.size} B of payload (crc_util.go:41-64)"
    else:  # block_manager.go:189-242
        blocks = dev_src[: nblk * B].cpu().numpy()
        out = np.empty(nblk * P, dtype=np.uint8)

        def run(a, b):
            fo, bad = ctypes.c_uint64(0), ctypes.c_int64(0)
            L.oc_read_from_disk(blocks.ctypes.data + a * B, (b - a) * B, B, 0, (b - a) * P,
                                out.ctypes.data + a * P, ctypes.byref(fo), ctypes.byref(bad))
        what = f"oc_read_from_disk over {nblk} stamped {B}-B blocks (block_manager.go:189-242)"
    nbytes = nblk * (P + B)
    pool = ThreadPoolExecutor(threads)

    def par():  # ctypes releases the GIL for the call
        list(pool.map(lambda t: run(t * per_t, (t + 1) * per_t), range(threads)))
    slices = _slices(par, per_t * threads * (P + B), budget_s, threads)
    one = _rate_cpu(lambda: run(0, nblk), nbytes, 0.3 * budget_s, 1)[1]
    pool.shutdown()
    return {"value": round(float(np.median(slices[0])), 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{what}, read+written bytes",
            **_spread(slices, budget_s, threads),
            "single_thread": round(one, 3), **cpu_host()}


# --------------------------------------------------------------------------
# Host-inclusive leg (N = 1, outside the timed device region): the blocks start
# and end in host memory (WAL segment files, SSTable files), so BASELINE.json's
# north star also asks for the rate with the H2D copy of the blocks and the D2H
# copy of the CRC words overlapped on side streams (the library's host
# pipelines), against the link's own pinned hipMemcpyAsync peak.
def _best_rate(fn, nbytes, reps):
    fn()  # warm: pipelines, page faults
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return nbytes / best / 1e9, best


def h2d_peak(torch, pinned, seconds=1.0):
    """GB/s of pinned host -> device hipMemcpyAsync (torch copies), 256 MiB
    chunks on two streams: the link's practical ceiling on this box."""
    chunk = min(256 << 20, pinned.numel())  # (a small --blocks run: one chunk of the whole buffer)
    n = pinned.numel() // chunk if chunk else 0
    if n == 0:
        return 0.0
    dst = [torch.empty(chunk, dtype=torch.uint8, device="cuda") for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    best = 0.0
    t_end = time.perf_counter() + seconds
    while True:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            with torch.cuda.stream(streams[k % 2]):
                dst[k % 3].copy_(pinned[k * chunk:(k + 1) * chunk], non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, n * chunk / (time.perf_counter() - t0) / 1e9)
        if time.perf_counter() > t_end:
            return best


def host_inclusive(torch, crc, dev_buf, dev_words, B, reps=3, wal_records=2_000_000):
    """hc_crc32_blocks over the north-star batch from pinned and from pageable
    host memory (words against the device run), hc_verify_blocks over a
    config-5-shaped WAL image in pinned memory (2M records framed as
    lsm/wal/wal.go:177-283, tools/walgen.c), and the same run's pinned H2D
    peak; rates in GB/s of block bytes per wall second, best of `reps`."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import walgen
    t_leg = time.perf_counter()
    n = dev_words.numel()
    nbytes = n * B
    want = dev_words.cpu().numpy().view(np.uint32)
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(dev_buf[:nbytes])
    peak = h2d_peak(torch, pinned)
    res = {"h2d_peak_gb_s": round(peak, 2), "pcie_nominal_gb_s": 63.0,
           "h2d_peak_note": "pinned hipMemcpyAsync H2D, 256 MiB chunks on 2 streams, this run"}
    words = {}

    def leg(name, host):
        out = {}
        r, t = _best_rate(lambda: out.__setitem__("w", crc.crc32_blocks(host, stride=B, ulen=B, nblocks=n)),
                          nbytes, reps)
        words[name] = out["w"]
        res[name] = {"workload": f"hc_crc32_blocks, {n} x {B} B", "gb_s": round(r, 2), "s": round(t, 4),
                     "frac_h2d_peak": round(r / peak, 3) if peak else None, "frac_pcie_gen5_x16": round(r / 63.0, 3),
                     "words_match_device": bool(np.array_equal(out["w"], want))}
    leg("crc32_blocks_pinned", pinned.numpy())
    pageable = np.empty(nbytes, dtype=np.uint8)
    pageable[:] = pinned.numpy()
    del pinned
    leg("crc32_blocks_pageable", pageable)
    del pageable
    plan = walgen.WalPlan(0x57414C, nrec=wal_records)
    nb = plan.nblocks
    img = torch.empty(nb * 4096, dtype=torch.uint8, pin_memory=True)
    host = img.numpy()
    step = 1 << 18
    for b0 in range(0, nb, step):
        plan.render(b0, min(nb, b0 + step), out=host[b0 * 4096:min(nb, b0 + step) * 4096], threads=cores_available())
    got = {}
    r, t = _best_rate(lambda: got.__setitem__("v", crc.verify_blocks(host, stride=4096, ulen=4096, nblocks=nb)),
                      nb * 4096, reps)
    err, bm, fb = got["v"]
    res["wal_verify_pinned"] = {"workload": f"hc_verify_blocks over a config-5 WAL image: {wal_records} records "
                                            f"(64 B - 64 KiB log-uniform) framed into {nb} x 4 KiB blocks",
                                "gb_s": round(r, 2), "s": round(t, 4), "frac_h2d_peak": round(r / peak, 3) if peak else None,
                                "frac_pcie_gen5_x16": round(r / 63.0, 3),
                                "all_blocks_verify": err is None and fb == -1 and not bm.any()}
    del img
    res["words_match_device"] = all(res[k]["words_match_device"] for k in ("crc32_blocks_pinned",
                                                                            "crc32_blocks_pageable"))
    res["leg_s"] = round(time.perf_counter() - t_leg, 1)
    return res


# --------------------------------------------------------------------------
def self_launch(argv, nproc, script=None):
    """`bench.py --gpus N` without WORLD_SIZE: run N ranks (one per GPU) as child
    processes with the torch.distributed.run environment; this process never
    touches the GPU.  The ranks get --rank-timeout seconds: when one fails or
    the deadline passes, the others are killed and this process prints ONE
    JSON error line (the failed ranks with their phase and error, the ranks
    still alive with their last phase).  Returns 0 or a non-zero status."""
    from hunddb_amd import shard
    cmd = [sys.executable, os.path.abspath(script or __file__)] + list(argv)
    try:
        tmo = parse(list(argv)).rank_timeout
    except SystemExit:  # (--help and the like: the children print it)
        tmo = 900.0
    rc, rep = shard.launch_ranks(cmd, nproc, timeout=tmo if tmo > 0 else None)
    if rep is not None:
        what = (f"{len(rep['alive'])} of {nproc} ranks still running after the {tmo:g} s deadline"
                if rep["reason"] == "timeout" else
                "rank " + ", ".join(str(f["rank"]) for f in rep["failed"]) + " failed")
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": nproc, "error": what,
                          "reason": rep["reason"], "rank_timeout_s": tmo, "elapsed_s": rep["elapsed_s"],
                          "failed_ranks": rep["failed"], "alive_ranks": rep["alive"]}), flush=True)
    return rc


def main(argv=None):
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.child:
        sys.exit(self_launch(sys.argv[1:] if argv is None else argv, args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args.gpus = world
    if args.workload is None:
        args.workload = "northstar" if world == 1 else "config4"

    traffic, pmc_note = None, "off"
    if not args.child and rank == 0 and world == 1 and args.pmc != "off":
        traffic, pmc_note = pmc_traffic(args)
        if traffic is None and args.pmc == "on":
            print(f"[bench] PMC collection failed: {pmc_note}", file=sys.stderr)

    import numpy as np
    import torch
    import torch.distributed as dist

    from hunddb_amd import crc, shard

    ndev = torch.cuda.device_count()
    local_dev = local % max(1, ndev)  # (rehearsal: ranks may share a GPU)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    backend = os.environ.get("HC_DIST_BACKEND", "nccl")
    if world > 1:
        # RCCL (backend "nccl") over xGMI; HC_DIST_BACKEND=gloo rehearses the
        # N>1 path with several ranks sharing one GPU.  Bounded: a rank that
        # never arrives ends init (and every later collective) with an error.
        import datetime
        phase("init")
        tmo = datetime.timedelta(seconds=args.rank_timeout if args.rank_timeout > 0 else 1800)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world, timeout=tmo)
    phase("fill")

    nblk, bsize, scaling = WORKLOADS[args.workload]
    if args.blocks:
        nblk = args.blocks
    scatter_in = args.input == "scatter" and world > 1 and scaling == "strong" and isinstance(bsize, int)
    if args.input == "scatter" and not scatter_in:
        raise SystemExit("--input scatter needs --gpus N > 1 and a uniform strong-scaling workload (config4)")
    full, scatter_s = None, None
    if scaling == "strong":  # one global batch, partitioned by block index
        lo, hi = shard.index_range(nblk, world, rank)
        total_blocks = nblk
    else:  # every rank owns its own full-size shard: global blocks rank*n .. rank*n+n-1
        lo, hi = nblk * rank, nblk * (rank + 1)
        total_blocks = nblk * world
    my = hi - lo
    counts = [shard.index_range(nblk, world, r)[1] - shard.index_range(nblk, world, r)[0]
              if scaling == "strong" else nblk for r in range(world)]
    stream = torch.cuda.current_stream()

    sample = None  # (host blocks, off, lens) for the CPU baseline
    out_sel = None  # the sample's entries of the GPU words (a permuted batch), else its first len(off)
    if bsize == "mixed":
        sizes = mixed_sizes(SEED, lo, my)
        off = np.zeros(my, dtype=np.uint64)
        off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
        total = int(off[-1]) + int(sizes[-1])
        doff = torch.from_numpy(off.view(np.int64)).to(dev)
        dlen = torch.from_numpy(sizes.view(np.int32)).to(dev)
        buf = torch.empty(total, dtype=torch.uint8, device=dev)
        crc.dev_fill_range(buf, SEED, lo, my, off=doff, lens=dlen)
        kw = dict(off=doff, lens=dlen, nblocks=my)
        step_bytes = total
        block_desc = "mixed 4/8/16 KiB, off/len arrays"
        k = int(np.searchsorted(off, 512 << 20))
        sample = (slice(0, int(off[k - 1]) + int(sizes[k - 1])), off[:k].copy(), sizes[:k].copy())
    elif bsize == "offlen4k":
        buf = torch.empty(my * 4096, dtype=torch.uint8, device=dev)
        crc.dev_fill_range(buf, SEED, lo, my, stride=4096, ulen=4096)
        doff = torch.arange(my, dtype=torch.int64, device=dev) * 4096
        dlen = torch.full((my,), 4096, dtype=torch.int32, device=dev)
        kw = dict(off=doff, lens=dlen, nblocks=my)
        step_bytes = my * 4096
        block_desc = "4096 B via off/len arrays"
        k = min(my, (512 << 20) // 4096)
        sample = (slice(0, k * 4096), np.arange(k, dtype=np.uint64) * 4096, np.full(k, 4096, np.uint32))
    elif bsize == "frame":
        npay = my * 4092 - 1000  # ragged last block
        rawn = (npay + 1 + (1 << 20) - 1) >> 20 << 20  # filled as 1 MiB blocks (one block of 4 GB is one wave's work)
        raw = torch.empty(rawn, dtype=torch.uint8, device=dev)
        crc.dev_fill_range(raw, SEED, lo << 20, rawn >> 20, stride=1 << 20, ulen=1 << 20)
        buf = raw[1:npay + 1]  # payload at an odd address
        dst = torch.empty(my * 4096, dtype=torch.uint8, device=dev)
        kw = None
        step_bytes = npay + my * 4096  # one read of the payload + one write of the blocks
        block_desc = "AddCRCsToData: 4092-B payload slices -> 4096-B stamped blocks"
    elif bsize == "verify":
        B = 8192
        buf = torch.empty(my * B, dtype=torch.uint8, device=dev)
        crc.dev_fill_range(buf, SEED, lo, my, stride=B, ulen=B)
        crc.dev_crc32_blocks(buf, None, stride=B, ulen=B, nblocks=my, flags=crc.HC_F_STAMP)
        bitmap = torch.empty((my + 31) // 32, dtype=torch.int32, device=dev)
        first_bad = torch.empty(1, dtype=torch.int64, device=dev)
        crc.dev_verify_prepare(bitmap, first_bad, my)  # all clean: nothing to reset per step
        kw = dict(stride=B, ulen=B, nblocks=my, bad_bitmap=bitmap, first_bad=first_bad)
        step_bytes = my * (B + 4)
        block_desc = "8192 B, verify mode (stamped; B read + 4 B written per block)"
        k = min(my, (512 << 20) // B)
        sample = (slice(0, k * B), np.arange(k, dtype=np.uint64) * B, np.full(k, B, np.uint32))
    elif bsize in ("records", "records_gapped", "records_shuffled"):
        lens_h = record_sizes(my) if not args.blocks else record_sizes(nblk)[:my]
        gap = 17 if bsize == "records_gapped" else 0
        off_h = np.zeros(my, dtype=np.uint64)
        off_h[1:] = np.cumsum(lens_h[:-1].astype(np.uint64) + np.uint64(gap), dtype=np.uint64)
        off_h += np.uint64(1 + gap)  # back to back (or 17 B apart) from an odd address
        total = (int(off_h[-1]) + int(lens_h[-1]) + 64 + (1 << 20) - 1) >> 20 << 20
        k = int(np.searchsorted(off_h, 512 << 20))
        sample = (slice(0, int(off_h[k - 1]) + int(lens_h[k - 1])), off_h[:k].copy(), lens_h[:k].copy())
        if bsize == "records_shuffled":  # the same records, listed in a permuted order
            perm = np.random.default_rng(SEED).permutation(my)
            off_h, lens_h = off_h[perm], lens_h[perm]
            sel = np.flatnonzero(off_h < np.uint64(512 << 20))  # the sample: the records of its first 512 MiB
            sample = (sample[0], off_h[sel].copy(), lens_h[sel].copy())
            out_sel = sel
        buf = torch.empty(total, dtype=torch.uint8, device=dev)
        crc.dev_fill_range(buf, SEED, lo << 20, total >> 20, stride=1 << 20, ulen=1 << 20)
        doff = torch.from_numpy(off_h.view(np.int64)).to(dev)
        dlen = torch.from_numpy(lens_h.view(np.int32)).to(dev)
        kw = dict(off=doff, lens=dlen, nblocks=my, flags=crc.HC_F_MESSAGES)
        step_bytes = int(lens_h.sum(dtype=np.uint64)) + 4 * my
        block_desc = ("GetCRC per record: log-uniform 64 B - 64 KiB records " +
                      ("with a 17-B gap before each" if gap else "back to back") +
                      (", listed in a permuted order" if bsize == "records_shuffled" else "") + " (off/len arrays)")
    elif bsize == "records4k_shuffled":
        buf = torch.empty(my * 4096, dtype=torch.uint8, device=dev)
        crc.dev_fill_range(buf, SEED, lo, my, stride=4096, ulen=4096)
        perm = np.random.default_rng(SEED).permutation(my).astype(np.uint64)
        off_h = perm * np.uint64(4096)
        lens_h = np.full(my, 4096, dtype=np.uint32)
        doff = torch.from_numpy(off_h.view(np.int64)).to(dev)
        dlen = torch.from_numpy(lens_h.view(np.int32)).to(dev)
        kw = dict(off=doff, lens=dlen, nblocks=my, flags=crc.HC_F_MESSAGES)
        step_bytes = my * 4096 + 4 * my
        block_desc = "GetCRC per record: aligned 4 KiB records in shuffled order (off/len arrays)"
        k = min(my, (512 << 20) // 4096)
        sample = (slice(0, my * 4096), off_h[:k].copy(), lens_h[:k].copy())
    elif bsize in UNFRAME_B:
        UB = UNFRAME_B[bsize]
        buf = torch.empty(my * UB, dtype=torch.uint8, device=dev)
        crc.dev_fill_range(buf, SEED, lo, my, stride=UB, ulen=UB)
        crc.dev_crc32_blocks(buf, None, stride=UB, ulen=UB, nblocks=my, flags=crc.HC_F_STAMP)
        dst = torch.empty(my * (UB - 4), dtype=torch.uint8, device=dev)
        bitmap = torch.empty((my + 31) // 32, dtype=torch.int32, device=dev)
        first_bad = torch.empty(1, dtype=torch.int64, device=dev)
        crc.dev_verify_prepare(bitmap, first_bad, my)
        kw = "unframe"
        step_bytes = my * UB + my * (UB - 4)  # one read of the blocks + one write of the payload
        block_desc = f"ReadFromDisk: verify {UB}-B blocks + strip CRCs"
    else:
        if scatter_in:
            # the batch starts on rank 0's GPU: its shards go out by RCCL send/recv
            if rank == 0:
                full = torch.empty(total_blocks * bsize, dtype=torch.uint8, device=dev)
                crc.dev_fill_range(full, SEED, 0, total_blocks, stride=bsize, ulen=bsize)
            bnd = [shard.index_range(nblk, world, r)[0] * bsize for r in range(world)] + [nblk * bsize]
            torch.cuda.synchronize()
            dist.barrier()
            ts = time.perf_counter()
            buf = shard.scatter_from_root(full, bnd, device=dev)
            torch.cuda.synchronize()
            dist.barrier()
            scatter_s = time.perf_counter() - ts
        else:
            buf = torch.empty(my * bsize, dtype=torch.uint8, device=dev)
            crc.dev_fill_range(buf, SEED, lo, my, stride=bsize, ulen=bsize)
        kw = dict(stride=bsize, ulen=bsize, nblocks=my)
        step_bytes = my * bsize
        block_desc = f"{bsize} B"
        k = min(my, (512 << 20) // bsize)
        sample = (slice(0, k * bsize), np.arange(k, dtype=np.uint64) * bsize, np.full(k, bsize, np.uint32))
    out = torch.empty(my, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def make_step(b, o, kw_):
        def step():
            if kw_ is None:
                crc.dev_add_crcs(b, dst, crc_out=o, stream=stream)
            elif kw_ == "unframe":
                crc.dev_read_blocks(b, UB, out=dst, crc_out=o, bad_bitmap=bitmap, first_bad=first_bad,
                                    stream=stream)
            else:
                crc.dev_crc32_blocks(b, o, stream=stream, **kw_)
        return step

    def timed(step, steps, warmup, barrier):
        """Clock settle + warmup (untimed), then `steps` launches bracketed by a
        barrier + synchronize on both sides; per-launch HIP events on the
        launch stream.  Returns (wall seconds, mean launch seconds)."""
        # memory-bound launches of ~1 ms right after the fill run below the
        # sustained clock (MI355X_MICROARCH.md "DVFS give-back")
        t_settle = time.perf_counter()
        while time.perf_counter() - t_settle < args.settle:
            for _ in range(8):
                step()
            torch.cuda.synchronize()
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        per_step = args.kernel_events == "step"
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps if per_step else 1)]
        if barrier:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if per_step:
            for i in range(steps):
                ev[i][0].record(stream)
                step()
                ev[i][1].record(stream)
        else:  # one pair around the K launches: the mean includes the gaps between them
            ev[0][0].record(stream)
            for i in range(steps):
                step()
            ev[0][1].record(stream)
        torch.cuda.synchronize()
        if barrier:
            dist.barrier()
        dt = time.perf_counter() - t0
        kern_ms = [a.elapsed_time(b) for a, b in ev]
        return dt, sum(kern_ms) / (steps if not per_step else len(kern_ms)) / 1e3

    step = make_step(buf, out, kw)
    phase("timed")
    dt, mean_kern_s = timed(step, args.steps, args.warmup, world > 1)
    phase("report")
    proof = None
    if world > 1:  # which device every rank really ran on, and its own kernel time
        proof = shard.device_proof(shard.gather_identities(shard.rank_identity(dev, mean_kern_s * 1e3)), backend)
        if backend == "nccl" and proof["distinct_devices"] != world:
            raise RuntimeError(f"{world} RCCL ranks ran on {proof['distinct_devices']} distinct GPU(s): "
                               f"{[(i['rank'], i['host'], i['bus_id']) for i in proof['ranks']]}")
    info = crc.last_launch()
    seg_mode = crc.seg_path() if args.workload in SEG_WORKLOADS else False
    verify_clean = None
    if bsize == "verify":  # every stamped block must have verified clean
        verify_clean = int(first_bad.item()) == 2**63 - 1 and int(bitmap.abs().sum().item()) == 0
        if not verify_clean:
            print("[bench] verify workload reported a bad block", file=sys.stderr)

    # max-over-ranks clock, summed bytes (all-reduce of 3 scalars, after the timed region)
    dt, mean_kern_s, all_bytes = shard.job_timing(dt, mean_kern_s, float(step_bytes), device=dev)
    job_bytes = all_bytes * args.steps

    if args.child:
        if world > 1:
            dist.destroy_process_group()
        return

    # CRC words to rank 0 (RCCL all-gather of 4 B per block), then the same
    # global batch on ONE GPU for the strong-scaling speedup and a word check
    multi = None
    if world > 1:
        phase("gather")
        torch.cuda.synchronize()
        tg = time.perf_counter()
        gathered = shard.gather_crcs(out, counts)
        gather_s = time.perf_counter() - tg
        ref1 = args.ref1 == "on" or (args.ref1 == "auto" and scaling == "strong")
        if rank == 0:
            multi = {"gathered_words": int(gathered.numel()), "gather_ms": round(gather_s * 1e3, 3),
                     "input": args.input, **proof}
            if scatter_s is not None:
                moved = total_blocks * bsize - counts[0] * bsize
                multi.update({"scatter_ms": round(scatter_s * 1e3, 3), "scatter_bytes": moved,
                              "scatter_gb_s": round(moved / scatter_s / 1e9, 2),
                              "scatter_note": "rank 0 -> every other rank, RCCL send/recv grouped; outside the "
                                              "timed CRC region (SURVEY.md 8e)"})
            if ref1 and isinstance(kw, dict) and "stride" in kw and scaling == "strong":
                phase("ref1")
                del step, buf, out  # the shard (the step closure holds it too)
                torch.cuda.empty_cache()
                if full is None:  # (scatter input: rank 0 still holds the whole batch)
                    full = torch.empty(total_blocks * bsize, dtype=torch.uint8, device=dev)
                    crc.dev_fill_range(full, SEED, 0, total_blocks, stride=bsize, ulen=bsize)
                outf = torch.empty(total_blocks, dtype=torch.int32, device=dev)
                t1, k1 = timed(make_step(full, outf, dict(stride=bsize, ulen=bsize, nblocks=total_blocks)),
                               args.steps, args.warmup, False)
                same = bool(torch.equal(gathered.to(dev), outf))
                multi.update({
                    "ref_1gpu_ms_per_step": round(t1 / args.steps * 1e3, 4),
                    "ref_1gpu_gib_s": round(total_blocks * bsize * args.steps / t1 / 2**30, 2),
                    "speedup_vs_1gpu": round((t1 / args.steps) / (dt / args.steps), 3),
                    "words_match_1gpu": same,
                    "words_check": f"all {total_blocks} gathered CRC words == rank 0's 1-GPU run of the same "
                                   f"global batch",
                })
                del full, outf
                if not same:
                    print("[bench] gathered CRC words differ from the 1-GPU run", file=sys.stderr)
        phase("final_barrier")
        dist.barrier()

    if rank == 0:
        gib_s = job_bytes / dt / 2**30
        achieved = step_bytes / mean_kern_s / 1e9  # algorithmic bytes per launch / launch time
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else round(traffic["bytes"]),
                "traffic_ratio": None if traffic is None else round(traffic["bytes"] / step_bytes, 4),
                "kernel": bytes_kernel(info["kernel"], seg_mode), "dispatch": info["kernel"],
                "bytes_per_launch": step_bytes,
                "mean_launch_ms": round(mean_kern_s * 1e3, 4),
                "launch_timing": ("HIP events on the launch stream around the K timed launches; mean = span / K "
                                  "(includes the gaps between launches)" if args.kernel_events == "bracket"
                                  else "HIP events on the launch stream around every timed launch"),
                "frac_vs_copy_ceiling": round(achieved / COPY_CEILING_GBS, 4),
                "copy_ceiling_note": "guide's measured float4 copy, 6.29 TB/s read+write; a read stream can exceed it",
                **({"launch_note": "one dispatch = k_seg_plan + k_seg_stream + k_seg_combine (+ the gated "
                                   "k_crc_grp launch for >= 2^18 records); `kernel` is the one the stream's mode "
                                   "word gave the bytes to (stream_mode)"}
                   if args.workload in SEG_WORKLOADS else {}),
                **({"traffic_by_kernel": traffic["by_kernel"]} if traffic else {}),
                "traffic_note": (f"PMC FETCH_SIZE*2*1024 + WRITE_SIZE*1024 per dispatch, summed over every kernel "
                                 f"it launches (fetch {traffic['fetch_bytes']:.4g} B, write "
                                 f"{traffic['write_bytes']:.4g} B)" if traffic else f"null: {pmc_note}")}
        host_leg = None
        if world == 1 and (args.host_leg == "on" or (args.host_leg == "auto" and args.workload == "northstar")):
            phase("host_leg")
            # the WAL image scales with a reduced --blocks run (2M records at the full 1M blocks)
            host_leg = host_inclusive(torch, crc, buf, out, bsize,
                                      wal_records=max(1000, min(2_000_000, 2 * my)))
        cpu = None
        if not args.cpu_threads:
            args.cpu_threads = cores_available()
        if world == 1 and args.cpu_seconds > 0:
            with pinned(args.cpu_threads) as pin:
                if bsize == "frame" or bsize in UNFRAME_B:
                    cpu = cpu_baseline_framing("frame" if bsize == "frame" else "unframe", buf, args.cpu_threads,
                                               args.cpu_seconds, B=UNFRAME_B.get(bsize, 4096))
                elif sample is not None:
                    sl, soff, slen = sample
                    host = buf[sl].cpu().numpy()
                    gw = out.cpu().numpy().view(np.uint32)
                    gw = gw[out_sel] if out_sel is not None else gw[: len(soff)]
                    cpu = cpu_baseline(host, soff, slen, args.cpu_threads, args.cpu_seconds,
                                       f"{args.workload} ({block_desc})", gpu_words=gw,
                                       messages=bsize in ("records", "records_gapped", "records4k_shuffled",
                                                          "records_shuffled"))
            if cpu is not None:
                cpu.update(pin.info())
        res = {
            "metric": METRIC,
            "value": round(gib_s, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 keyed by global block index, generated in HBM)",
            "config": {"workload": args.workload, "blocks_total": total_blocks, "blocks_per_gpu": my,
                       "block_bytes": block_desc, "bytes_per_gpu_step": step_bytes,
                       "parallelism": f"shard-by-block-index x{world}",
                       "dist_backend": backend if world > 1 else None,
                       "hbm_frac_of_8TBps": round(job_bytes / dt / world / 1e12 / 8.0, 4),
                       **({"verify_clean": verify_clean} if verify_clean is not None else {}),
                       **({"packed_stream_taken": seg_mode not in ("fallback", "fallback_grp"), "stream_mode": seg_mode}
                          if seg_mode is not False else {})},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if host_leg is not None:
            res["host_inclusive"] = host_leg
        res["workload_note"] = WORKLOAD_NOTE
        if multi is not None:
            res["multi_gpu"] = multi
            if "speedup_vs_1gpu" in multi:
                res["speedup_vs_1gpu"] = multi["speedup_vs_1gpu"]
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    phase("done")
    if world > 1:
        dist.destroy_process_group()


def _run():
    """main(), and on any exception ONE JSON error line naming the rank, then a
    non-zero exit (never a re-exec, never a silent partial line).  Under the
    self-launcher the rank records the error with its phase instead, and the
    launcher prints the one line for the whole job."""
    try:
        main()
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        rank = int(os.environ.get("RANK", "0"))
        msg = f"rank {rank}: {type(e).__name__}: {e}"
        from hunddb_amd import shard
        if os.environ.get(shard.PHASE_ENV):
            shard.report_phase("error", error=msg)
        else:
            print(json.dumps({"metric": METRIC, "value": None, "error": msg, "rank": rank,
                              "world_size": int(os.environ.get("WORLD_SIZE", "1"))}), flush=True)
        sys.exit(3)


if __name__ == "__main__":
    _run()
