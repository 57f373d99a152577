"""bench.py --gpus N without torchrun: the self-launcher starts N ranks with the
torch.distributed.run environment before touching the GPU, rank 0 prints one
line, and the ranks' gathered CRC words (one global batch split by block index,
filled by global index) equal a single-process run of the whole batch.  gloo
on CPU; the per-GPU kernel is replaced by the oracle in tests/bench_cpu_rank.py."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_self_launch_strong_scaling_words(world):
    """world 8 is the size of the driver's scaling run (Next 4): 8
    ranks spawned, an 8-row device table, one JSON line."""
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.self_launch(['--blocks', '3001', '--gpus', '%d'], %d, "
            "script=%r))" % (ROOT, world, world, os.path.join(ROOT, "tests", "bench_cpu_rank.py")))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == world and res["scaling"] == "strong"
    assert sum(res["counts"]) == 3001 and res["bytes"] == 3001 * 4096
    assert res["words_match_1proc"] is True
    # the multi_gpu proof fields bench.py prints at N > 1 (hunddb_amd.shard.device_proof)
    m = res["multi_gpu"]
    assert [r["rank"] for r in m["ranks"]] == list(range(world))
    assert len({r["pid"] for r in m["ranks"]}) == world
    assert all(r["kernel_ms"] is not None and r["bus_id"] == "cpu" for r in m["ranks"])
    assert m["comm_world_size"] == world and m["backend"] == "gloo" and m["rccl_version"] is None
    assert m["kernel_ms_min"] <= m["kernel_ms_max"]
    # every rank on one host and no GPU: flagged as a rehearsal, not an N-GPU run
    assert m["distinct_devices"] == 1 and m["rehearsal"] is True and "rehearsal" in m["rehearsal_note"]


def test_device_proof_distinct_devices():
    """distinct_devices counts (host, PCI address) pairs: N ranks on N GPUs is
    not a rehearsal; two ranks on one GPU, or one address on two hosts' ranks
    seen as the same host, are."""
    from hunddb_amd import shard
    ids = [{"rank": r, "host": "h", "bus_id": f"0000:{0x11 + r:02x}:00", "kernel_ms": 1.0 + r} for r in range(8)]
    p = shard.device_proof(ids, "gloo")
    assert p["distinct_devices"] == 8 and p["rehearsal"] is False and "rehearsal_note" not in p
    assert (p["kernel_ms_min"], p["kernel_ms_max"]) == (1.0, 8.0)
    ids[3]["bus_id"] = ids[2]["bus_id"]
    p = shard.device_proof(ids, "gloo")
    assert p["distinct_devices"] == 7 and p["rehearsal"] is True


def test_bench_error_line_names_the_rank():
    """Any exception in a bench rank ends in ONE JSON error line naming the
    rank, and a non-zero exit."""
    code = ("import sys, os; sys.path.insert(0, %r); import bench; "
            "bench.main = lambda: (_ for _ in ()).throw(ValueError('boom')); bench._run()" % ROOT)
    env = dict(os.environ, RANK="2", WORLD_SIZE="4")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 3
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["rank"] == 2 and res["value"] is None and res["error"] == "rank 2: ValueError: boom"


def test_cpu_baseline_reports_cores_it_used(oracle):
    """cpu_baseline's `cores` is the thread count it timed, cores_available is
    the affinity set capped by the cgroup quota, and the spread is reported
    against the median."""
    import numpy as np

    import bench
    n, B = 2000, 4096
    buf = np.random.default_rng(1).integers(0, 256, n * B, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * B
    lens = np.full(n, B, dtype=np.uint32)
    threads = bench.cores_available()
    assert threads == min(len(os.sched_getaffinity(0)), int(bench.cgroup_cpu_quota() or 1 << 30))
    res = bench.cpu_baseline(buf, off, lens, threads, 0.5, "test",
                             gpu_words=oracle.crc32_blocks(buf, stride=B, ulen=B))
    assert res["cores"] == threads == res["cores_available"]
    assert res["logical_cpus"] == os.cpu_count() and res["affinity_cpus"] == len(os.sched_getaffinity(0))
    lo, hi = res["spread_pct"]
    assert lo <= 0.0 <= hi and res["matches_gpu"] is True
    assert "nproc" not in res
    # rates per CPU second of the pinned threads, the wall clock beside them
    assert len(res["slices"]) == len(res["slices_busy"]) == len(res["wall_clock"]["slices"]) == bench.N_SLICES
    assert all(0.0 < b <= 1.5 for b in res["slices_busy"])
    wlo, whi = res["wall_clock"]["spread_pct"]
    assert wlo <= 0.0 <= whi and res["wall_clock"]["value"] > 0
    assert "cache-resident" in res["sample"] and "listed" in res["sample"]


def test_self_launch_parent_never_imports_torch_cuda():
    """The launching process must not initialise the GPU (no exec after HIP
    init on this pool): bench.self_launch only imports hunddb_amd.shard."""
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "rc = bench.self_launch(['--help'], 1, script=%r); "
            "assert 'torch' not in sys.modules, 'parent imported torch'; sys.exit(rc)"
            % (ROOT, os.path.join(ROOT, "bench.py")))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]


def test_spawn_ranks_propagates_failure():
    from hunddb_amd import shard
    rc = shard.spawn_ranks([sys.executable, "-c",
                            "import os, sys, time; r = int(os.environ['RANK']); "
                            "time.sleep(0.2); sys.exit(7 if r == 1 else 0)"], 3)
    assert rc == 7


def _launch(world, extra_args, env_extra, timeout):
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.self_launch(%r, %d, script=%r))"
            % (ROOT, ["--blocks", "3001", "--gpus", str(world)] + extra_args, world,
               os.path.join(ROOT, "tests", "bench_cpu_rank.py")))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    import time
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines, time.monotonic() - t0


def test_self_launch_deadline_names_the_hung_rank():
    """the first 8-GPU run gets a deadline.  World 4, rank 2
    sleeps 120 s in its timed phase, --rank-timeout 20: the launcher kills the
    ranks and prints ONE JSON error line naming the ranks still alive and their
    last phase, and exits non-zero, within 30 s of the deadline's start."""
    r, lines, dt = _launch(4, ["--rank-timeout", "20"], {"HC_BENCH_STALL": "2:timed:120"}, 120)
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["value"] is None and res["reason"] == "timeout" and res["n_gpus"] == 4
    assert "deadline" in res["error"] and res["failed_ranks"] == []
    alive = {a["rank"]: a for a in res["alive_ranks"]}
    assert alive[2]["phase"] == "timed" and alive[2]["phase_age_s"] >= 10
    assert set(alive) == {0, 1, 2, 3}  # the others wait for rank 2 in a collective
    assert dt < 20 + 30, dt


def test_self_launch_failed_rank_is_named():
    """A rank that raises ends the job at once: its peers are killed, and the
    one JSON line names the failed rank, its phase and its error."""
    r, lines, dt = _launch(4, ["--rank-timeout", "120"], {"HC_BENCH_FAIL": "1:fill"}, 180)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["reason"] == "rank_failed" and res["value"] is None
    first = res["failed_ranks"][0]
    assert first["rank"] == 1 and first["phase"] == "error" and "HC_BENCH_FAIL at fill" in first["error"]
    assert res["error"].startswith("rank 1")
    assert dt < 90, dt
