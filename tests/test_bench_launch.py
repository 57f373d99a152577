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


@pytest.mark.parametrize("world", [2, 3])
def test_self_launch_strong_scaling_words(world):
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
