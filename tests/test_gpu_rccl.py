"""RCCL (torch.distributed backend "nccl") on the GPU box: the collectives
bench.py issues at N > 1 -- shard.gather_crcs's all_gather of the CRC words and
shard.job_timing's float64 MAX/SUM all-reduces -- run over a real RCCL
communicator, with the HIP path hashing the shard.  The box has one GPU, so the
group has one rank (RCCL refuses two ranks on one device); the gloo tests
(tests/test_shard.py, tests/test_bench_launch.py) cover 2-3 ranks."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_gather_and_reduce_one_rank(cuda, oracle):
    from hunddb_amd import shard
    n = 3001
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(shard.free_port()))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_rccl_rank.py"), str(n)],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["kernel"] == "k_crc_grp"
    assert res["gathered_device"].startswith("cuda")  # all_gather ran on device tensors
    assert res["max"] == [1.5, 2.5] and res["sum"] == float(n)
    p = res["proof"]  # bench.py's multi_gpu proof fields, gathered over RCCL
    assert p["comm_world_size"] == 1 and p["distinct_devices"] == 1 and p["rehearsal"] is False
    assert p["backend"] == "nccl" and p["rccl_version"] and not p["rccl_version"].startswith("unknown")
    r0 = p["ranks"][0]
    assert r0["rank"] == 0 and r0["device"] == 0 and r0["kernel_ms"] == 1.25
    assert r0["hc_devices"] >= 1 and len(r0["bus_id"].split(":")) == 3
    B = 8192
    host, _, _ = oracle.fill_blocks(0x5EED, n, B)
    want = oracle.crc32_blocks(host, stride=B, ulen=B)
    assert np.array_equal(np.asarray(res["words"], dtype=np.uint32), want)
