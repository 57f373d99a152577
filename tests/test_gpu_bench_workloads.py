"""bench.py end to end on the GPU, every workload at a small size: one JSON
line whose roofline names the workload's kernel and whose algorithmic bytes
match the workload's definition.  The full-size
numbers are the bench runs under profiles/; this only checks that each
workload's path runs and is accounted for as documented."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# workload -> (blocks, kernel named in the roofline, bytes per launch for those blocks or None)
CASES = {
    "northstar": (4096, "k_crc_grp", 4096 * 8192),
    "verify": (4096, "k_crc_grp", 4096 * (8192 + 4)),
    "config2": (4096, "k_crc_grp", 4096 * 4096),
    "16k": (1024, "k_crc_grp", 1024 * 16384),
    "config3": (4096, "k_crc_grp+k_crc_any", None),
    "offlen4k": (4096, "k_crc_grp+k_crc_any", 4096 * 4096),
    "config4": (4096, "k_crc_grp", 4096 * 8192),
    "frame": (4096, "k_frame", (4096 * 4092 - 1000) + 4096 * 4096),
    "unframe": (4096, "k_unframe", 4096 * (4096 + 4092)),
    "unframe8k": (2048, "k_unframe", 2048 * (8192 + 8188)),
    "unframe16k": (1024, "k_unframe", 1024 * (16384 + 16380)),
    "records": (4096, "k_seg_stream", None),                 # packed: the stream did the bytes
    "records_gapped": (4096, "k_seg_stream", None),
    # >= HC_SEG_GRP_MIN (2^18) shuffled aligned records: the stream refuses them and the
    # gated k_crc_grp launch moves the bytes (name that kernel)
    "records4k_shuffled": (300_000, "k_crc_grp", 300_000 * (4096 + 4)),
    "records_shuffled": (4096, None, None),                   # unsorted records: the stream refuses them
    "blocks4092": (4096, "k_seg_stream", 4096 * 4092),        # the message stream (round 6; k_crc_any before)
    "blocks8188": (4096, None, 4096 * 8188),                  # the message stream (launch_seg_blocks)
}


@pytest.mark.gpu
@pytest.mark.parametrize("workload", sorted(CASES))
def test_bench_workload_small(workload):
    blocks, kernel, nbytes = CASES[workload]
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--blocks", str(blocks),
           "--steps", "2", "--warmup", "1", "--cpu-seconds", "0", "--pmc", "off", "--settle", "0",
           "--host-leg", "off" if workload != "northstar" else "on"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["config"]["workload"] == workload
    assert res["value"] > 0 and res["ms_per_step"] > 0
    roof = res["roofline"]
    assert roof["bound"] == "hbm" and roof["peak"] == 8000.0 and 0 < roof["frac"]
    if kernel:
        assert roof["kernel"] == kernel
    if nbytes:
        assert roof["bytes_per_launch"] == nbytes
    if workload == "verify":
        assert res["config"]["verify_clean"] is True
    if workload == "records4k_shuffled":
        assert res["config"]["stream_mode"] == "fallback_grp"
        assert roof["dispatch"].startswith("k_seg_plan")


@pytest.mark.gpu
def test_north_star_meets_its_target():
    """BASELINE.json's north star: >= 70 % of MI355X HBM peak for device-resident
    CRC32 over 1M x 8 KiB blocks, at full size (bench.py's HIP-event timing of
    k_crc_grp; 85-88 % on the boxes of round 4, profiles/r4/)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "northstar", "--steps", "10",
           "--warmup", "3", "--cpu-seconds", "0", "--pmc", "off", "--host-leg", "off"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["config"]["blocks_total"] == 1_000_000 and res["config"]["block_bytes"] == "8192 B"
    assert res["roofline"]["frac"] >= 0.70, res["roofline"]
