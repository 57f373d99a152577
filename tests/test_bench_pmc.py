"""bench.py's PMC accounting for multi-kernel dispatches:
roofline.traffic sums every kernel a timed dispatch launches, and
roofline.kernel names the kernel the stream's mode word gave the bytes to.
Pure host logic on synthetic rocprofv3 counter rows (no GPU)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(bench)

NS = "void hc::(anonymous namespace)::"


def rows(seq):
    return [{"Kernel_Name": NS + k + "(unsigned char const*, unsigned long)", "Counter_Value": str(v)} for k, v in seq]


def test_dispatch_traffic_sums_the_dispatch_kernels():
    steps = 3
    seq = [("k_fill", 1e6), ("k_crc_grp<false, true>", 777.0)]  # setup: the fill and a stamp launch
    for i in range(steps + 1):  # warmup + timed
        seq += [("k_seg_plan<14u>", 10 + i), ("k_seg_stream<14u>", 5.0), ("k_seg_combine<14u>", 2.0),
                ("k_crc_grp<true, false>", 1000.0 + i)]
    got = bench.dispatch_traffic(rows(seq), steps)
    assert set(got) == {"k_seg_plan<14u>", "k_seg_stream<14u>", "k_seg_combine<14u>", "k_crc_grp<true, false>"}
    assert got["k_seg_plan<14u>"] == (11 + 12 + 13) / 3  # the last `steps` rows: the timed dispatches
    assert got["k_crc_grp<true, false>"] == 1002.0


def test_setup_launch_of_the_timed_kernel_is_dropped():
    steps = 3
    seq = [("k_crc_grp<false, true>", 5000.0)] + [("k_crc_grp<false, true>", 100.0)] * (steps + 1)
    assert bench.dispatch_traffic(rows(seq), steps) == {"k_crc_grp<false, true>": 100.0}


def test_bytes_kernel_follows_the_stream_mode():
    seg = "k_seg_plan+k_seg_stream+k_seg_combine"
    assert bench.bytes_kernel(seg, "fallback_grp") == "k_crc_grp"
    assert bench.bytes_kernel(seg, "packed") == "k_seg_stream"
    assert bench.bytes_kernel(seg, "gapped") == "k_seg_stream"
    assert bench.bytes_kernel(seg, "gapped_wide") == "k_seg_stream"
    assert bench.bytes_kernel(seg, "fallback") == "k_seg_combine"
    assert bench.bytes_kernel(seg, "sorted_packed") == "k_seg_stream"  # the sort ran in the stream kernel
    assert bench.bytes_kernel("k_crc_any", "fallback") == "k_crc_any"  # not a stream dispatch
    assert bench.bytes_kernel("k_crc_grp", False) == "k_crc_grp"


def test_quiet_cores_pick_distinct_physical_cores():
    """The CPU baseline pins itself to one logical CPU per physical core (VERDICT r5
    item 5: its slices spread -31 % unpinned on a shared host)."""
    n = min(2, len(os.sched_getaffinity(0)))
    cpus = bench.quiet_cores(n, sample_s=0.05)
    if cpus is None:
        return  # topology not readable here: the line then says "pinning": "none"
    assert len(cpus) == n and set(cpus) <= os.sched_getaffinity(0)
    cores = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        cores.add((open(base + "physical_package_id").read(), open(base + "core_id").read()))
    assert len(cores) == n
    before = os.sched_getaffinity(0)
    with bench.pinned(n) as p:
        assert os.sched_getaffinity(0) == set(p.cpus)
    assert os.sched_getaffinity(0) == before and p.info()["pinned_cpus"] == p.cpus
