"""Run-to-run spread of device ReadFromDisk (k_unframe) across processes:
one process = one allocation of the blocks and the payload buffer, the
buffers' device addresses printed beside the rate (is the spread tied to
where the buffers land?).  Usage: python tools/unf_var.py <block bytes> <nblk> <reps>"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hunddb_amd import crc  # noqa: E402

UB, n, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dev = torch.device("cuda:0")
buf = torch.empty(n * UB, dtype=torch.uint8, device=dev)
crc.dev_fill_range(buf, 1234, 0, n, stride=UB, ulen=UB)
crc.dev_crc32_blocks(buf, None, stride=UB, ulen=UB, nblocks=n, flags=crc.HC_F_STAMP)
dst = torch.empty(n * (UB - 4), dtype=torch.uint8, device=dev)
o = torch.empty(n, dtype=torch.int32, device=dev)
bm = torch.empty((n + 31) // 32, dtype=torch.int32, device=dev)
fb = torch.empty(1, dtype=torch.int64, device=dev)
crc.dev_verify_prepare(bm, fb, n)
s = torch.cuda.current_stream()
for _ in range(50):
    crc.dev_read_blocks(buf, UB, out=dst, crc_out=o, bad_bitmap=bm, first_bad=fb, stream=s)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(s)
for _ in range(reps):
    crc.dev_read_blocks(buf, UB, out=dst, crc_out=o, bad_bitmap=bm, first_bad=fb, stream=s)
b.record(s)
torch.cuda.synchronize()
ms = a.elapsed_time(b) / reps
gbs = n * (2 * UB - 4) / ms / 1e6
print(f"UB {UB} src {buf.data_ptr():#x} dst {dst.data_ptr():#x} d-s {(dst.data_ptr() - buf.data_ptr()) / 2**20:.1f} MiB "
      f"ms {ms:.4f} GB/s {gbs:.1f} frac {gbs / 8000:.4f} clean {int(fb.item()) == 2**63 - 1}", flush=True)
