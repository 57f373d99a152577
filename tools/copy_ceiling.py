"""Copy ceiling on this GPU for the framing kernels' footprint: torch's own
device-to-device copy of 4092 MB (aligned and from an odd source address),
timed with HIP events.  Prints GB/s of read+write bytes."""
import torch

n = 1_000_000 * 4092
src = torch.empty(n + 16, dtype=torch.uint8, device="cuda").random_(0, 256)
dst = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
for name, s, d in (("aligned", src[:n], dst[:n]), ("src+1", src[1:n + 1], dst[:n])):
    for _ in range(3):
        d.copy_(s)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        d.copy_(s)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    print(f"copy {name}: {ms:.3f} ms  {2 * n / ms / 1e6:.0f} GB/s (read+write)", flush=True)
