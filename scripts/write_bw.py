"""Measure the device's streaming write bandwidth (torch fill_ and memset) on
a buffer the size of the config-B packed distance output (2.7 GB fp64)."""
import time
import torch

n = 26000 * 25999 // 2
x = torch.empty(n, dtype=torch.float64, device="cuda")
for name, fn in [("fill_", lambda: x.fill_(1.5)), ("zero_", lambda: x.zero_())]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name}: {ms:.3f} ms  {n * 8 / ms / 1e9:.2f} TB/s", flush=True)
y = torch.empty_like(x)
for _ in range(2):
    y.copy_(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    y.copy_(x)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(f"copy: {ms:.3f} ms  {2 * n * 8 / ms / 1e9:.2f} TB/s (read+write)", flush=True)
