"""Per-kernel dispatch cost on the box: N tiny dependent kernels back to back on one stream."""
import time
import torch

x = torch.zeros(64, device="cuda:0")
for n in (1000, 4000):
    for _ in range(50):
        x.add_(1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        x.add_(1.0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{n} tiny kernels: host {(t1 - t0) / n * 1e6:.2f} us/launch, wall {(t2 - t0) / n * 1e6:.2f} us/kernel",
          flush=True)
