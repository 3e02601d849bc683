"""Device -> page-locked host copy rate on this box (the link the Estimate results cross).
Usage: python scripts/pcie_probe.py"""
import torch

torch.cuda.init()
for mb in (4.65, 9.3, 18.6, 37.2):
    n = int(mb * 1e6) // 4
    d = torch.empty(n, dtype=torch.int32, device="cuda")
    h = torch.empty(n, dtype=torch.int32, pin_memory=True)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(10):
        s.record()
        h.copy_(d, non_blocking=True)
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e))
    print(f"D2H {mb:6.2f} MB: {best * 1e3:8.1f} us, {mb / best:6.1f} GB/s", flush=True)
