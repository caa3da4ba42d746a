#!/usr/bin/env python3
"""Raw PCIe copy rates on this box (pinned host memory): H2D alone, D2H alone, both concurrently on two
streams.  Context for the host-resident e2e number of the engine."""
import time
import torch
n = 1 << 30
h1 = torch.empty(n, dtype=torch.uint8).pin_memory(); h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d1 = torch.empty(n, dtype=torch.uint8, device="cuda"); d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def t(f):
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter(); f(); torch.cuda.synchronize(); return time.perf_counter() - t0
def h2d():
    with torch.cuda.stream(s1): d1.copy_(h1, non_blocking=True)
def d2h():
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
def both():
    h2d(); d2h()
a, b, c = t(h2d), t(d2h), t(both)
print(f"H2D {n/a/1e9:.1f} GB/s  D2H {n/b/1e9:.1f} GB/s  concurrent {2*n/c/1e9:.1f} GB/s aggregate")
