#!/usr/bin/env python3
"""Achievable HBM bandwidth reference: torch copy of 1.6 GB (4 columns x 100M fp32)."""
import time

import torch

n = 400_000_000
a = torch.empty(n, device="cuda").uniform_()
b = torch.empty_like(a)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    b.copy_(a)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 10
print(f"copy 1.6 GB: {dt * 1e3:.3f} ms, {2 * n * 4 / dt / 1e12:.2f} TB/s (read + write)")
t0 = time.perf_counter()
for _ in range(10):
    s = a.sum()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 10
print(f"read 1.6 GB: {dt * 1e3:.3f} ms, {n * 4 / dt / 1e12:.2f} TB/s")
