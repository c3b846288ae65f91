#!/usr/bin/env python3
"""Time the device generator of the reference stream against the host generator."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parallel_kd_tree_amd as pk  # noqa: E402
from parallel_kd_tree_amd.ops import native  # noqa: E402

n, dim = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000, 3
dev = torch.device("cuda:0")
out = torch.empty((n, dim), dtype=torch.float32, device=dev)
native().generate_gpu(42, 0, out)  # warm (charpoly + jump polynomials cached)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    native().generate_gpu(42, 0, out)
torch.cuda.synchronize()
gpu_ms = (time.perf_counter() - t0) / 3 * 1e3
t0 = time.perf_counter()
host = pk.generate_slice(42, dim, 0, n)
host_ms = (time.perf_counter() - t0) * 1e3
same = torch.equal(out.cpu(), host)
S, C, R = native().devgen_plan(n * dim)
print(f"generate {n} x {dim}: device {gpu_ms:.2f} ms ({n * dim / gpu_ms / 1e6:.2f} G draws/s), host {host_ms:.1f} ms, "
      f"chunks {C} x {S} draws, {R} jump rounds, bit-identical {same}", flush=True)
