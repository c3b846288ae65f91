#!/usr/bin/env python3
"""Native global builder on one rank with 2^k pipelined leaves: per-build time and the middle-bucket
all-gather scale (1 = no overflow retry) -- the distributed top levels' health check."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd.parallel.native_global import NativeGlobalBuilder
n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
x = pk.generate_slice(42, 3, 0, n, device=dev)
g = NativeGlobalBuilder(n, 3, dev, pipeline_k=k)
for i in range(4):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    g.build(x, 1)
    torch.cuda.synchronize()
    print(f"build {i}: {1e3 * (time.perf_counter() - t0):.3f} ms, scale {g._g.middle_scale()}, err {g.read_error()}", flush=True)
