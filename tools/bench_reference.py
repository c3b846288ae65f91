#!/usr/bin/env python3
"""Reference-mode GPU build (csrc/gpu/build_reference.hip: the reference's own tree by per-level
rank selection, tie-checked) against the exact builder, same points, warm timings. Usage: bench_reference.py [--n 10000000 ...] [--dim 3]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import parallel_kd_tree_amd as pk  # noqa: E402
from parallel_kd_tree_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[10_000_000])
ap.add_argument("--dim", type=int, default=3)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
dev = torch.device("cuda:0")


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / args.reps


for n in args.n:
    x = pk.generate_slice(42, args.dim, 0, n, device=dev)
    rb = ops.ReferenceTreeBuilder(n, args.dim)
    eb = ops.GpuTreeBuilder(n, args.dim, 0, 0)
    ref_ms = timed(lambda: rb.build(x, None, 1))
    exact_ms = timed(lambda: eb.build(x, None, 1))
    print(json.dumps({"n": n, "dim": args.dim, "reference_ms": round(ref_ms, 3), "exact_ms": round(exact_ms, 3),
                      "global_levels": rb._b.global_levels, "sorted_levels": rb._b.sorted_levels,
                      "ties": rb.read_ties()}), flush=True)
