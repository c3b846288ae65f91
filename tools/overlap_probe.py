#!/usr/bin/env python3
"""Concurrency probe: do independent sub-builds on separate HIP streams overlap?

Times (one MI355X) a full n-point build against 2^k independent builds of n / 2^k points each
(separate builders and workspaces), issued on one stream or spread over S streams. If the
memory-bound partition passes of one sub-build overlap the LDS-bound subtree kernel of another,
the S-stream total is below the sum of the parts: the case for a split build after the top levels.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd.ops import GpuTreeBuilder

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--dim", type=int, default=3)
ap.add_argument("--parts", type=int, nargs="+", default=[2, 4, 8])
ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 4])
ap.add_argument("--steps", type=int, default=10)
args = ap.parse_args()
dev = torch.device("cuda:0")
x = pk.uniform_points(args.n, args.dim, seed=1, device=dev)
main = torch.cuda.current_stream()


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


full = GpuTreeBuilder(args.n, args.dim)
fp, fi = full.build(x)
ms_full = timed(lambda: full.build(x, None, 0, fp, fi), args.steps)
print(json.dumps({"case": "full", "n": args.n, "ms": round(ms_full, 3)}), flush=True)
del full, fp, fi
torch.cuda.empty_cache()

for parts in args.parts:
    m = args.n // parts
    xs = [x[i * m:(i + 1) * m] for i in range(parts)]
    bs = [GpuTreeBuilder(m, args.dim, 2) for _ in range(parts)]
    outs = [b.build(xi) for b, xi in zip(bs, xs)]
    torch.cuda.synchronize()
    for ns in args.streams:
        streams = [torch.cuda.Stream() for _ in range(ns)]

        def step():
            for s in streams:
                s.wait_stream(main)
            for i in range(parts):
                with torch.cuda.stream(streams[i % ns]):
                    bs[i].build(xs[i], None, 0, outs[i][0], outs[i][1])
            for s in streams:
                main.wait_stream(s)

        ms = timed(step, args.steps)
        print(json.dumps({"case": "split", "parts": parts, "streams": ns, "n_part": m, "ms": round(ms, 3),
                          "vs_full": round(ms / ms_full, 3)}), flush=True)
    del bs, outs, xs
    torch.cuda.empty_cache()
