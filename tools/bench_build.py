#!/usr/bin/env python3
"""Time single-GPU builds for several (n, dim, subtree_max) settings in one process and
check each result against the previous setting (the exact tree is unique)."""
import argparse
import json
import time

import torch
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd.ops import GpuTreeBuilder

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[10_000_000, 100_000_000])
ap.add_argument("--dim", type=int, nargs="+", default=[3])
ap.add_argument("--subtree", type=int, nargs="+", default=[0])
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--data", default="device")
args = ap.parse_args()
dev = torch.device("cuda:0")
for dim in args.dim:
    for n in args.n:
        if args.data == "device":
            x = pk.uniform_points(n, dim, seed=1, device=dev)
        else:
            x = pk.generate_problem(42, dim, n).to(dev)
        ref_ids = None
        for sm in args.subtree:
            b = GpuTreeBuilder(n, dim, 0, sm)
            tp, ti = b.build(x)
            torch.cuda.synchronize()
            err = b.read_error()
            same = None
            if ref_ids is not None:
                same = bool(torch.equal(ref_ids, ti))
            else:
                ref_ids = ti.clone()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                b.build(x, None, 0, tp, ti)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            if os.environ.get("PKD_SUBTREE_STAMPS"):
                from parallel_kd_tree_amd.ops import native
                print(native().subtree_stamp_report(), flush=True)
            if os.environ.get("PKD_TAIL_STAMPS"):
                from parallel_kd_tree_amd.ops import native
                print(native().tail_stamp_report(), flush=True)
            print(json.dumps({"n": n, "dim": dim, "subtree_max": b.subtree_max, "global_levels": b.global_levels,
                              "ms": round(ms, 3), "mpts_s": round(n / ms / 1e3, 1), "err": err, "same_as_first": same}),
                  flush=True)
        del x, ref_ids
        torch.cuda.empty_cache()
