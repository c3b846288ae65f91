#!/usr/bin/env python3
"""Warm timing of the exact 1-NN kernels on one GPU: brute force and traversal over the
reference generator's points (default: the reference's eval config, 500k x 128D, 10 queries)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parallel_kd_tree_amd as pk  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=500_000)
ap.add_argument("--dim", type=int, default=128)
ap.add_argument("--queries", type=int, default=10)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda:0")
x = pk.generate_slice(42, args.dim, 0, args.n + args.queries, device=dev)
tree = pk.KDTree.build(x[:args.n], id_base=1)
q = x[args.n:].contiguous()
res = {"n": args.n, "dim": args.dim, "queries": args.queries}
from parallel_kd_tree_amd import ops  # noqa: E402
nat = ops.native()
out = {}
# traversal at high dimension visits every node from one thread per query (as the reference's
# search does at d=128): only timed where it is the right method
methods = ("brute", "traverse") if args.dim <= 16 else ("brute",)
for method in methods:
    for _ in range(3):
        out[method] = tree.query_packed(q, method)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        tree.query_packed(q, method)
    torch.cuda.synchronize()
    res[method + "_ms"] = round((time.perf_counter() - t0) * 1e3 / args.reps, 4)
    # device time of the kernel alone (events around a pre-initialised output, no allocation)
    into = torch.empty(q.shape[0], dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        into.fill_(-1)
        tree.query_packed(q, method, into)
    e1.record()
    torch.cuda.synchronize()
    res[method + "_dev_ms"] = round(e0.elapsed_time(e1) / args.reps, 4)
if "traverse" in out:
    res["same"] = bool(torch.equal(out["brute"], out["traverse"]))
print(json.dumps(res), flush=True)
