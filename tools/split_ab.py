#!/usr/bin/env python3
"""A/B/A/B timing of split-build variants (environment knobs read at builder construction /
per build), each tree checked against the one-stream build. Usage:
  split_ab.py --var unsplit:PKD_SPLIT=0 breadth:PKD_SPLIT_ORDER=breadth ... [--rounds 3]"""
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
ap.add_argument("--var", nargs="+", required=True, help="name:K=V,K=V")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--fresh", action="store_true", help="a new builder per measurement, destroyed after it")
ap.add_argument("--graph", action="store_true", help="time hipGraph replays of the build instead of eager builds")
args = ap.parse_args()
dev = torch.device("cuda:0")
x = pk.uniform_points(args.n, args.dim, seed=7, device=dev)
knobs = sorted({kv.split("=")[0] for v in args.var for kv in v.split(":", 1)[1].split(",") if kv})


def apply(spec):
    os.environ["PKD_AB"] = "1"  # the variants' knobs are A/B knobs
    for k in knobs:
        os.environ.pop(k, None)
    for kv in spec.split(","):
        if kv:
            k, v = kv.split("=")
            os.environ[k] = v


ref = None
res = {v.split(":")[0]: [] for v in args.var}
builders = {}
for r in range(args.rounds):
    for v in args.var:
        name, spec = v.split(":", 1)
        apply(spec)
        if name not in builders:
            b = GpuTreeBuilder(args.n, args.dim)
            tp, ti = b.build(x)
            torch.cuda.synchronize()
            if ref is None:
                ref = ti.clone()
            assert b.read_error() == 0 and torch.equal(ti, ref), f"{name}: tree differs"
            builders[name] = (b, tp, ti)
        b, tp, ti = builders[name]
        if args.fresh and r > 0:  # one builder (and its side streams) alive at a time
            b = GpuTreeBuilder(args.n, args.dim)
        b.build(x, None, 0, tp, ti)
        torch.cuda.synchronize()
        g = None
        if args.graph:
            cs = torch.cuda.Stream()
            cs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cs):
                b.build(x, None, 0, tp, ti)
            torch.cuda.current_stream().wait_stream(cs)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                b.build(x, None, 0, tp, ti)
            g.replay()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            if g is not None:
                g.replay()
            else:
                b.build(x, None, 0, tp, ti)
        torch.cuda.synchronize()
        del g
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        res[name].append(round(ms, 3))
        if args.fresh:
            assert b.read_error() == 0 and torch.equal(ti, ref), f"{name}: tree differs"
            builders[name] = (None, tp, ti)
            del b
            torch.cuda.synchronize()
        print(json.dumps({"round": r, "var": name, "ms": round(ms, 3)}), flush=True)
    for name, (_, tp, ti) in builders.items():
        assert torch.equal(ti, ref), f"{name}: tree differs after timing"
print(json.dumps({"summary": {k: {"min": min(v), "all": v} for k, v in res.items()}}), flush=True)
