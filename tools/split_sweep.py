#!/usr/bin/env python3
"""Split-build sweep: (split level, parts, streams) against the one-stream build.

Every configuration's tree is compared slot for slot with the unsplit tree (the exact tree is
unique), then timed. The knobs are read when a builder is constructed, so one process can
sweep them (PKD_SPLIT*, see csrc/gpu/build_global.hip split_cfg).
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
ap.add_argument("--n", type=int, nargs="+", default=[100_000_000])
ap.add_argument("--dim", type=int, nargs="+", default=[3])
ap.add_argument("--cfg", nargs="+", default=["2,4,4", "2,4,2", "4,16,4", "4,8,4", "4,16,8", "6,16,4"],
                help="level,parts,streams")
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--min-n", type=int, default=None, help="PKD_SPLIT_MIN_N for the split builders")
ap.add_argument("--graph", action="store_true", help="also time a hipGraph replay of each build")
args = ap.parse_args()
dev = torch.device("cuda:0")


def host_ms(b, x, tp, ti):
    """Host time to enqueue one build (no synchronisation inside)."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b.build(x, None, 0, tp, ti)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) * 1e3


def graph_ms(b, x, tp, ti, steps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        b.build(x, None, 0, tp, ti)  # warm: side streams exist before the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.build(x, None, 0, tp, ti)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def timed(b, x, tp, ti, steps):
    b.build(x, None, 0, tp, ti)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        b.build(x, None, 0, tp, ti)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


for dim in args.dim:
    for n in args.n:
        x = pk.uniform_points(n, dim, seed=7, device=dev)
        os.environ["PKD_SPLIT"] = "0"
        b0 = GpuTreeBuilder(n, dim)
        rp, ri = b0.build(x)
        ms0 = timed(b0, x, rp, ri, args.steps)
        extra = {"host_ms": round(host_ms(b0, x, rp, ri), 3)}
        if args.graph:
            extra["graph_ms"] = round(graph_ms(b0, x, rp, ri, args.steps), 3)
        print(json.dumps({"n": n, "dim": dim, "cfg": "unsplit", "ms": round(ms0, 3), "err": b0.read_error(), **extra}),
              flush=True)
        del b0
        os.environ["PKD_SPLIT"] = "1"
        os.environ["PKD_AB"] = "1"  # the PKD_SPLIT_* sweep knobs are A/B knobs
        if args.min_n is not None:
            os.environ["PKD_SPLIT_MIN_N"] = str(args.min_n)
        for cfg in args.cfg:
            lv, parts, streams = cfg.split(",")
            os.environ["PKD_SPLIT_LEVEL"], os.environ["PKD_SPLIT_PARTS"], os.environ["PKD_SPLIT_STREAMS"] = lv, parts, streams
            b = GpuTreeBuilder(n, dim)
            desc = b.describe().splitlines()[0]
            tp, ti = b.build(x)
            torch.cuda.synchronize()
            err = b.read_error()
            same = bool(torch.equal(ti, ri)) and bool(torch.equal(tp, rp))
            ms = timed(b, x, tp, ti, args.steps)
            same2 = bool(torch.equal(ti, ri))
            extra = {"host_ms": round(host_ms(b, x, tp, ti), 3)}
            if args.graph:
                extra["graph_ms"] = round(graph_ms(b, x, tp, ti, args.steps), 3)
                extra["same_after_graph"] = bool(torch.equal(ti, ri))
            print(json.dumps({"n": n, "dim": dim, "cfg": cfg, "ms": round(ms, 3), "vs_unsplit": round(ms / ms0, 3),
                              "err": err, "same": same, "same_after_repeat": same2,
                              "split": "split at" in desc, **extra}), flush=True)
            if not (same and same2 and err == 0 and extra.get("same_after_graph", True)):
                print("MISMATCH", desc, flush=True)
                sys.exit(1)
            del b, tp, ti
        del x, rp, ri
        torch.cuda.empty_cache()
