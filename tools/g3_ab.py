#!/usr/bin/env python3
"""A/B of the sampled triples (k_g3_*) in one process: knob sets (A/B env variables, read when a
builder is constructed) x sizes; per run the build time, the tree checked against the first
setting's (the exact tree is unique), the error word and, from g3_report(), the staged fraction
of the last sampled triple (rows the sample could not place / rows)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parallel_kd_tree_amd as pk  # noqa: E402
from parallel_kd_tree_amd.ops import GpuTreeBuilder  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[100_000_000, 12_500_000])
ap.add_argument("--dim", type=int, default=3)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--reps", type=int, default=1, help="rounds over the sets (interleaved, median reported)")
ap.add_argument("--sets", nargs="+", default=["PKD_G3=0", ""],
                help="knob sets, each 'K=V,K=V' ('' = defaults)")
args = ap.parse_args()
dev = torch.device("cuda:0")
os.environ["PKD_AB"] = "1"
for n in args.n:
    x = pk.uniform_points(n, args.dim, seed=1, device=dev)
    ref = None
    times = {ks: [] for ks in args.sets}
    for ks in [k for _ in range(args.reps) for k in args.sets]:
        kv = dict(p.split("=", 1) for p in ks.split(",") if p)
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        b = GpuTreeBuilder(n, args.dim, 0, 0)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        tp, ti = b.build(x)
        b.build(x, None, 0, tp, ti)
        torch.cuda.synchronize()
        err = b.read_error()
        same = None
        if ref is None:
            ref = ti.clone()
        else:
            same = bool(torch.equal(ref, ti))
        t0 = time.perf_counter()
        for _ in range(args.steps):
            b.build(x, None, 0, tp, ti)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        times[ks].append(ms)
        rep = b.g3_report()
        staged = None
        if rep is not None:
            lvl, segs = rep
            tot = sum(s[0] for s in segs)
            st = [sum(s[1 + t] for s in segs) for t in range(7)]
            staged = {"level": lvl, "frac": round(sum(st) / max(1, tot), 4),
                      "by_tag": [round(v / max(1, tot), 4) for v in st], "bad": sum(s[24] for s in segs)}
        print(json.dumps({"n": n, "dim": args.dim, "set": ks or "default", "ms": round(ms, 3), "err": err,
                          "same_as_first": same, "g3": " g3" in b.describe(), "staged": staged}), flush=True)
        del b
    if args.reps > 1:
        for ks, v in times.items():
            v = sorted(v)
            print(json.dumps({"n": n, "dim": args.dim, "set": ks or "default", "median_ms": round(v[len(v) // 2], 3),
                              "all_ms": [round(t, 3) for t in v]}), flush=True)
    del x, ref, tp, ti
    torch.cuda.empty_cache()
