#!/usr/bin/env python3
"""Sampled top levels (csrc/gpu/top4.hpp) against the CPU exact builder and against the
paired-levels path (PKD_TOP=0), over sizes / dims / depth0 / duplicates; then timings.
Usage: top_check.py [--quick] [--time N ...]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PKD_AB", "1")  # PKD_TOP_MIN_N is an A/B knob
os.environ.setdefault("PKD_TOP_MIN_N", "0")
import torch  # noqa: E402

import parallel_kd_tree_amd as pk  # noqa: E402
from parallel_kd_tree_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--quick", action="store_true")
ap.add_argument("--time", type=int, nargs="*", default=[])
ap.add_argument("--dim", type=int, default=3)
args = ap.parse_args()
dev = torch.device("cuda:0")


def check(x, depth0=0, label=""):
    b = ops.GpuTreeBuilder(x.shape[0], x.shape[1], depth0, 0)
    t0 = time.perf_counter()
    tp, ti = b.build(x.to(dev))
    torch.cuda.synchronize()
    err = b.read_error_detail()
    cp, ci = ops.build_cpu(x, None, "exact", depth0, 8)
    same = torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)
    rep = b.top_band_report() if b.sampled_top else None
    print(json.dumps({"case": label, "n": x.shape[0], "dim": x.shape[1], "depth0": depth0, "sampled": b.sampled_top,
                      "err": err, "same": same, "bands": rep}), flush=True)
    return same and err[0] == 0


ok = True
cases = [(200_000, 3, 0), (300_001, 2, 0), (1_000_003, 3, 1), (500_000, 5, 2), (400_000, 8, 0), (2_000_000, 4, 3)]
if args.quick:
    cases = cases[:2]
for n, d, d0 in cases:
    ok &= check(pk.generate_problem(n + d, d, n), d0, "uniform")
ok &= check(torch.randint(0, 7, (400_000, 3)).float(), 0, "dups7")
ok &= check(torch.randint(0, 1000, (600_000, 3)).float(), 1, "dups1000")
xs = pk.generate_problem(9, 3, 300_000)
xs = xs[torch.argsort(xs[:, 0])].contiguous()
ok &= check(xs, 0, "sorted-x")
print("ALL_OK" if ok else "FAILED", flush=True)

for n in args.time:
    x = pk.generate_slice(42, args.dim, 0, n, device=dev)
    for top in ("1", "0"):
        os.environ["PKD_TOP"] = top
        b = ops.GpuTreeBuilder(n, args.dim, 0, 0)
        tp, ti = b.build(x, None, 1)
        torch.cuda.synchronize()
        for _ in range(2):
            b.build(x, None, 1, tp, ti)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            b.build(x, None, 1, tp, ti)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        if top == "1":
            ref = ti.clone()
            e = b.read_error_detail()
        else:
            same = torch.equal(ref, ti)
        print(json.dumps({"n": n, "dim": args.dim, "top": top, "ms": round(ms, 3), "sampled": b.sampled_top,
                          "err": b.read_error_detail(), **({"same": same} if top == "0" else {})}), flush=True)
    os.environ["PKD_TOP"] = "1"
