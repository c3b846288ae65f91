#!/usr/bin/env python3
"""One rank of a P-rank global build, timed as a whole chain on one GPU (csrc/cpu/global_builder.cpp
emulate_rank): the P ranks run once as threads over the loopback communicator while rank `rank`
records its collective outputs; then that rank alone rebuilds against a replay communicator
(stream-ordered device copies of the recorded outputs), profiled. Prints the phase JSON; the
exchange there is a device copy, so `chain_ex_exchange_ms` = total - exchange is the number to
compare with the single-GPU build of N / P points.
Usage: emulate_rank.py [--n 100000000] [--dim 3] [--P 8] [--rank 0] [--k -1] [--reps 5]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import parallel_kd_tree_amd as pk  # noqa: E402
from parallel_kd_tree_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--dim", type=int, default=3)
ap.add_argument("--P", type=int, default=8)
ap.add_argument("--rank", type=int, nargs="+", default=[0])
ap.add_argument("--k", type=int, default=-1)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--seed", type=int, default=42)
args = ap.parse_args()
torch.cuda.init()
x = pk.generate_slice(args.seed, args.dim, 0, args.n, device=torch.device("cuda:0")).cpu().contiguous()
for r in args.rank:
    d = ops.native().global_emulate_rank(x, args.P, r, args.k, args.reps)
    d = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items()}
    d["chain_ex_exchange_ms"] = round(d["total_ms"] - d["exchange_span_ms"], 4)
    print(json.dumps({"n": args.n, "dim": args.dim, "P": args.P, "rank": r, **d}), flush=True)
