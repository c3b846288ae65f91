#!/usr/bin/env python3
"""Timing of the sampled top pass's pieces (PKD_TOP_DIAG, no tree built): the full build, the
build stopped after the scatter (diag 1), and the scatter without its reservation atomics
(diag 2), for several scatter grids (PKD_TOP_BLOCKS). Usage: top_diag.py [N] [blocks ...]"""
import json
import os
import sys
import time

os.environ["PKD_AB"] = "1"  # PKD_TOP_DIAG / PKD_TOP_BLOCKS are A/B knobs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import parallel_kd_tree_amd as pk  # noqa: E402
from parallel_kd_tree_amd.ops import GpuTreeBuilder  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
blocks = [int(b) for b in sys.argv[2:]] or [0]
x = pk.generate_slice(42, 3, 0, n, device=torch.device("cuda:0"))


def timed(env, reps=10):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        b = GpuTreeBuilder(n, 3, 0, 0)
        tp, ti = b.build(x, None, 1)
        torch.cuda.synchronize()
        for _ in range(2):
            b.build(x, None, 1, tp, ti)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            b.build(x, None, 1, tp, ti)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / reps
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


for bl in blocks:
    r = {"n": n, "blocks": bl}
    for name, env in (("full", {}), ("to_scatter", {"PKD_TOP_DIAG": 1}), ("to_scatter_noatomic", {"PKD_TOP_DIAG": 2}),
                      ("scatter_nostore", {"PKD_TOP_DIAG": 3})):
        env = dict(env, PKD_TOP_BLOCKS=bl)
        r[name] = round(timed(env), 3)
    print(json.dumps(r), flush=True)
r = {"n": n, "pairs_build": round(timed({"PKD_TOP": 0}), 3)}
print(json.dumps(r), flush=True)
