#!/usr/bin/env python3
"""Reference-mode GPU build (csrc/gpu/build_reference.hip: the reference's own tree by per-level
rank selection, tie-checked) against the exact builder, same points, warm timings; then the END-TO-END
reference mode a user gets (ops.build_reference_gpu_checked: the GPU tree plus the host repair of the
tied subtrees and their ancestors' sorts), and the host std::sort builder (threaded, and single-threaded
up to --single-max points) for comparison. Usage: bench_reference.py [--n 10000000 ...] [--dim 3]"""
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
ap.add_argument("--single-max", type=int, default=1_000_000)
ap.add_argument("--seed", type=int, default=42)
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
    x = pk.generate_slice(args.seed, args.dim, 0, n, device=dev)
    rb = ops.ReferenceTreeBuilder(n, args.dim)
    eb = ops.GpuTreeBuilder(n, args.dim, 0, 0)
    ref_ms = timed(lambda: rb.build(x, None, 1))
    exact_ms = timed(lambda: eb.build(x, None, 1))
    import warnings
    from parallel_kd_tree_amd.ops.build import cpu_threads
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        e2e_ms = timed(lambda: ops.build_reference_gpu_checked(x, None, 1))
        _, ti_h, _ = ops.build_reference_gpu_checked(x, None, 1)
    slots = rb.read_tie_slots()
    ties = rb.read_ties()
    xh = x.cpu()
    ids = (torch.arange(n) + 1).to(torch.int32)
    t0 = time.perf_counter()
    _, ci = ops.build_cpu(xh, ids, "reference", 0, cpu_threads())
    host_mt_ms = (time.perf_counter() - t0) * 1e3
    host_1_ms = None
    if n <= args.single_max:
        t0 = time.perf_counter()
        ops.build_cpu(xh, ids, "reference", 0, 1)
        host_1_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"n": n, "dim": args.dim, "seed": args.seed, "reference_gpu_ms": round(ref_ms, 3),
                      "exact_ms": round(exact_ms, 3), "ties": ties, "tie_slots": len(slots),
                      "end_to_end_ms": round(e2e_ms, 3), "end_to_end_equals_host_tree": bool(torch.equal(ti_h.cpu(), ci)),
                      "host_threads": cpu_threads(), "host_threaded_ms": round(host_mt_ms, 1),
                      "host_single_thread_ms": None if host_1_ms is None else round(host_1_ms, 1),
                      "global_levels": rb._b.global_levels, "sorted_levels": rb._b.sorted_levels}), flush=True)
