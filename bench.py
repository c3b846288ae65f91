#!/usr/bin/env python3
"""Headline benchmark: Mpoints/sec kd-tree build, 100M x 3D float32 (BASELINE.json).

One step = one complete exact kd-tree build of the whole point set, from the input points
resident in HBM to the finished implicit in-order tree (ids + coordinates) in HBM.

* N = 1: the level-synchronous HIP builder on one MI355X.
* N > 1: global decomposition over RCCL (one process per GPU, torchrun env): each rank holds
  its generation-order slice (the reference's MPI slicing, kdtree_mpi.cpp:204-224); the top
  log2(N) levels are split with allreduced histograms, points are redistributed with one
  all-to-all, and each GPU builds its subtree. Strong scaling: the total point count is
  fixed, so `value` is the whole-job throughput.

Data: the reference generator stream (std::mt19937 + uniform_real<float>(-100,100), seed 42),
each rank's slice generated on its own GPU by the device generator (csrc/gpu/generator.hip,
bit-identical to the host stream; untimed).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_MPTS = 100e6 / 924.3 / 1e6  # reference build, 100M x 3D, 924.3 s (1 core)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--data", choices=["reference", "reference-host", "device"], default="reference",
                    help="reference: the reference stream generated on the GPU (bit-identical to the host "
                         "generator); reference-host: same stream generated on the host; device: torch RNG")
    ap.add_argument("--profile-levels", action="store_true", help="print per-phase timings to stderr")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("bench.py --gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
    # Rehearsal knobs for a one-GPU box (never set by the driver): PKD_BENCH_SHARE_GPU=1 puts
    # every rank on cuda:0 and PKD_BENCH_BACKEND=gloo replaces RCCL, which refuses two ranks
    # on one device. The timing is then meaningless; the control flow is the real one.
    if os.environ.get("PKD_BENCH_SHARE_GPU") == "1":
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from parallel_kd_tree_amd.parallel import comm
    if world > 1:
        comm.init(backend=os.environ.get("PKD_BENCH_BACKEND", "nccl"), device=dev)
    if rank == 0 and os.environ.get("PKD_SKIP_BUILD") != "1":
        from parallel_kd_tree_amd import _build
        _build.build()  # no-op when the in-tree extension is up to date
    if world > 1:
        comm.barrier()
    import parallel_kd_tree_amd as pk

    n, dim = args.points, args.dim
    if world > 1:
        from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
        first, count = comm.forest_slice(n, world, rank)
    else:
        first, count = 0, n

    if args.data == "reference":
        x = pk.generate_slice(args.seed, dim, first, count, device=dev)
    elif args.data == "reference-host":
        x = pk.generate_slice(args.seed, dim, first, count).to(dev)
    else:
        x = pk.uniform_points(count, dim, seed=args.seed * 1000 + rank, device=dev)
    ids = None

    if world > 1:
        builder = GlobalTreeBuilder(n, dim, device=dev)
        step = lambda: builder.build(x, id_base=first + 1)
    else:
        from parallel_kd_tree_amd.ops import GpuTreeBuilder
        b = GpuTreeBuilder(n, dim)
        out_pts = torch.empty_like(x)
        out_ids = torch.empty(n, dtype=torch.int32, device=dev)
        step = lambda: b.build(x, ids, 1, out_pts, out_ids)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        comm.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = comm.max_float(dt)
    # the device error word of the last build (outside the timed region)
    err = builder.read_error() if world > 1 else b.read_error()
    if err:
        sys.exit(f"bench.py: rank {rank}: device build reported error flags {err}")
    ms = dt * 1e3 / args.steps
    mpts = n / (ms / 1e3) / 1e6
    if rank == 0:
        print(json.dumps({
            "metric": "Mpoints/sec kd-tree build, 100M x 3D float32, at 1/2/4/8 MI355X",
            "value": round(mpts, 3),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(mpts / BASELINE_MPTS, 1),
            "dtype": "fp32",
            "data": f"synthetic: reference generator stream (mt19937 seed {args.seed}, uniform(-100,100))"
                    if args.data.startswith("reference") else "synthetic: on-device uniform(-100,100), reference value map",
            "config": {"model": "exact median-split kd-tree, cycling axis (implicit in-order layout)",
                       "global_batch": n, "seq_len": dim, "n_points": n, "dim": dim,
                       "parallelism": f"global{world}" if world > 1 else "single"},
        }), flush=True)
    if world > 1:
        comm.destroy()


if __name__ == "__main__":
    main()
