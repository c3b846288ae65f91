"""Python CLI with the reference protocol, single process or one rank per GPU (torchrun).

    python -m parallel_kd_tree_amd.cli [--decomp single|forest|global] [--mode exact|reference]
                                       [--device cuda|cpu] [SEED DIM_POINTS NUM_POINTS]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m parallel_kd_tree_amd.cli --decomp global 42 3 100000000

With no positional arguments rank 0 prints READY, reads the seed from stdin and uses dim=128,
N=500000 (Utility.cpp:92-102); the config is broadcast to every rank (kdtree_mpi.cpp:199).
forest reproduces kdtree_mpi.cpp (independent per-rank trees + MIN reduction), global builds
one distributed tree (parallel/global_tree.py). Only rank 0 prints.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch


def _all_ok(comm, err: int, device) -> None:
    """Raise on every rank if any rank's build reported a device error (no rank prints
    results from a corrupt tree, and none is left waiting in a collective)."""
    flags = torch.tensor([1 if err else 0], dtype=torch.int64, device=device)
    comm.all_reduce_(flags)
    if err:
        raise RuntimeError(f"rank {comm.rank()}: GPU kd-tree build reported device error word {err:#x}")
    if int(flags[0]):
        raise RuntimeError("another rank's GPU kd-tree build reported a device error")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="parallel_kd_tree_amd.cli", add_help=True)
    ap.add_argument("--decomp", choices=["single", "forest", "global"], default=None)
    ap.add_argument("--mode", choices=["exact", "reference"], default="exact")
    ap.add_argument("--device", choices=["cuda", "cpu"], default=None)
    ap.add_argument("--pipeline-k", type=int, default=-1,
                    help="--decomp global: extra distributed top levels (more, smaller leaf builds; -1: auto)")
    ap.add_argument("--query", choices=["auto", "brute", "traverse"], default="auto")
    ap.add_argument("--queries", type=int, default=10)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--host-gen", action="store_true", help="generate the data on the host (default on a GPU: "
                                                            "the bit-identical device generator)")
    ap.add_argument("--metrics-json", action="store_true")
    ap.add_argument("--save", default=None, help="write the built tree (PKDTREE file); forest: one file per rank "
                    "(<path>.rank<r>), global: the assembled tree from rank 0")
    ap.add_argument("--leaf-threshold", type=int, default=0,
                    help="largest segment finished by the LDS subtree kernel (0 = auto from dim)")
    ap.add_argument("--ranks", type=int, default=0,
                    help="--decomp forest: logical forest ranks (the reference's mpirun -np R, Makefile:36) spread "
                         "over the processes; 0 = one per process")
    ap.add_argument("positional", nargs="*")
    a = ap.parse_args(argv)
    tick = time.perf_counter()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_type = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    device = torch.device("cuda", local_rank) if dev_type == "cuda" else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    decomp = a.decomp or ("forest" if world > 1 else "single")

    from .parallel import comm
    if world > 1:
        comm.init(backend="nccl" if device.type == "cuda" else "gloo", device=device)
    from .utils import protocol
    debug = a.debug or bool(a.positional) or os.environ.get("KDTREE_DEBUG", "0") not in ("", "0")
    cfg = [0, 0, 0]
    if rank == 0:
        if debug:
            cfg = list(protocol.specify_problem_argv(sys.argv[0], a.positional))
        else:
            cfg = list(protocol.specify_problem_stdin())
    if world > 1:
        cfg = comm.broadcast_ints(cfg)
    seed, dim, n = cfg
    Q = a.queries

    import parallel_kd_tree_amd as pk
    from . import ops
    t_gen = time.perf_counter()
    if decomp == "single":
        first, cnt = 0, n
    else:
        first, cnt = comm.forest_slice(n, world, rank)
    R = a.ranks or world
    if R != world and decomp != "forest":
        raise SystemExit("--ranks applies to --decomp forest")
    gen_dev = device if (device.type == "cuda" and not a.host_gen) else None
    x = pk.generate_slice(seed, dim, first, cnt, device=gen_dev).to(device) if R == world else None
    q = pk.generate_slice(seed, dim, n, Q, device=gen_dev).to(device)
    if device.type == "cuda":
        torch.cuda.synchronize()
    t_build = time.perf_counter()
    if decomp == "single":
        tree = pk.KDTree.build(x, id_base=1, mode=a.mode, subtree_max=a.leaf_threshold)
        from .parallel.global_tree import _local_packed
        packed = _local_packed(tree, q, a.query)
        tree.check()  # device error word, read after the queries are enqueued
        if a.save:
            tree.save(a.save)
    elif decomp == "forest":
        from .parallel.forest import ForestTree, forest_min_packed, logical_ranks
        # R logical ranks over the processes (R = world: one each, the reference's mpirun -np P)
        trees = []
        for lr in logical_ranks(R, world, rank):
            f0, c0 = comm.forest_slice(n, R, lr)
            xs = x if R == world else pk.generate_slice(seed, dim, f0, c0, device=gen_dev).to(device)
            trees.append((lr, ForestTree.build(xs, f0, n, id_base=1, mode=a.mode)))
        packed = forest_min_packed([t for _, t in trees], q, a.query)
        err = 0
        for _, t in trees:
            err |= t.local_error()
        _all_ok(comm, err, device)
        if a.save:
            for lr, t in trees:
                t.local.save(f"{a.save}.rank{lr}")
    else:
        if a.mode != "exact":
            raise SystemExit("--decomp global builds exact trees only")
        if device.type == "cuda":  # the native builder on its own RCCL communicator
            from .parallel.native_global import NativeGlobalBuilder
            gb = NativeGlobalBuilder(n, dim, device, pipeline_k=a.pipeline_k)
        else:  # host tensors over gloo: the same schedule in torch
            from .parallel.global_tree import GlobalTreeBuilder
            gb = GlobalTreeBuilder(n, dim, device=device, pipeline_k=a.pipeline_k)
        t = gb.build(x, id_base=first + 1)
        packed = t.query_packed(q, a.query)
        _all_ok(comm, gb.read_error() if device.type == "cuda" else 0, device)
        if a.save:
            tp, ti = t.gather_full()
            if rank == 0:
                pk.KDTree(tp.cpu(), ti.cpu(), 0, "exact").save(a.save)
    if device.type == "cuda":
        torch.cuda.synchronize()
    t_done = time.perf_counter()
    dist_sq = ops.unpack(packed.cpu())[0]
    d = ops.query.sqrt_exact(dist_sq).numpy()
    if rank == 0:
        lines = [protocol.result_line(n + i, float(np.float32(d[i]))) for i in range(Q)]
        print("\n".join(lines), flush=True)
        if debug:
            print(f"elapsed time {time.perf_counter() - tick:g} second", flush=True)
        print("DONE", flush=True)
        if a.metrics_json:
            print(json.dumps({"decomp": decomp, "ranks": world, "gen_ms": (t_build - t_gen) * 1e3,
                              "build_query_ms": (t_done - t_build) * 1e3}), file=sys.stderr, flush=True)
    if world > 1:
        comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
