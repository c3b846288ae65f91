#!/usr/bin/env python3
"""Headline benchmark: Mpoints/sec kd-tree build, 100M x 3D float32 (BASELINE.json).

One step = one complete exact kd-tree build of the whole point set, from the input points
resident in HBM to the finished implicit in-order tree (ids + coordinates) in HBM.

* N = 1: the level-synchronous HIP builder on one MI355X.
* N > 1: global decomposition over RCCL (one process per GPU, any N): each rank holds its
  generation-order slice (the reference's MPI slicing, kdtree_mpi.cpp:204-224); the top
  levels are split with allreduced histograms, points are redistributed with all-to-all
  rounds, and each GPU builds its leaves' subtrees (csrc/cpu/global_builder.cpp). Strong
  scaling: the total point count is fixed, so `value` is the whole-job throughput. After the
  timed loop rank 0 prints the per-phase breakdown of one extra (untimed, profiled) build on
  stderr -- top levels, pack, plan wait, exchange (bytes, GB/s), id rebuild, leaf builds --
  as the MAX over ranks.

Launch: under torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in the env), or
plain `python bench.py --gpus N`: without WORLD_SIZE the process becomes a launcher that never
touches a GPU, starts N child ranks (the reference's `mpirun -np P`, Makefile:36) and exits
with the first failing rank's status.

Data: the reference generator stream (std::mt19937 + uniform_real<float>(-100,100), seed 42),
each rank's slice generated on its own GPU by the device generator (csrc/gpu/generator.hip,
bit-identical to the host stream; untimed). After the timed loop (untimed) the last tree is
checked: device error word, kd invariant on every node, ids a permutation (N = 1: the error
words of EVERY timed build are folded on the device; a build whose sampled band missed is charged
its unsampled rebuild); at N > 1 also
every block of every rank against every top-tree pivot above it (cross-rank routing).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_MPTS = 100e6 / 924.3 / 1e6  # reference build, 100M x 3D, 924.3 s (1 core)
METRIC = "Mpoints/sec kd-tree build, 100M x 3D float32, at 1/2/4/8 MI355X"
HEADLINE = (100_000_000, 3)


def metric_name(n: int, dim: int) -> str:
    """The BASELINE metric for the headline config; other sizes are labelled as what they are."""
    if (n, dim) == HEADLINE:
        return METRIC
    size = f"{n // 1_000_000_000}B" if n % 1_000_000_000 == 0 else (
        f"{n // 1_000_000}M" if n % 1_000_000 == 0 else str(n))
    return f"Mpoints/sec kd-tree build, {size} x {dim}D float32 (not the headline config)"


def _parse(argv=None):
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
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: run the same control flow on host tensors over gloo (launcher / CI check; "
                         "timings meaningless)")
    ap.add_argument("--no-check", action="store_true", help="skip the untimed correctness check of the last tree")
    ap.add_argument("--decomp", choices=["auto", "single", "global"], default="auto",
                    help="auto: one GPU builds alone, N > 1 GPUs build one global tree; global also at N = 1 "
                         "(the multi-GPU code path on one rank)")
    ap.add_argument("--pipeline-k", type=int, default=-1,
                    help="global: extra top levels (leaves per rank = 2^k at power-of-two N; -1: auto)")
    ap.add_argument("--timeout", type=float, default=300.0,
                    help="global: bound of every host wait on the communicator (s); a stuck peer raises")
    ap.add_argument("--no-profile", action="store_true", help="N > 1: skip the per-phase breakdown build")
    return ap.parse_args(argv)


def _ensure_built(who: str) -> None:
    """Bring the in-tree extension / executables up to date (file-locked, no GPU involved).
    PKD_BENCH_TRACE_BUILD=1 reports on stderr what this process compiled and how long it took."""
    if os.environ.get("PKD_SKIP_BUILD") == "1":
        return
    from parallel_kd_tree_amd import _build
    _build.build()
    if os.environ.get("PKD_BENCH_TRACE_BUILD") == "1":
        lb = _build.LAST_BUILD
        what = ",".join(lb["compiled"]) if lb["compiled"] else "up to date"
        print(f"bench.py: {who}: build {what} ({lb['seconds'] * 1e3:.0f} ms)", file=sys.stderr, flush=True)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(nprocs: int, argv) -> int:
    """Start `nprocs` ranks of this script and wait for them. The launcher itself never
    initialises a GPU (no HIP call happens before the children exist). If a rank fails, the
    others are stopped (they would block in a collective) and its exit status is returned."""
    port = _free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            p.kill()
        raise
    for p in procs:
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc


def _check_tree(tp, ti, depth0, id_lo, id_hi, permutation=True) -> str:
    """'' when (tp, ti) is a valid exact kd-tree (on its device) whose ids are distinct and in
    [id_lo, id_hi) -- all of that range when `permutation`."""
    from parallel_kd_tree_amd import ops
    v = int(ops.native().invariant_violations(tp.contiguous(), ti.contiguous(), depth0))
    if v:
        return f"{v} kd-invariant violations"
    n = ti.numel()
    if n == 0:
        return "" if (not permutation or id_hi == id_lo) else "empty tree"
    idl = ti.to(torch.int64) & 0xFFFFFFFF
    if int(idl.min()) < id_lo or int(idl.max()) >= id_hi:
        return "ids out of range"
    seen = torch.zeros(id_hi - id_lo, dtype=torch.int32, device=ti.device)
    seen.index_add_(0, idl - id_lo, torch.ones_like(idl, dtype=torch.int32))
    if int(seen.max()) > 1:
        return "duplicate ids"
    if permutation and n != id_hi - id_lo:
        return f"{n} ids for {id_hi - id_lo} points"
    return ""


def _check_share(t, n: int) -> str:
    """'' when a rank's share of the distributed tree is valid: every block (complete subtree)
    satisfies the kd invariant from its own root depth, ids are distinct and in 1..n, and every
    block lies on the correct side of every top-tree pivot above it (cross-rank routing)."""
    for off, m, depth, _ in t.blocks:
        if m > 0:
            p = _check_tree(t.tree_pts[off:off + m], t.tree_ids[off:off + m], t.depth0 + depth, 1, n + 1,
                            permutation=False)
            if p:
                return p
    p = _distinct_ids(t.tree_ids, n) if t.tree_ids.numel() else ""
    return p or t.check_top_routing()


def _distinct_ids(ids, n: int) -> str:
    idl = ids.to(torch.int64) & 0xFFFFFFFF
    if int(idl.min()) < 1 or int(idl.max()) > n:
        return "ids out of range"
    seen = torch.zeros(n + 1, dtype=torch.int32, device=ids.device)
    seen.index_add_(0, idl, torch.ones_like(idl, dtype=torch.int32))
    return "duplicate ids" if int(seen.max()) > 1 else ""


def main(argv=None):
    args = _parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # the launcher never touches the GPU: it is the place to compile, before any rank exists
        # (a rank building while its peers wait in a collective could outlast their timeout)
        _ensure_built("launcher")
        sys.exit(launch(args.gpus, sys.argv[1:] if argv is None else argv))
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    share = os.environ.get("PKD_BENCH_SHARE_GPU") == "1"
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    cpu = args.device == "cpu"
    # Rehearsal knobs for a one-GPU box (never set by the driver): PKD_BENCH_SHARE_GPU=1 puts
    # every rank on cuda:0 and PKD_BENCH_BACKEND=gloo replaces RCCL, which refuses two ranks
    # on one device. The timing is then meaningless; the control flow is the real one.
    if cpu:
        dev = torch.device("cpu")
    else:
        if share:
            local_rank = 0
            # RCCL refuses two ranks on one device ("Duplicate GPU detected") unless they look
            # like different hosts: a per-rank host id makes every rank its own "node" and the
            # ranks talk over the loopback socket transport. The collectives, their grouping
            # and the builder's schedule are the real ones; only the transport differs from xGMI.
            os.environ.setdefault("NCCL_HOSTID", f"pkd-share-rank{rank}")
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)

    # Every rank checks the in-tree build BEFORE joining the communicator: under torchrun there
    # is no launcher of ours, so the first rank to take the build lock compiles (if anything is
    # stale) and the rest find the signatures up to date; nobody waits inside a collective.
    _ensure_built(f"rank {rank}")
    from parallel_kd_tree_amd.parallel import comm
    if world > 1:
        comm.init(backend="gloo" if cpu else os.environ.get("PKD_BENCH_BACKEND", "nccl"), device=dev)
        comm.barrier()
    if os.environ.get("PKD_BENCH_FAIL_RANK") == str(rank):  # launcher test: this rank dies, the rest block
        os._exit(7)
    import parallel_kd_tree_amd as pk

    n, dim = args.points, args.dim
    first, count = comm.forest_slice(n, world, rank) if world > 1 else (0, n)
    if args.data == "reference" and not cpu:
        x = pk.generate_slice(args.seed, dim, first, count, device=dev)
    elif args.data.startswith("reference"):
        x = pk.generate_slice(args.seed, dim, first, count).to(dev)
    else:
        x = pk.uniform_points(count, dim, seed=args.seed * 1000 + rank, device=dev)

    sync = (lambda: None) if cpu else torch.cuda.synchronize
    distributed = world > 1 or args.decomp == "global"
    if args.decomp == "single" and world > 1:
        sys.exit("bench.py: --decomp single needs --gpus 1")
    if world == 1 and distributed and cpu:
        sys.exit("bench.py: --decomp global on one rank runs the native builder (GPU)")
    builder = None
    if distributed:
        if not cpu:
            from parallel_kd_tree_amd.parallel.native_global import NativeGlobalBuilder
            builder = NativeGlobalBuilder(n, dim, dev, pipeline_k=args.pipeline_k, timeout_s=args.timeout)
            # bounded: a stuck or failed peer raises here instead of hanging the device sync
            sync = lambda: (builder.sync(), torch.cuda.synchronize())  # noqa: E731
        else:
            from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
            builder = GlobalTreeBuilder(n, dim, device=dev, pipeline_k=args.pipeline_k)
        res = {}

        def step():
            res["t"] = builder.build(x, id_base=first + 1)
    elif cpu:
        from parallel_kd_tree_amd import ops
        res = {}

        def step():
            res["t"] = ops.build_cpu(x, None, "exact", 0, os.cpu_count() or 1)
    else:
        from parallel_kd_tree_amd.ops import GpuTreeBuilder
        b = GpuTreeBuilder(n, dim)
        out_pts = torch.empty_like(x)
        out_ids = torch.empty(n, dtype=torch.int32, device=dev)
        # every timed build's error word, folded on the device (OR, builds with an error, builds
        # whose sampled bands missed): no host round trip per build, and no missed build goes
        # unnoticed (sample positions are salted per build, so a miss can hit any step)
        err_acc = torch.zeros(4, dtype=torch.int32, device=dev)

        def step():
            b.build(x, None, 1, out_pts, out_ids)
            b.accumulate_error(err_acc)

    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        comm.barrier()
    sync()
    if not distributed and not cpu:
        err_acc.zero_()
        sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    if world > 1:
        comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = comm.max_float(dt)

    # ---- untimed: the last build's tree must be right --------------------------------
    problem = ""
    if distributed:
        err = builder.read_error() if not cpu else 0
        t = res["t"]
        if err:
            problem = f"device build reported error flags {err}"
        elif not args.no_check:
            problem = _check_share(t, n)
            if not problem:
                idl = t.tree_ids.to(torch.int64) & 0xFFFFFFFF
                stats = torch.tensor([idl.numel(), int(idl.sum()) if idl.numel() else 0], dtype=torch.int64,
                                     device=dev)
                if world > 1:
                    comm.all_reduce_(stats)
                top_ids = [int(t.top_rows[i, dim:].contiguous().view(torch.int32).item()) & 0xFFFFFFFF
                           for i, s in enumerate(t.top_slots) if s >= 0]
                cnt, tot = int(stats[0]) + len(top_ids), int(stats[1]) + sum(top_ids)
                if not problem and (cnt != n or tot != n * (n + 1) // 2):
                    problem = f"the distributed tree holds {cnt} points (id sum {tot}) for ids 1..{n}"
    elif cpu:
        tp, ti = res["t"]
        problem = "" if args.no_check else _check_tree(tp, ti + 1, 0, 1, n + 1)
    else:
        acc = [int(v) & 0xFFFFFFFF for v in err_acc.tolist()]
        if acc[0] & ~GpuTreeBuilder.TOP_BAND_MISS:
            problem = (f"a timed build reported error flags {acc[0]:#x} ({acc[1]} of {args.steps} builds; last "
                       f"build's detail {b.read_error_detail()})")
        elif acc[2]:
            # A sampled band missed its median in `misses` timed builds: such a build stops at the
            # failed check and the user then pays an unsampled rebuild (ops.build_gpu_checked).
            # Charge that rebuild to the timing: one untimed warm-up, then one timed fallback build
            # per miss. The last tree checked is the rebuilt one when the last build missed.
            misses = acc[2]
            fb = GpuTreeBuilder(n, dim, allow_top=False)
            fb_pts, fb_ids = torch.empty_like(x), torch.empty(n, dtype=torch.int32, device=dev)
            fb.build(x, None, 1, fb_pts, fb_ids)
            sync()
            t1 = time.perf_counter()
            for _ in range(misses):
                fb.build(x, None, 1, fb_pts, fb_ids)
            sync()
            dt += time.perf_counter() - t1
            print(f"bench.py: {misses} of {args.steps} timed builds missed a sampled band; their unsampled "
                  f"rebuilds are included in the timing", file=sys.stderr, flush=True)
            if b.read_error() & GpuTreeBuilder.TOP_BAND_MISS:
                out_pts, out_ids = fb_pts, fb_ids
        if not problem and not args.no_check:
            problem = _check_tree(out_pts, out_ids, 0, 1, n + 1)
    if world > 1:
        bad = torch.tensor([1 if problem else 0], dtype=torch.int64, device=dev)
        comm.all_reduce_(bad)
        if int(bad[0]) and not problem:
            problem = "another rank's tree check failed"
    if problem:
        print(f"bench.py: rank {rank}: {problem}", file=sys.stderr, flush=True)
        if world > 1:
            comm.destroy()
        sys.exit(3)

    # ---- untimed: where one build's time goes (N > 1, native): one profiled build -------
    if distributed and not cpu and not args.no_profile:
        builder.set_profile(True)
        step()
        ph = builder.phases()
        builder.set_profile(False)
        keys = sorted(ph)
        v = torch.tensor([ph[k] for k in keys], dtype=torch.float64, device=dev)
        if world > 1:
            comm.all_reduce_(v, torch.distributed.ReduceOp.MAX)
        ph = dict(zip(keys, v.tolist()))
        if rank == 0:
            gbs = ph["sent_bytes"] / max(ph["exchange_ms"], 1e-9) / 1e6
            print(json.dumps({"phases_max_over_ranks_ms": {k: round(ph[k], 4) for k in keys if k.endswith("_ms")},
                              "exchange_sent_bytes_max": int(ph["sent_bytes"]),
                              "exchange_max_peer_bytes": int(ph["max_peer_bytes"]),
                              "exchange_GBps_per_rank": round(gbs, 2), "rounds": int(ph["rounds"]),
                              "top_levels": builder.top_levels, "retries": int(ph["retries"])}),
                  file=sys.stderr, flush=True)

    ms = dt * 1e3 / args.steps
    mpts = n / (ms / 1e3) / 1e6
    misses = int(err_acc[2]) if (not distributed and not cpu) else 0
    if rank == 0:
        metric = metric_name(n, dim)
        if share or cpu:  # a rehearsal of the control flow, not a measurement of N GPUs
            metric += " [rehearsal: " + ("all ranks on ONE shared GPU" if share else "host tensors over gloo") + \
                      ", not a multi-GPU measurement]"
        print(json.dumps({
            "metric": metric,
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
                       "parallelism": f"global{world}" if distributed else "single",
                       "impl": "python-host (gloo)" if cpu and distributed else "native",
                       "headline": (n, dim) == HEADLINE and not share and not cpu,
                       "shared_gpu": share and world > 1,
                       "device": "cpu (gloo rehearsal)" if cpu else (
                           f"MI355X (1 GPU shared by {world} ranks)" if share and world > 1 else "MI355X"),
                       "tree_checked": not args.no_check,
                       "errors_checked": "every timed build" if (not distributed and not cpu) else
                                         "last build (leaf misses are rebuilt inside each build)",
                       "sampling_misses_rebuilt": misses},
        }), flush=True)
    if world > 1:
        comm.destroy()


if __name__ == "__main__":
    main()
