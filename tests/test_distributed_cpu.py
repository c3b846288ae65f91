"""Multi-process (gloo) tests of the forest and global decompositions on CPU.

The global tree assembled from P ranks must be slot-for-slot the single-process exact tree
(unique under the (key, id) order); forest and global queries must equal brute force; the
reference-mode forest must reproduce the reference MPI binary's per-rank search."""
import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        torch.set_num_threads(1)
        from parallel_kd_tree_amd.parallel import comm
        comm.init(backend="gloo", timeout_s=150)
        fn(rank, world, *args)
        comm.barrier()
        comm.destroy()
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))


def run(world, fn, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    errs = []
    try:
        for _ in range(world):
            errs.append(q.get(timeout=240))
    except Exception:  # a rank died or hangs in a collective: end the group instead of hanging
        for p in procs:
            if p.is_alive():
                p.kill()
        raise AssertionError(f"only {len(errs)} of {world} ranks finished: {[e for _, e in errs if e]}")
    for p in procs:
        p.join(60)
    bad = [e for _, e in errs if e]
    assert not bad, bad[0]


def _global_case(rank, world, n, dim, seed):
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
    first, cnt = comm.forest_slice(n, world, rank)
    x = pk.generate_slice(seed, dim, first, cnt)
    b = GlobalTreeBuilder(n, dim, device=torch.device("cpu"))
    t = b.build(x, id_base=first)
    tp, ti = t.gather_full()
    full = pk.generate_problem(seed, dim, n + 7)
    cp, ci = ops.build_cpu(full[:n], None, "exact", 0, 1)
    assert torch.equal(ti, ci), f"rank {rank}: global tree differs from the single-process tree"
    assert torch.equal(tp, cp)
    q = full[n:]
    packed = t.query_packed(q)
    d2, ids = ops.unpack(packed)
    ref = ((full[:n][None].double() - q[:, None].double()) ** 2).sum(-1).min(1).values
    got = ((full[:n][ids].double() - q.double()) ** 2).sum(-1)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("world,n,dim", [(2, 5000, 3), (4, 20000, 3), (2, 3001, 2), (4, 1000, 5), (2, 7, 3),
                                         (8, 3000, 3), (3, 6001, 3), (5, 4000, 2), (6, 3000, 3), (3, 4, 3)])
def test_global_tree_equals_single(world, n, dim):
    run(world, _global_case, n, dim, 11)


def _global_dupes(rank, world):
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
    g = torch.Generator().manual_seed(3)
    full = torch.randint(0, 3, (6000, 3), generator=g).float()
    lo, hi = rank * 3000, (rank + 1) * 3000
    t = GlobalTreeBuilder(6000, 3, device=torch.device("cpu")).build(full[lo:hi], id_base=lo)
    _, ti = t.gather_full()
    _, ci = ops.build_cpu(full, None, "exact", 0, 1)
    assert torch.equal(ti, ci)


def test_global_tree_duplicates():
    run(2, _global_dupes)


def _forest_case(rank, world, n, dim, mode):
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.forest import ForestTree
    first, cnt = comm.forest_slice(n, world, rank)
    x = pk.generate_slice(5, dim, first, cnt)
    f = ForestTree.build(x, first, n, id_base=1, mode=mode)
    full = pk.generate_problem(5, dim, n + 10)
    q = full[n:]
    d2, ids = ops.unpack(f.query_packed(q))
    if mode == "exact":
        ref = ((full[:n][None].double() - q[:, None].double()) ** 2).sum(-1).min(1).values
        got = ((full[:n][ids - 1].double() - q.double()) ** 2).sum(-1)
        assert torch.equal(got, ref)
    else:
        # each rank's reference search, MIN over ranks (kdtree_mpi.cpp:234-253)
        best = None
        for r in range(world):
            fr, cr = comm.forest_slice(n, world, r)
            tr = pk.KDTree.build(full[fr:fr + cr], id_base=fr + 1, mode="reference")
            dr, _ = tr.query(q)
            best = dr if best is None else torch.minimum(best, dr)
        assert torch.equal(ops.query.sqrt_exact(d2), best)


@pytest.mark.parametrize("world,mode", [(2, "exact"), (4, "exact"), (3, "exact"), (4, "reference")])
def test_forest(world, mode):
    run(world, _forest_case, 4000, 3, mode)


def _forest_tiny(rank, world):
    # N < P: ranks without points must not crash (reference segfaults)
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.forest import ForestTree
    first, cnt = comm.forest_slice(2, world, rank)
    full = pk.generate_problem(9, 3, 2 + 10)
    f = ForestTree.build(full[first:first + cnt], first, 2)
    d2, ids = ops.unpack(f.query_packed(full[2:]))
    assert bool((ids >= 1).all()) and bool((ids <= 2).all())


def test_forest_n_less_than_p():
    run(4, _forest_tiny)


def _pipelined_case(rank, world, n, dim, k):
    """Extra top levels on gloo: one all-to-all round per leaf of a rank, with real async work
    handles, each leaf subtree built while the next round is in flight; the tree must not
    depend on k."""
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm, global_tree
    from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
    handles = []
    orig = comm.all_to_all_single_async

    def spy(*a, **kw):
        h = orig(*a, **kw)
        handles.append(h)
        return h

    global_tree.comm.all_to_all_single_async = spy
    try:
        first, cnt = comm.forest_slice(n, world, rank)
        x = pk.generate_slice(13, dim, first, cnt)
        b = GlobalTreeBuilder(n, dim, device=torch.device("cpu"), pipeline_k=k)
        t = b.build(x, id_base=first)
    finally:
        global_tree.comm.all_to_all_single_async = orig
    assert len(handles) == b.layout["R"] and all(h is not None and hasattr(h, "wait") for h in handles)
    if world & (world - 1) == 0:
        assert b.layout["R"] == 1 << k
    assert t.check_top_routing() == ""
    tp, ti = t.gather_full()
    full = pk.generate_problem(13, dim, n)
    cp, ci = ops.build_cpu(full, None, "exact", 0, 1)
    assert torch.equal(ti, ci) and torch.equal(tp, cp)


@pytest.mark.parametrize("world,k", [(2, 0), (2, 1), (2, 3), (4, 2), (8, 1), (3, 1), (6, 0)])
def test_global_tree_pipelined_rounds(world, k):
    run(world, _pipelined_case, 30_001, 3, k)


def _plan_consistency(rank, world):
    """A leaf total that disagrees with the tree geometry raises on EVERY rank (the count
    matrix is all-gathered), so no rank is left waiting inside the exchange."""
    from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
    b = GlobalTreeBuilder(1000, 3, device=torch.device("cpu"), pipeline_k=0)
    T = b.layout["T"]
    counts = torch.zeros((T, 4), dtype=torch.int64)
    for t in range(T):  # every rank claims an equal share of every leaf ...
        counts[t, 0] = b.layout["leaf_n"][t] // world + (1 if rank < b.layout["leaf_n"][t] % world else 0)
    if rank == 0:
        counts[1, 0] += 1  # ... but rank 0 claims one extra row for leaf 1
    with pytest.raises(RuntimeError, match="would receive"):
        b._exchange_plan(counts)


def test_exchange_plan_fails_on_every_rank():
    run(4, _plan_consistency)


def _routing_check_catches(rank, world):
    """DistTree.check_top_routing sees a point on the wrong side of a top pivot (the bench's
    cross-rank check), which no per-rank invariant check can."""
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
    n = 4000
    first, cnt = comm.forest_slice(n, world, rank)
    t = GlobalTreeBuilder(n, 3, device=torch.device("cpu")).build(pk.generate_slice(2, 3, first, cnt), id_base=1)
    assert t.check_top_routing() == ""
    if rank == 1:  # move rank 1's first point to the far low end of axis 0 (left of the root pivot)
        t.tree_pts[0, 0] = -1000.0
        assert "pivot of top node 0" in t.check_top_routing()


def test_top_routing_check():
    run(2, _routing_check_catches)


def _routed_queries(rank, world, n, dim, nq):
    """Routed queries (home leaf first, then only the blocks the best ball reaches) give the
    brute-force distances with ~1/P of the (query, block) searches per rank."""
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
    first, cnt = comm.forest_slice(n, world, rank)
    x = pk.generate_slice(17, dim, first, cnt)
    t = GlobalTreeBuilder(n, dim, device=torch.device("cpu")).build(x, id_base=first + 1)
    full = pk.generate_problem(17, dim, n + nq)
    q = full[n:]
    d2, _ = ops.unpack(t.query_packed(q))
    work = t.last_query_work
    d2a, _ = ops.unpack(t.query_packed(q, routed=False))
    ref = ((full[:n][None].double() - q[:, None].double()) ** 2).sum(-1).min(1).values
    assert torch.equal(d2.double(), ref.float().double()) or torch.allclose(d2.double(), ref, rtol=1e-6)
    assert torch.equal(d2, d2a)
    tot = torch.tensor([work], dtype=torch.int64)
    comm.all_reduce_(tot)
    assert int(tot) < 1.5 * nq, f"routed queries searched {int(tot)} (query, block) pairs for {nq} queries"


@pytest.mark.parametrize("world,dim", [(4, 3), (3, 2)])
def test_routed_queries(world, dim):
    run(world, _routed_queries, 20_000, dim, 300)
