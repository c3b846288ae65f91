"""The whole global decomposition on the GPU with several ranks sharing one card.

The box this runs on has a single MI355X, and RCCL refuses two ranks on one device, so the
ranks talk over gloo (device tensors are staged through the host by parallel.comm) while
every per-rank op is the HIP kernel path used with RCCL on a multi-GPU node. The assembled
tree must be slot-for-slot the single-GPU tree and queries must equal brute force."""
import pytest
import torch

from test_distributed_cpu import run

pytestmark = pytest.mark.gpu


def _case(rank, world, n, dim, seed, dupes, explicit=False):
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.global_tree import GlobalTreeBuilder
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    first, cnt = comm.forest_slice(n, world, rank)
    if dupes:
        g = torch.Generator().manual_seed(seed)
        full = torch.randint(0, 3, (n + 10, dim), generator=g).float()
    else:
        full = pk.generate_problem(seed, dim, n + 10)
    x = full[first:first + cnt].to(dev)
    b = GlobalTreeBuilder(n, dim, device=dev, timings=True)
    # implicit ids take the compact exchange (12-B rows + destination bitmaps), explicit ids
    # the 16-B rows
    ids = (torch.arange(cnt, dtype=torch.int32) + first + 1).to(dev) if explicit else None
    t = b.build(x, ids, id_base=first + 1)
    t = b.build(x, ids, id_base=first + 1)  # reuse of the builder's workspaces
    assert b.read_error() == 0
    assert t.tree_pts.is_cuda and set(t.timings) >= {"bbox", "pack", "all_to_all", "local_build"}
    tp, ti = t.gather_full()
    cp, ci = ops.build_cpu(full[:n], None, "exact", 0, 1)
    assert torch.equal(ti.cpu(), ci + 1), f"rank {rank}: global tree differs from the single-process tree"
    assert torch.equal(tp.cpu(), cp)
    q = full[n:].to(dev)
    d2, ids = ops.unpack(t.query_packed(q))
    ref = ((full[:n][None].double() - full[n:][:, None].double()) ** 2).sum(-1).min(1).values
    got = ((full[:n][ids.cpu() - 1].double() - full[n:].double()) ** 2).sum(-1)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("world,n,dim,dupes", [(2, 300_000, 3, False), (4, 400_000, 3, False),
                                               (4, 50_001, 5, False), (2, 40_000, 2, True), (4, 7, 3, False),
                                               (8, 800_003, 3, False)])
def test_global_tree_gpu(world, n, dim, dupes):
    run(world, _case, n, dim, 21, dupes)


def test_global_tree_gpu_explicit_ids():
    run(4, _case, 300_000, 3, 22, False, True)


@pytest.mark.parametrize("world,k", [(2, 0), (2, 3), (4, 2), (8, 1)])
def test_global_tree_gpu_pipeline_depth(monkeypatch, world, k):
    """Exchange rounds: every rank's subtree split k levels further by the distributed top
    levels, leaf subtrees built while the next leaf's rows are in flight (k = 0: one
    all-to-all). Same tree for every k."""
    monkeypatch.setenv("PKD_PIPELINE_K", str(k))
    run(world, _case, 200_001, 3, 23, False)
