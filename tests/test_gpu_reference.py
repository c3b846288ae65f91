"""GPU reference mode: the reference's own quirky tree (kdtree_sequential.cpp:46-48 sorts only the
first n - 1 points of every segment) and its search procedure (:75-130), on the GPU
(csrc/gpu/build_reference.hip, nn_traverse_reference in csrc/gpu/query.hip).

Oracle: the CPU reference-mode builder and search (csrc/cpu/cpu_tree.cpp), which the parity
tests pin to the compiled reference binary. std::sort is unstable, so the tree is only
defined up to ties: the builder tests use tie-free data (a random permutation of distinct
values per axis); the CLI tests use the reference generator at sizes where its
~22.5 M distinct values per axis (F5) leave the reference's segments tie-free."""
import subprocess
from pathlib import Path

import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops
from parallel_kd_tree_amd.ops.build import cpu_threads

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "bin"


def tie_free(n, dim, seed):
    g = torch.Generator().manual_seed(seed)
    cols = [(torch.randperm(n, generator=g).float() + 0.5) / max(n, 1) * 200 - 100 for _ in range(dim)]
    return torch.stack(cols, 1).contiguous() if n else torch.empty((0, dim))


@pytest.mark.parametrize("n,dim", [(1, 3), (2, 3), (3, 2), (5, 1), (100, 3), (1023, 3), (1024, 3), (4097, 2),
                                   (100_000, 3), (30_000, 8), (20_000, 16)])
def test_reference_tree_equals_cpu(gpu_device, n, dim):
    x = tie_free(n, dim, n + dim)
    b = ops.ReferenceTreeBuilder(n, dim)
    tp, ti = b.build(x.to(gpu_device), None, 1)
    cp, ci = ops.build_cpu(x, (torch.arange(n) + 1).to(torch.int32), "reference", 0, 1)
    assert b.read_ties() == 0, "tie-free data reported a deciding tie"
    assert torch.equal(ti.cpu(), ci), "GPU reference tree differs from the CPU reference tree"
    assert torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("n,dim", [(1_000_003, 3), (600_000, 2), (300_000, 5)])
def test_reference_selection_large_tie_free(gpu_device, n, dim):
    """Several device-wide selection levels (segments > 2048 rows: middle-zone refine, left
    maximum to the left segment's last slot, the last row kept) then the LDS finish."""
    x = tie_free(n, dim, 7 * n + dim)
    b = ops.ReferenceTreeBuilder(n, dim)
    assert b.global_levels >= 8
    tp, ti = b.build(x.to(gpu_device), None, 1)
    cp, ci = ops.build_cpu(x, (torch.arange(n) + 1).to(torch.int32), "reference", 0, 1)
    assert b.read_ties() == 0
    assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("n,dim", [(300_001, 3), (123_457, 2), (200_000, 5), (70_000, 8), (4_099, 1)])
def test_reference_finish_rank_equals_moving_finish(gpu_device, monkeypatch, n, dim):
    """The LDS finish by rank propagation (default) builds the tree the row-moving finish
    (PKD_REF_FIN=0) builds, and the CPU reference's; on tie-heavy data both report ties."""
    x = tie_free(n, dim, 3 * n + dim)
    out = {}
    for fin in ("0", "1"):
        monkeypatch.setenv("PKD_REF_FIN", fin)
        b = ops.ReferenceTreeBuilder(n, dim)
        out[fin] = b.build(x.to(gpu_device), None, 1)
        assert b.read_ties() == 0
    cp, ci = ops.build_cpu(x, (torch.arange(n) + 1).to(torch.int32), "reference", 0, 1)
    for tp, ti in out.values():
        assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)
    y = torch.randint(0, 300, (n, dim), generator=torch.Generator().manual_seed(n)).float()
    for fin in ("0", "1"):
        monkeypatch.setenv("PKD_REF_FIN", fin)
        b = ops.ReferenceTreeBuilder(n, dim)
        b.build(y.to(gpu_device), None, 1)
        assert b.read_ties() > 0


@pytest.mark.parametrize("n,vals", [(50_000, 7), (200_000, 1000), (3_001, 3)])
def test_reference_ties_detected_and_rebuilt(gpu_device, n, vals):
    """Heavy duplicates: equal keys decide segments (where std::sort's order is its library's
    business). The GPU build must COUNT them, and KDTree.build(mode='reference') must then return
    the CPU std::sort builder's tree (the reference binary's), with a warning -- never a tree that
    silently differs."""
    g = torch.Generator().manual_seed(n + vals)
    x = torch.randint(0, vals, (n, 3), generator=g).float()
    b = ops.ReferenceTreeBuilder(n, 3)
    b.build(x.to(gpu_device), None, 1)
    assert b.read_ties() > 0
    with pytest.warns(RuntimeWarning, match="std::sort"):
        t = pk.KDTree.build(x.to(gpu_device), id_base=1, mode="reference")
    cp, ci = ops.build_cpu(x, (torch.arange(n) + 1).to(torch.int32), "reference", 0, 1)
    assert torch.equal(t.tree_ids.cpu(), ci) and torch.equal(t.tree_pts.cpu(), cp)


def test_kdtree_gpu_reference_ties_repaired():
    """The reference generator at 3 M points (~22.5 M distinct values per axis) puts
    equal keys on deciding ranks: kdtree_gpu --mode reference repairs exactly those subtrees on the
    host (their ancestors' sorts replayed by the std::sort replica), notes it on stderr, and prints
    kdtree_sequential --mode reference's answers (the reference binary's)."""
    g = _run([BIN / "kdtree_gpu", "--mode", "reference", 11, 2, 3_000_000])
    c = _run([BIN / "kdtree_sequential", "--mode", "reference", 11, 2, 3_000_000])
    assert g.returncode == 0 and c.returncode == 0, g.stderr + c.stderr
    assert "replayed their sorts on the host" in g.stderr
    strip = lambda out: [l for l in out.splitlines() if not l.startswith("elapsed time")]  # noqa: E731
    assert strip(g.stdout) == strip(c.stdout)


def test_reference_tree_is_not_exact(gpu_device):
    """The reference tree violates the kd invariant: the mode is not a relabel
    of the exact tree."""
    x = tie_free(50_000, 3, 4)
    t = pk.KDTree.build(x.to(gpu_device), id_base=1, mode="reference")
    assert t.mode == "reference" and t.invariant_violations() > 0


@pytest.mark.parametrize("n,dim", [(20_000, 3), (5_000, 8), (2_000, 64)])
def test_reference_search_equals_cpu(gpu_device, n, dim):
    """KDTree(mode='reference') on the GPU answers exactly what the CPU reference search answers
    -- including the queries where the quirky tree makes it miss the true nearest neighbour."""
    x = tie_free(n + 400, dim, dim)
    pts, q = x[:n], x[n:]
    tg = pk.KDTree.build(pts.to(gpu_device), id_base=1, mode="reference")
    tc = pk.KDTree.build(pts, id_base=1, mode="reference")
    dg, _ = tg.query(q.to(gpu_device))
    dc, _ = tc.query(q)
    assert torch.equal(dg.cpu(), dc)
    if dim <= 3:  # the reference search really is approximate here (F1): some answers are not the NN
        brute = ((pts[None].double() - q[:, None].double()) ** 2).sum(-1).min(1).values.sqrt().float()
        assert bool((dc > brute).any())


def _run(args, **kw):
    return subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=300, **kw)


@pytest.mark.parametrize("seed,dim,n", [(42, 3, 1024), (7, 2, 5000), (3, 128, 2000)])
def test_kdtree_gpu_reference_mode_cli(seed, dim, n):
    """bin/kdtree_gpu --mode reference prints what kdtree_sequential --mode reference (the
    reference binary's output, tests/test_reference_parity.py) prints."""
    g = _run([BIN / "kdtree_gpu", "--mode", "reference", seed, dim, n])
    c = _run([BIN / "kdtree_sequential", "--mode", "reference", seed, dim, n])
    assert g.returncode == 0 and c.returncode == 0, g.stderr + c.stderr
    strip = lambda out: [l for l in out.splitlines() if not l.startswith("elapsed time")]  # noqa: E731
    assert strip(g.stdout) == strip(c.stdout)


def test_kdtree_dist_reference_forest_share_gpu():
    """kdtree_dist --mode reference: per-rank reference trees + the reference search + MIN reduce,
    i.e. the reference MPI program (kdtree_mpi.cpp); three ranks over RCCL on one card."""
    g = _run([BIN / "kdtree_dist", "--gpus", "3", "--share-gpu", "--mode", "reference", 5, 3, 4000])
    assert g.returncode == 0, g.stderr[-2000:]
    lines = [l for l in g.stdout.splitlines() if l.startswith("ID:")]
    x = pk.generate_problem(5, 3, 4010)
    q = x[4000:]
    best = None
    for r in range(3):
        first, cnt = 1333 * r, 1333 + (1 if r == 2 else 0)
        t = pk.KDTree.build(x[first:first + cnt], id_base=first + 1, mode="reference")
        d, _ = t.query(q)
        best = d if best is None else torch.minimum(best, d)
    from parallel_kd_tree_amd.utils import protocol
    assert lines == [protocol.result_line(4000 + i, float(best[i])) for i in range(10)]


def test_cli_save_and_leaf_threshold(tmp_path):
    """--save writes the tree file (utils/io.py format) and --leaf-threshold only changes how it
    is built, never the tree."""
    a, b = tmp_path / "a.pkd", tmp_path / "b.pkd"
    r1 = _run([BIN / "kdtree_gpu", "--save", a, 9, 3, 300_000])
    r2 = _run([BIN / "kdtree_gpu", "--save", b, "--leaf-threshold", "256", 9, 3, 300_000])
    assert r1.returncode == 0 and r2.returncode == 0, r1.stderr + r2.stderr
    strip = lambda out: [l for l in out.splitlines() if not l.startswith("elapsed time")]  # noqa: E731
    assert strip(r1.stdout) == strip(r2.stdout)
    ta, tb = pk.KDTree.load(a), pk.KDTree.load(b)
    x = pk.generate_problem(9, 3, 300_000)
    cp, ci = ops.build_cpu(x, None, "exact", 0, 8)
    assert torch.equal(ta.tree_ids, ci + 1) and torch.equal(ta.tree_pts, cp)
    assert torch.equal(tb.tree_ids, ta.tree_ids) and torch.equal(tb.tree_pts, ta.tree_pts)


@pytest.mark.parametrize("gpus", [2, 3])
def test_kdtree_dist_global_save_share_gpu(tmp_path, gpus):
    """kdtree_dist --decomp global --save: every rank writes its share into one file, rank 0 the
    boundary top rows; the file is the single-GPU exact tree (any rank count)."""
    f = tmp_path / "g.pkd"
    r = _run([BIN / "kdtree_dist", "--gpus", gpus, "--share-gpu", "--decomp", "global", "--save", f, 13, 3, 250_001])
    assert r.returncode == 0, r.stderr[-2000:]
    t = pk.KDTree.load(f)
    x = pk.generate_problem(13, 3, 250_001)
    cp, ci = ops.build_cpu(x, None, "exact", 0, 8)
    assert torch.equal(t.tree_ids, ci + 1) and torch.equal(t.tree_pts, cp)


@pytest.mark.parametrize("ranks,gpus,cfg", [(16, 2, (42, 3, 20000)), (16, 3, (5, 3, 16003)), (5, 2, (7, 2, 9001))])
def test_kdtree_dist_logical_ranks_reference(ranks, gpus, cfg):
    """kdtree_dist --ranks R --gpus P: the reference's `mpirun -np 16` (Makefile:36) forest on
    fewer GPUs. Every logical rank keeps the reference slicing at R, so reference-mode answers
    (which depend on the forest) are those of R reference ranks: here the CPU
    reference-mode builder per slice, which the parity tests pin to the reference MPI driver at
    -np 16 (tests/test_reference_parity.py::test_mpi_16_ranks_on_fewer_processes)."""
    seed, dim, n = cfg
    g = _run([BIN / "kdtree_dist", "--gpus", gpus, "--ranks", ranks, "--share-gpu", "--mode", "reference",
              seed, dim, n])
    assert g.returncode == 0, g.stderr[-2000:]
    lines = [l for l in g.stdout.splitlines() if l.startswith("ID:")]
    x = pk.generate_problem(seed, dim, n + 10)
    q = x[n:]
    best = None
    local = n // ranks
    for r in range(ranks):
        first, cnt = local * r, local + (n % ranks if r == ranks - 1 else 0)
        t = pk.KDTree.build(x[first:first + cnt], id_base=first + 1, mode="reference")
        d, _ = t.query(q)
        best = d if best is None else torch.minimum(best, d)
    from parallel_kd_tree_amd.utils import protocol
    assert lines == [protocol.result_line(n + i, float(best[i])) for i in range(10)]
    e = _run([BIN / "kdtree_dist", "--gpus", gpus, "--ranks", ranks, "--share-gpu", seed, dim, n])
    assert e.returncode == 0, e.stderr[-2000:]
    c = _run([BIN / "kdtree_sequential", seed, dim, n])  # exact mode: any forest answers the true NN
    strip = lambda out: [l for l in out.splitlines() if l.startswith("ID:")]  # noqa: E731
    assert strip(e.stdout) == strip(c.stdout)


@pytest.mark.parametrize("seed,dim,n", [(42, 3, 1_000_000), (11, 2, 3_000_000), (3, 128, 500_000), (42, 128, 500_000)])
def test_reference_mode_on_the_reference_stream_is_the_reference_tree(gpu_device, seed, dim, n):
    """The reference's own data (its generator stream) ties at every size: the hybrid reference mode
    (GPU tree + host repair of the tied subtrees and their ancestors' sorts) must be slot for slot
    the host std::sort builder's tree -- which the parity tests pin to the reference binary -- and
    must leave most of the GPU's slots alone when the ties sit deep in the tree. (Every measured
    size but 500 k x 128D with seed 3 ties.)"""
    x = pk.generate_problem(seed, dim, n)
    b = ops.ReferenceTreeBuilder(n, dim)
    b.build(x.to(gpu_device), None, 1)
    ties = b.read_ties()
    slots = b.read_tie_slots()
    assert len(slots) == ties
    if ties:
        with pytest.warns(RuntimeWarning, match="patched"):
            tp, ti, t2 = ops.build_reference_gpu_checked(x.to(gpu_device), None, 1)
    else:  # (500 k x 128D, seed 3: no deciding tie; the GPU tree stands as built)
        tp, ti, t2 = ops.build_reference_gpu_checked(x.to(gpu_device), None, 1)
    # (the count inside a tied subtree depends on how the GPU happened to order that subtree's equal
    # keys, which the repair replaces anyway: it may differ by a few between builds)
    assert (t2 > 0) == (ties > 0)
    cp, ci = ops.build_cpu(x, (torch.arange(n) + 1).to(torch.int32), "reference", 0, cpu_threads())
    assert torch.equal(ti.cpu(), ci), "repaired GPU reference tree differs from the std::sort tree"
    assert torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("seed", [3, 42])
def test_eval_reference_mode_matches_reference_fixture(seed):
    """The graded evaluation problem (seed on stdin, 500 k x 128D) in reference mode on the GPU:
    byte-identical to what the reference binary printed (tests/fixtures)."""
    fix = (Path(__file__).parent / "fixtures" / f"ref_eval_seed{seed}.txt").read_text().splitlines()
    g = _run([BIN / "kdtree_gpu", "--mode", "reference"], input=f"{seed}\n")
    assert g.returncode == 0, g.stderr
    assert [l for l in g.stdout.splitlines() if not l.startswith("elapsed time")] == fix
