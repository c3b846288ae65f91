"""GPU builder vs the CPU exact oracle: the exact tree is unique, so the in-order ids must be
identical slot for slot. Covers global levels (fused histogram / partition / refine), the LDS
subtree kernel, duplicates (radix refine path), dims 1..128, and the query kernels."""
import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops

pytestmark = pytest.mark.gpu


def check_same(x, dev, depth0=0, subtree_max=0, allow_top=True):
    b = ops.GpuTreeBuilder(x.shape[0], x.shape[1], depth0, subtree_max, allow_top=allow_top)
    tp, ti = b.build(x.to(dev))
    cp, ci = ops.build_cpu(x, None, "exact", depth0, 8)
    torch.cuda.synchronize()
    assert b.read_error() == 0
    assert torch.equal(ti.cpu(), ci), "GPU tree differs from the CPU exact tree"
    assert torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 100, 1000, 4095, 4096, 4097, 10000])
def test_small_n_dim3(gpu_device, n):
    check_same(pk.generate_problem(n, 3, n), gpu_device)


@pytest.mark.parametrize("dim", [1, 2, 3, 4, 5, 8, 16, 128])
def test_dims_global_levels(gpu_device, dim):
    n = 200_000 if dim <= 16 else 20_000
    check_same(pk.generate_problem(dim, dim, n), gpu_device)


def test_large_3d(gpu_device):
    check_same(pk.generate_problem(1, 3, 3_000_000), gpu_device)


def test_forced_small_subtree(gpu_device):
    # more global levels, deep segments, many blocks per level
    check_same(pk.generate_problem(4, 3, 300_000), gpu_device, subtree_max=256)


@pytest.mark.parametrize("cfg", ["1x768", "3x256", "6x128", "2x384", "2x512", "1x1024", "4x256"])
@pytest.mark.parametrize("dim", [3, 5, 8])
def test_subtree_launch_shapes(gpu_device, monkeypatch, cfg, dim):
    """Segments of 513..768 points (100M x 8D: 763) under every LDS subtree launch shape for that
    capacity: the same exact tree (uniform and duplicate-heavy rows)."""
    monkeypatch.setenv("PKD_AB", "1")
    monkeypatch.setenv("PKD_SUBTREE_CFG", cfg)
    n = 763 * 512 + 17
    check_same(pk.generate_problem(dim + 40, dim, n), gpu_device, subtree_max=1024)
    check_same(torch.randint(0, 9, (n, dim)).float(), gpu_device, subtree_max=1024, depth0=dim - 1)


@pytest.mark.parametrize("cfg", ["6x256", "4x384", "2x768", ""])
@pytest.mark.parametrize("dim", [2, 3, 4])
def test_subtree_launch_shapes_1536(gpu_device, monkeypatch, cfg, dim):
    """Segments of 1025..1536 points (100M x 3D: 1525) under the launch shapes of that capacity."""
    monkeypatch.setenv("PKD_AB", "1")
    monkeypatch.setenv("PKD_SUBTREE_CFG", cfg)
    n = 1525 * 256 + 9
    check_same(pk.generate_problem(dim + 50, dim, n), gpu_device, subtree_max=2048)
    check_same(torch.randint(0, 9, (n, dim)).float(), gpu_device, subtree_max=2048, depth0=1)


def test_duplicates(gpu_device):
    g = torch.randint(0, 5, (300_000, 3)).float()
    check_same(g, gpu_device)
    check_same(torch.zeros(50_000, 2), gpu_device)
    check_same(torch.randint(0, 2, (20_000, 3)).float(), gpu_device)


@pytest.mark.parametrize("atomic,stage,wide", [("0", "1", "8"), ("0", "1", "4"), ("0", "0", "4"), ("1", "1", "8")])
@pytest.mark.parametrize("triple_from", ["0", "3"])
def test_triple_levels(gpu_device, monkeypatch, triple_from, atomic, stage, wide):
    """Three levels per scatter pass (k_scan2 + k_partition3, from level 0 or 3) with zone ranks
    from wave ballots (stores through an LDS tile, or from registers) or LDS atomics (also in the
    pair scatters): slot for slot the CPU exact tree on uniform, duplicate-heavy, 2-D, 8-D and
    odd-depth inputs."""
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_PART3_STAGE", stage)
    monkeypatch.setenv("PKD_WIDE_KI", wide)
    monkeypatch.setenv("PKD_TAIL", "0")  # the last three levels stay triples too
    monkeypatch.setenv("PKD_TRIPLE_FROM", triple_from)
    monkeypatch.setenv("PKD_PART_ATOMIC", atomic)
    monkeypatch.setenv("PKD_PART3_ATOMIC", atomic)
    b = ops.GpuTreeBuilder(1_000_000, 3)
    assert "triple" in b.describe(), b.describe()
    check_same(pk.generate_problem(11, 3, 1_000_000), gpu_device)
    check_same(torch.randint(0, 7, (600_000, 3)).float(), gpu_device)
    check_same(pk.generate_problem(12, 2, 700_001), gpu_device)
    check_same(pk.generate_problem(13, 8, 400_000), gpu_device)
    check_same(pk.generate_problem(15, 6, 300_001), gpu_device, depth0=4)
    check_same(pk.generate_problem(14, 3, 900_000), gpu_device, depth0=2)


@pytest.mark.parametrize("n", [1025, 1100, 1525, 1536, 1537, 3100, 6143, 12_500_000])
def test_subtree_capacity_1536(gpu_device, n):
    """3-D leaf segments of 1025..1536 points take the non-power-of-two LDS subtree shape
    (3 items x 512 threads: bucket counts capped at the capacity, u16 slot
    table, bitmaps aliasing the bucket-order index list): slot for slot the CPU exact tree,
    also with heavy duplicates."""
    check_same(pk.generate_problem(n % 97, 3, n), gpu_device)
    if n < 100_000:
        check_same(torch.randint(0, 3, (n, 3)).float(), gpu_device)
        check_same(pk.generate_problem(n % 89, 3, n), gpu_device, depth0=1)


@pytest.mark.parametrize("slim12,pipe", [("0", "1"), ("1", "1"), ("2", "1"), ("2", "0")])
@pytest.mark.parametrize("n,dim", [(40_000, 3), (70_000, 3), (100_000, 3), (200_000, 1), (150_000, 2), (120_000, 5),
                                   (60_000, 8)])
def test_tail_levels(gpu_device, monkeypatch, n, dim, slim12, pipe):
    """The last three global levels in one workgroup per segment (k_tail3: bucket bins, wave
    ranking of the median bin or the radix-select fallback for heavy duplicates, LDS-staged
    leaf scatter): slot for slot the CPU exact tree. 16-item shapes (100 k at 3-D) and, with
    PKD_TAIL_SLIM12, the 12-item shapes run with all keys + ids (0), two key register sets and
    ids read on demand (1) or two key sets + ids (2, the default); PKD_TAIL_PIPE=0 moves the
    columns without the next column's loads in flight and with one stage buffer."""
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_TAIL", "1")
    monkeypatch.setenv("PKD_TAIL_SLIM12", slim12)
    monkeypatch.setenv("PKD_TAIL_PIPE", pipe)
    b = ops.GpuTreeBuilder(n, dim)
    assert "tail" in b.describe(), b.describe()
    check_same(pk.generate_problem(n % 101, dim, n), gpu_device)
    check_same(torch.randint(0, 3, (n, dim)).float(), gpu_device)
    check_same(torch.randint(0, 200, (n, dim)).float(), gpu_device)
    check_same(pk.generate_problem(n % 103, dim, n), gpu_device, depth0=dim + 1)


def test_tail_levels_off_equal(gpu_device, monkeypatch):
    x = pk.generate_problem(5, 3, 3_000_000).to(gpu_device)
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_TAIL", "1")
    _, ti = ops.GpuTreeBuilder(3_000_000, 3).build(x)
    monkeypatch.setenv("PKD_TAIL", "0")
    b = ops.GpuTreeBuilder(3_000_000, 3)
    assert "tail" not in b.describe()
    _, ti0 = b.build(x)
    torch.cuda.synchronize()
    assert torch.equal(ti, ti0)


def test_depth0(gpu_device):
    check_same(pk.generate_problem(8, 3, 100_000), gpu_device, depth0=1)


def test_queries_exact(gpu_device):
    x = pk.generate_problem(3, 3, 200_010)
    t = pk.KDTree.build(x[:200_000].to(gpu_device))
    q = torch.cat([x[200_000:], torch.rand(5000, 3) * 200 - 100]).to(gpu_device)
    pb = t.query_packed(q, "brute")
    pt = t.query_packed(q, "traverse")
    assert torch.equal(pb, pt)
    raw = ops.nn_gpu(x[:200_000].to(gpu_device), None, q, "brute")
    d2a, _ = ops.unpack(pb)
    d2b, _ = ops.unpack(raw)
    assert torch.equal(d2a, d2b)


def test_queries_high_dim(gpu_device):
    x = pk.generate_problem(9, 128, 30_010)
    t = pk.KDTree.build(x[:30_000].to(gpu_device), id_base=1)
    d, ids = t.query(x[30_000:].to(gpu_device), method="brute")
    tc = pk.KDTree.build(x[:30_000], id_base=1)
    dc, idc = tc.query(x[30_000:])
    assert torch.equal(d.cpu(), dc) and torch.equal(ids.cpu(), idc)


def test_large_stage2_pairs(gpu_device):
    # 20M points: levels 0 and 1 both need the second-stage histogram, so the first pair
    # runs k_hist2p / k_select2 for its second level and the block-reserve count pass
    check_same(pk.generate_problem(5, 3, 20_000_000), gpu_device)


@pytest.mark.parametrize("dim,n,depth0", [(32, 100_000, 0), (64, 60_000, 5), (128, 100_000, 0), (128, 33_333, 127)])
def test_narrow_columns(gpu_device, dim, n, depth0):
    # high-dim AoS input: the global levels move only their keys, the ids and the input row index;
    # medians and subtree rows are gathered from the input
    check_same(pk.generate_problem(dim + depth0, dim, n), gpu_device, depth0=depth0)


def test_narrow_columns_explicit_ids(gpu_device, monkeypatch):
    dim, n = 96, 50_000
    x = pk.generate_problem(11, dim, n)
    ids = torch.randperm(n, generator=torch.Generator().manual_seed(3)).to(torch.int32) + 7
    cp, ci = ops.build_cpu(x, ids, "exact", 0, 8)
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    for narrow in ("1", "0"):
        monkeypatch.setenv("PKD_NARROW", narrow)
        b = ops.GpuTreeBuilder(n, dim, 0, 0)
        tp, ti = b.build(x.to(gpu_device), ids.to(gpu_device))
        torch.cuda.synchronize()
        assert b.read_error() == 0
        assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("prefix", ["1", "0"])
def test_large_stage2_pairs_prefix_placement(gpu_device, monkeypatch, prefix):
    # prefix placement of the top pairs (per-block offsets from k_hist2p's counts) on skewed
    # data: one axis takes few distinct values, so median buckets are huge and many rows are
    # appended with cursor atomics after the certain rows; PKD_PART_PREFIX=0 is the counting pass
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_PART_PREFIX", prefix)
    x = pk.generate_problem(6, 3, 18_000_000)
    x[:, 1] = torch.round(x[:, 1] / 25.0) * 25.0
    check_same(x, gpu_device, allow_top=False)  # (the paired levels from level 0)
    _check_sampled_or_rebuilt(x, gpu_device)


def _check_sampled_or_rebuilt(x, dev):
    """The default (sampled-top) build of duplicate-heavy data either succeeds exactly or reports
    the band miss (a staging arena too large to stream); the checked entry point is exact."""
    b = ops.GpuTreeBuilder(x.shape[0], x.shape[1], 0, 0)
    tp, ti = b.build(x.to(dev))
    cp, ci = ops.build_cpu(x, None, "exact", 0, 8)
    torch.cuda.synchronize()
    err = b.read_error()
    if err == 0:
        assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)
    else:
        assert b.sampled and err & ops.GpuTreeBuilder.TOP_BAND_MISS, (err, b.describe())
    tp2, ti2, _ = ops.build_gpu_checked(x.to(dev), None, 0, 0)
    torch.cuda.synchronize()
    assert torch.equal(ti2.cpu(), ci) and torch.equal(tp2.cpu(), cp)


@pytest.mark.parametrize("n,dim,depth0", [(1, 3, 0), (1000, 3, 0), (200_000, 3, 0), (100_000, 5, 2), (30_000, 8, 0)])
def test_device_invariant_checker(gpu_device, n, dim, depth0):
    """The HIP checker (semantic race detector) passes on built trees and catches corruption."""
    x = pk.generate_problem(n + dim, dim, n)
    t = pk.KDTree.build(x.to(gpu_device), id_base=1, depth0=depth0)
    assert t.invariant_violations() == 0
    cpu = pk.KDTree(t.tree_pts.cpu(), t.tree_ids.cpu(), depth0)
    assert cpu.invariant_violations() == 0
    if n > 2:  # swap the root with its left neighbour: both sides break
        r = n // 2
        for a in (t.tree_pts, t.tree_ids):
            tmp = a[r].clone()
            a[r] = a[r - 1]
            a[r - 1] = tmp
        assert t.invariant_violations() > 0
        assert pk.KDTree(t.tree_pts.cpu(), t.tree_ids.cpu(), depth0).invariant_violations() > 0


def _check_headline(x, dev):
    """A full correctness proof of one build without a CPU oracle: device error word 0, the
    exact kd invariant at every node (k_check), ids a permutation of 1..n and every output
    row the input row its id names (so the multiset of rows is preserved)."""
    n, dim = x.shape
    b = ops.GpuTreeBuilder(n, dim)
    tp, ti = b.build(x, None, 1)
    torch.cuda.synchronize()
    assert b.read_error() == 0, b.read_error_detail()
    assert pk.KDTree(tp, ti, 0).invariant_violations() == 0
    idx = ti.to(torch.int64) - 1
    assert int(idx.min()) == 0 and int(idx.max()) == n - 1
    seen = torch.zeros(n, dtype=torch.int32, device=dev)
    seen.index_add_(0, idx, torch.ones_like(idx, dtype=torch.int32))
    assert bool((seen == 1).all()), "ids are not a permutation"
    assert torch.equal(tp, x[idx]), "an output row differs from the input row of its id"
    return b


@pytest.mark.slow
def test_headline_100m_3d(gpu_device):
    """BASELINE's headline config, 100 M x 3D: the >= 64 M path (2048-block level grids) that
    bench.py times."""
    x = pk.generate_slice(42, 3, 0, 100_000_000, device=gpu_device)
    b = _check_headline(x, gpu_device)
    assert b.global_levels == 16


@pytest.mark.slow
def test_headline_100m_8d(gpu_device):
    x = pk.generate_slice(42, 8, 0, 100_000_000, device=gpu_device)
    _check_headline(x, gpu_device)


@pytest.mark.slow
def test_64m_3d_equals_cpu_exact(gpu_device):
    """Slot-for-slot against the multi-threaded CPU exact builder at >= 64 M points."""
    n = 64_000_000
    x = pk.generate_slice(5, 3, 0, n, device=gpu_device)
    b = _check_headline(x, gpu_device)
    tp, ti = b.build(x, None, 1)
    cp, ci = ops.build_cpu(x.cpu(), None, "exact", 0, 16)
    assert torch.equal(ti.cpu(), ci + 1)
    assert torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("n", [100_000, 12_500_000])
def test_hipgraph_replay_equals_eager(gpu_device, n):
    """A build captured in a hipGraph (torch.cuda.CUDAGraph) replays to the eager tree. 12.5 M
    is the size whose replay used to fault: the stage-2 histogram resets were runtime
    hipMemsetAsync nodes; they are now zero-fill kernels of our own (tools/graph_check.py)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
    import graph_check
    graph_check.check(n)


@pytest.mark.parametrize("level,parts,streams", [(2, 4, 4), (2, 4, 2), (4, 16, 3), (4, 8, 1), (6, 64, 4)])
def test_split_build_equals_cpu(gpu_device, monkeypatch, level, parts, streams):
    """Split build (from a pair boundary on, segment ranges on several HIP streams with their own
    histogram sets) at sizes below its default threshold: slot for slot the CPU exact tree."""
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_SPLIT_MIN_N", "0")
    monkeypatch.setenv("PKD_SPLIT_LEVEL", str(level))
    monkeypatch.setenv("PKD_SPLIT_PARTS", str(parts))
    monkeypatch.setenv("PKD_SPLIT_STREAMS", str(streams))
    for seed, dim, n in ((21, 3, 3_000_001), (22, 2, 1_000_000), (23, 8, 700_000)):
        b = ops.GpuTreeBuilder(n, dim)
        assert b.split_parts == min(parts, 2 ** level), b.describe()
        check_same(pk.generate_problem(seed, dim, n), gpu_device)


def test_split_build_stage2_skewed(gpu_device, monkeypatch):
    """Split build whose parts start with second-stage levels and prefix placement (18 M
    points, split after the first pair) on skewed data."""
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_SPLIT_MIN_N", "0")
    x = pk.generate_problem(6, 3, 18_000_000)
    x[:, 1] = torch.round(x[:, 1] / 25.0) * 25.0
    check_same(x, gpu_device, allow_top=False)
    _check_sampled_or_rebuilt(x, gpu_device)


def test_split_build_hipgraph(gpu_device, monkeypatch):
    """A split build captured into a hipGraph (fork / join events across the side streams)
    replays to the eager tree."""
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_SPLIT_MIN_N", "0")
    n, dim = 2_000_003, 3
    x = pk.generate_slice(9, dim, 0, n, device=gpu_device)
    b = ops.GpuTreeBuilder(n, dim)
    assert b.split_parts > 1
    ep, ei = b.build(x, None, 1)
    torch.cuda.synchronize()
    gp, gi = torch.empty_like(ep), torch.empty_like(ei)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        b.build(x, None, 1, gp, gi)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.build(x, None, 1, gp, gi)
    gp.zero_()
    gi.zero_()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert b.read_error() == 0
    assert torch.equal(gi, ei) and torch.equal(gp, ep)


def test_removed_subtree_impl_knob_fails_loudly(gpu_device, monkeypatch):
    """Only the shipped subtree kernel exists: the old selector is rejected, not ignored."""
    monkeypatch.setenv("PKD_SUBTREE_IMPL", "wave")
    with pytest.raises(Exception, match="PKD_SUBTREE_IMPL was removed"):
        ops.GpuTreeBuilder(1000, 3)


def test_nearest_neighbor_no_tree_copy(gpu_device, monkeypatch):
    """KDTree.nearest_neighbor / Node on a 10 M GPU tree: the id -> slot lookup runs on the
    device and a Node reads one row; the whole tree never crosses to the host (any device ->
    host copy larger than a few rows fails the test)."""
    from parallel_kd_tree_amd.models.node import Point
    n = 10_000_000
    x = pk.generate_slice(12, 3, 0, n + 1, device=gpu_device)
    t = pk.KDTree.build(x[:n], id_base=1)
    q = x[n:].cpu().numpy()[0]
    orig = torch.Tensor.cpu
    moved = []

    def spy(self, *a, **kw):
        moved.append(self.numel() * self.element_size())
        return orig(self, *a, **kw)

    monkeypatch.setattr(torch.Tensor, "cpu", spy)
    node = t.nearest_neighbor(Point(3, n + 1, q))
    monkeypatch.setattr(torch.Tensor, "cpu", orig)
    assert max(moved, default=0) <= 64, moved
    d, ids = t.query(x[n:])
    assert node.point.ID == int(ids[0].item())
    assert t._host is None


@pytest.mark.parametrize("n,dim,nq,depth0", [(1_000_000, 3, 3000, 0), (300_000, 8, 2000, 0), (200_000, 5, 1000, 2),
                                             (100_000, 12, 500, 0), (1000, 3, 100, 0), (700, 2, 50, 1)])
def test_traversal_kernels_equal_brute(gpu_device, monkeypatch, n, dim, nq, depth0):
    """The wave-per-query traversal (bucket scans of 512-point sub-trees) and the older
    thread-per-query traversal both return exactly the brute-force (d2, id) minimum,
    including queries on and off the data, and trees rooted below depth 0."""
    x = pk.generate_problem(n + dim, dim, n + nq)
    t = pk.KDTree.build(x[:n].to(gpu_device), id_base=1, depth0=depth0)
    q = torch.cat([x[n:], x[: nq // 4]]).to(gpu_device)  # a quarter of the queries hit a point exactly
    pb = t.query_packed(q, "brute")
    pw = t.query_packed(q, "traverse")
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_TRAVERSE", "thread")
    pt = t.query_packed(q, "traverse")
    assert torch.equal(pb, pw) and torch.equal(pb, pt)


@pytest.mark.parametrize("k", [-1, 0, 2])
def test_native_global_builder_one_rank(gpu_device, k):
    """parallel/native_global.py (the C++ GlobalBuilder on an RCCL communicator of one rank,
    the multi-GPU code path of bench.py) gives the single-GPU tree slot for slot."""
    from parallel_kd_tree_amd.parallel.native_global import NativeGlobalBuilder
    n, dim = 300_001, 3
    x = pk.generate_slice(5, dim, 0, n, device=gpu_device)
    g = NativeGlobalBuilder(n, dim, gpu_device, pipeline_k=k)
    for _ in range(2):  # buffers reused by the second build
        t = g.build(x, id_base=1)
    assert g.read_error() == 0 and t.slot_lo == 0 and t.tree_ids.numel() == n
    assert g._g.middle_scale() == 1, "the top levels' middle buckets overflowed their all-gather slots"
    b = ops.GpuTreeBuilder(n, dim)
    tp, ti = b.build(x, None, 1)
    assert torch.equal(t.tree_ids, ti) and torch.equal(t.tree_pts, tp)


def test_bench_native_global_one_rank():
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--decomp", "global", "--points", "3000000", "--steps", "2",
                        "--warmup", "1", "--pipeline-k", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["parallelism"] == "global1" and line["config"]["tree_checked"]
