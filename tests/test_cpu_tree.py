"""CPU tree: exact builder invariants, NN vs brute force, reference-mode parity, save/load,
Point/Node facade (Node.hpp:9-45)."""
import numpy as np
import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops


def brute_d2(x, q):
    d = ((x[None, :, :].double() - q[:, None, :].double()) ** 2).sum(-1)
    return d.min(1)


@pytest.mark.parametrize("n,dim", [(1, 3), (2, 3), (3, 1), (7, 2), (100, 3), (1024, 3), (5000, 1), (3000, 8),
                                   (500, 128)])
def test_exact_invariant_and_nn(n, dim):
    x = pk.generate_problem(n + dim, dim, n + 20)
    t = pk.KDTree.build(x[:n])
    assert t.invariant_violations() == 0
    assert sorted(t.tree_ids.tolist()) == list(range(n))
    d, ids = t.query(x[n:])
    ref, _ = brute_d2(x[:n], x[n:])
    # exact: the NN distance equals brute force (same fp32 point, recomputed in fp64 here)
    got = ((x[ids] .double() - x[n:].double()) ** 2).sum(-1)
    torch.testing.assert_close(got, ref, rtol=0, atol=0)


def test_exact_ties_total_order():
    # heavy duplicates: integer grid, 3 distinct values per axis
    g = torch.randint(0, 3, (4000, 3)).float()
    t = pk.KDTree.build(g)
    assert t.invariant_violations() == 0
    same = torch.zeros(2000, 2)
    t2 = pk.KDTree.build(same)
    assert t2.invariant_violations() == 0
    # unique tree: permuting the input rows (with ids attached) gives the same tree
    perm = torch.randperm(4000)
    t3 = pk.KDTree.build(g[perm], ids=perm.to(torch.int32))
    assert torch.equal(t3.tree_ids, t.tree_ids)


def test_threaded_build_equals_serial():
    x = pk.generate_problem(3, 3, 200000)
    a = ops.build_cpu(x, None, "exact", 0, 1)
    b = ops.build_cpu(x, None, "exact", 0, 8)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])


def test_reference_mode_quirk_differs_from_exact():
    # the off-by-one sort makes the reference search miss some NNs at low dim
    x = pk.generate_problem(2, 2, 2100)
    tr = pk.KDTree.build(x[:2000], mode="reference")
    te = pk.KDTree.build(x[:2000])
    dr, _ = tr.query(x[2000:])
    de, _ = te.query(x[2000:])
    assert (dr >= de).all()
    assert te.invariant_violations() == 0


def test_depth0_axis_offset():
    x = pk.generate_problem(5, 3, 3000)
    t = pk.KDTree.build(x, depth0=2)
    assert t.invariant_violations() == 0
    assert t.root.axis == 2


def test_save_load_roundtrip(tmp_path):
    x = pk.generate_problem(1, 3, 1000)
    t = pk.KDTree.build(x, id_base=1)
    p = tmp_path / "t.pkd"
    t.save(p)
    u = pk.KDTree.load(p)
    assert torch.equal(u.tree_pts, t.tree_pts) and torch.equal(u.tree_ids, t.tree_ids)
    assert u.mode == "exact" and u.depth0 == 0


def test_point_node_facade():
    x = pk.generate_problem(42, 8, 100)
    t = pk.KDTree.build(x, id_base=1)
    r = t.root
    assert r.slot == 50 and r.left.n == 50 and r.right.n == 49
    p = r.point
    # Node.cpp:16-28 prints at most 5 coordinates then ", , ..., last"
    s = repr(p)
    assert s.startswith(f"Point(ID={p.ID}, dimension=8, coordinates=[") and ", , ..., " in s
    q = pk.Point(8, 101, x[0].numpy())
    nn = pk.nearest_neighbor(r, q)
    assert nn.point.ID == 1 and q.distance(nn.point) == 0.0
    assert pk.Point.compare(pk.Point(2, 0, [1, 2]), pk.Point(2, 1, [2, 0]), 0)


def test_tree_height():
    for n, h in [(0, 0), (1, 1), (2, 2), (3, 2), (4, 3), (1023, 10), (1024, 11), (500000, 19)]:
        assert pk.tree_height(n) == h


def test_cpu_invariant_checker_catches_corruption():
    x = pk.generate_problem(3, 3, 5000)
    t = pk.KDTree.build(x, id_base=1)
    assert t.invariant_violations() == 0
    tp, ti = t.tree_pts.clone(), t.tree_ids.clone()
    tp[[10, 4000]] = tp[[4000, 10]]
    ti[[10, 4000]] = ti[[4000, 10]]
    assert pk.KDTree(tp, ti).invariant_violations() > 0


def test_ab_knobs_need_opt_in(monkeypatch, capfd):
    """A/B tuning knobs (PKD_PAIR, PKD_TOP_Z, ...) change the build only under PKD_AB=1: a stray
    setting is ignored with a note on stderr, so the defaults are what runs."""
    from parallel_kd_tree_amd.ops import native as _ext

    monkeypatch.delenv("PKD_AB", raising=False)
    monkeypatch.setenv("PKD_TOP_Z", "0.5")
    assert _ext().ab_knob("PKD_TOP_Z") is None
    assert "PKD_TOP_Z is an A/B knob" in capfd.readouterr().err
    monkeypatch.setenv("PKD_AB", "1")
    assert _ext().ab_knob("PKD_TOP_Z") == "0.5"
    monkeypatch.delenv("PKD_TOP_Z")
    assert _ext().ab_knob("PKD_TOP_Z") is None


@pytest.mark.parametrize("n,dim", [(200_000, 3), (50_001, 2), (30_000, 128)])
def test_reference_threaded_same_tree(n, dim):
    """The threaded reference-mode builder (children of a sorted segment on two threads) gives
    the single-threaded std::sort tree bit for bit: std::sort is deterministic for one input
    order, and sibling segments are disjoint. The generator's data has ties (it holds ~22.5 M
    distinct values per axis), so this also pins the unstable sort's tie order."""
    x = pk.generate_problem(n + dim, dim, n)
    ids = torch.arange(n, dtype=torch.int32)
    p1, i1 = ops.build_cpu(x, ids, "reference", 0, 1)
    for th in (2, 8, 64):
        pt, it = ops.build_cpu(x, ids, "reference", 0, th)
        assert torch.equal(it, i1) and torch.equal(pt, p1), th


def test_reference_depth0():
    """Reference mode with depth0 > 0 (a subtree of a deeper tree): axis (depth0 + depth) % dim,
    the same as the single-threaded recursion started at that depth."""
    x = pk.generate_problem(5, 3, 10_000)
    ids = torch.arange(10_000, dtype=torch.int32)
    p0, i0 = ops.build_cpu(x, ids, "reference", 0, 1)
    # rotating the columns by depth0 and building at depth 0 is the same split sequence
    p2, i2 = ops.build_cpu(x, ids, "reference", 2, 4)
    xr = x[:, [2, 0, 1]].contiguous()
    pr, ir = ops.build_cpu(xr, ids, "reference", 0, 1)
    assert torch.equal(i2, ir)
    assert not torch.equal(i2, i0)


@pytest.mark.parametrize("n,vals", [(0, 3), (1, 3), (17, 2), (100, 5), (5000, 3), (5000, 10_000), (200_000, 7),
                                    (300_000, 1 << 30), (1_000_003, 1000)])
def test_std_sort_replica_is_bit_exact(n, vals):
    """The parallel replica of libstdc++'s std::sort (introsort) returns std::sort's permutation
    itself -- the order it leaves equal keys in included -- for any thread count. Duplicate-heavy
    keys exercise the unguarded partitions; 2 distinct values drive the heapsort fallback."""
    g = torch.Generator().manual_seed(n + vals)
    keys = torch.randint(0, vals, (n,), generator=g).float()
    ref = ops.native().sort_indices(keys, False, 1)
    for th in (1, 4, 32):
        assert torch.equal(ops.native().sort_indices(keys, True, th), ref), th
    s = keys[ref.long()]
    assert bool((s[1:] >= s[:-1]).all())


def test_std_sort_replica_adversarial_depth_limit():
    """An organ-pipe input (median-of-three killer shape) and all-equal keys: the depth limit's
    heapsort and the unguarded scans both run; still std::sort's exact permutation."""
    n = 1 << 17
    organ = torch.cat([torch.arange(n // 2), torch.arange(n // 2, 0, -1)]).float()
    same = torch.zeros(n)
    for keys in (organ, same, organ.flip(0)):
        ref = ops.native().sort_indices(keys.contiguous(), False, 1)
        assert torch.equal(ops.native().sort_indices(keys.contiguous(), True, 16), ref)


def _tie_segments(x, depth0=0):
    """Median slots of the segments of the reference tree of x whose deciding ranks tie (host
    recursion over the reference's own order, for small inputs)."""
    n, dim = x.shape
    perm = list(range(n))
    out = []

    def rec(lo, m, d):
        if m < 3:
            return
        ax = (depth0 + d) % dim
        seg = sorted(perm[lo:lo + m - 1], key=lambda r: float(x[r, ax]))  # (stable: only the tie set matters)
        k = [float(x[r, ax]) for r in seg]
        h = m // 2
        if k[h - 1] == k[h] or (h >= 2 and k[h - 2] == k[h - 1]) or (h + 1 <= m - 2 and k[h] == k[h + 1]):
            out.append(lo + h)
        perm[lo:lo + m - 1] = seg
        rec(lo, h, d + 1)
        rec(lo + h + 1, m - h - 1, d + 1)

    rec(0, n, 0)
    return out


@pytest.mark.parametrize("n,vals,dim", [(3000, 40, 3), (5000, 9, 2), (2047, 300, 4), (20000, 20000, 3)])
def test_reference_repair_restores_tied_subtrees(n, vals, dim):
    """reference_repair (the hybrid reference mode's host half): given a tree that is right
    everywhere except inside the subtrees of the tied segments (here: the true reference tree with
    every tied subtree's slots scrambled), replaying the ancestors' sorts and the tied subtrees
    with the std::sort replica restores the reference tree exactly, touching only those slots."""
    g = torch.Generator().manual_seed(n * vals + dim)
    x = torch.randint(0, vals, (n, dim), generator=g).float()
    ids = torch.arange(n, dtype=torch.int32)
    _, ref_rows = ops.build_cpu(x, ids, "reference", 0, 1)
    tied = _tie_segments(x)
    assert tied, "the input is meant to have deciding ties"
    bad = ref_rows.clone()
    from parallel_kd_tree_amd.parallel.geometry import segment
    for s in tied:  # scramble the whole subtree of every tied segment (what an arbitrary tie order does)
        h, lo, m = 0, 0, n
        while lo + m // 2 != s:
            h = 2 * h + (1 if s < lo + m // 2 else 2)
            lo, m = segment(n, h)
        bad[lo:lo + m] = bad[lo:lo + m].flip(0)
    perm, slots = ops.native().reference_repair(x, bad, tied, 0, 8)
    assert torch.equal(perm, ref_rows)
    assert slots.numel() > 0
    if n // 2 not in tied:  # (a tied root makes the whole tree the host's)
        assert slots.numel() < n
