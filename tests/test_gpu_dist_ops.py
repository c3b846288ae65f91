"""The global decomposition's HIP kernels (csrc/gpu/dist_ops.hip) against the torch/numpy
reference path that the multi-process CPU tests validate end to end. The kernels are per-rank
code, so one process checks them; test_gpu_multirank.py runs the whole pipeline with several
ranks sharing the card."""
import numpy as np
import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops
from parallel_kd_tree_amd.parallel.geometry import composite_u64, make_params, segment
from parallel_kd_tree_amd.parallel.global_tree import DONE, _HostOps, _to_rows

pytestmark = pytest.mark.gpu


def _pivots(x, n, dim, levels, seed):
    """Fake but valid pivots: composite keys of random points, per heap node."""
    rng = np.random.default_rng(seed)
    piv = np.zeros(max((1 << levels) - 1, 1), dtype=np.uint64)
    for h in range((1 << levels) - 1):
        i = int(rng.integers(0, n))
        ax = ((h + 1).bit_length() - 1) % dim
        piv[h] = composite_u64(x[i:i + 1, ax].numpy(), np.array([i + 1], dtype=np.uint32))[0]
    return piv


def _cells(nodes_total, dim, seed):
    """Random cells [h][dim][2] shaped like the builder's: a child's cell is its parent's except
    on the parent's split axis (so a node's histogram may be bucketed over its parent's cell)."""
    rng = np.random.default_rng(seed)
    c = np.zeros((nodes_total, dim, 2), dtype=np.float32)
    c[0, :, 0] = rng.uniform(-120, -20, size=dim)
    c[0, :, 1] = rng.uniform(20, 120, size=dim)
    for h in range(1, nodes_total):
        p = (h - 1) // 2
        a = ((p + 1).bit_length() - 1) % dim
        c[h] = c[p]
        c[h, a, 0] = rng.uniform(-120, -20)
        c[h, a, 1] = rng.uniform(20, 120)
    return c


def test_fill_u64_multi(gpu_device):
    """Several fills in one launch: each segment gets its own value, nothing past its end is written."""
    ts = [torch.zeros(n + 3, dtype=torch.int64, device=gpu_device) for n in (1, 6, 4096, 70_001)]
    vals = [0xFFFFFFFF, -1 & 0xFFFFFFFFFFFFFFFF, 0, 0x123456789]
    ops.native().fill_u64_multi([(t, t.numel() - 3, v) for t, v in zip(ts, vals)])
    for t, v in zip(ts, vals):
        h = t.cpu().numpy().view(np.uint64)
        assert (h[:-3] == np.uint64(v)).all() and (h[-3:] == 0).all()


@pytest.mark.parametrize("n,dim", [(123_457, 5), (2_000_003, 3), (1_500_001, 8)])
def test_bbox(gpu_device, n, dim):
    x = pk.generate_problem(3, dim, n)
    x[17, 2] = -0.0
    box = torch.full((2 * dim,), 0xFFFFFFFF, dtype=torch.int64, device=gpu_device)
    nat = ops.native()
    nat.top_bbox(x.to(gpu_device), box)
    cells = torch.zeros(2 * dim, dtype=torch.float32, device=gpu_device)
    nat.top_root_cell(box, dim, cells)
    c = cells.cpu().view(dim, 2)
    assert torch.equal(c[:, 0], x.amin(0)) and torch.equal(c[:, 1], x.amax(0))


@pytest.mark.parametrize("level,dim", [(0, 3), (1, 3), (2, 3), (3, 2), (2, 8)])
def test_route_hist_select_collect_pivot(gpu_device, level, dim):
    n = 60_000
    x = pk.generate_problem(level + 7, dim, n)
    rows = _to_rows(x, None, 1)
    piv = _pivots(x, n, dim, level, level)
    cells = _cells(4 << level, dim, level)
    nat = ops.native()
    xg = x.to(gpu_device)
    node_c = torch.zeros(n, dtype=torch.int64)
    node_g = torch.zeros(n, dtype=torch.int32, device=gpu_device)
    cells_g = torch.from_numpy(cells.reshape(-1).copy()).to(gpu_device)
    piv_g = torch.from_numpy(piv.view(np.int64).copy()).to(gpu_device)
    for l in range(level + 1):
        nl = 1 << l
        bins = 8192 // nl
        axis, prev = l % dim, (l - 1) % dim
        params = np.stack([np.array(make_params(cells[nl - 1 + j, axis, 0], cells[nl - 1 + j, axis, 1], bins))
                           for j in range(nl)]).astype(np.float32)
        hc = _HostOps.route_hist(rows, dim, node_c, l, piv, prev, axis, params, bins)
        hg = torch.zeros(nl * bins, dtype=torch.int32, device=gpu_device)
        nat.top_route_hist(xg, None, 1, node_g, l, piv_g, prev, axis, cells_g, bins, hg)
        assert torch.equal(hc, hg.cpu()), f"histogram mismatch at level {l}"
        if l > 0:
            assert torch.equal(node_c.to(torch.int32), node_g.cpu()), f"routing mismatch at level {l}"
    # select: per node the bucket holding rank size/2 of the (local, here global) histogram
    nl = 1 << level
    bins = 8192 // nl
    hh = hc.numpy().astype(np.int64).reshape(nl, bins)
    sizes = [int(v) for v in hh.sum(1)]
    sel = torch.zeros(128, dtype=torch.int32, device=gpu_device)
    err = torch.zeros(4, dtype=torch.int32, device=gpu_device)
    nat.top_select(hg, level, bins, sizes, sel, err)
    s = sel.cpu().numpy().reshape(32, 4)
    for j in range(nl):
        if sizes[j] == 0:
            continue
        cum = np.cumsum(hh[j])
        b = int(np.searchsorted(cum, sizes[j] // 2, side="right"))
        assert s[j, 0] == b and s[j, 1] == (cum[b - 1] if b else 0) and s[j, 2] == hh[j, b]
    assert int(err[0]) == 0
    # fused collect + route + next histogram, pivot, fix-up (one rank: the gathered buffer is the
    # local one); select zeroes the next histogram and the staging header
    axis, next_axis = level % dim, (level + 1) % dim
    next_bins = 8192 // (2 * nl)
    cap = 8192
    words = nat.top_middle_words(dim, cap)
    buf = torch.full((words,), 7.0, dtype=torch.float32, device=gpu_device)
    hn = torch.full((8192,), 5, dtype=torch.int32, device=gpu_device)
    nat.top_select(hg, level, bins, sizes, sel, err, hn, buf)
    node_f = node_g.clone()
    nat.top_collect_route(xg, None, 1, node_f, level, axis, next_axis, cells_g, bins, next_bins, sel, buf, cap, hn)
    staged = int(buf[:1].view(torch.int32).item())
    assert staged == int(sel.cpu().view(32, 4)[:nl, 2].sum()), "staged rows differ from the median buckets' counts"
    pivots = torch.full((2 * nl,), -1, dtype=torch.int64, device=gpu_device)
    top_rows = torch.zeros((2 * nl, dim + 1), dtype=torch.float32, device=gpu_device)
    cg = cells_g.clone()
    nat.top_pivot(buf, 1, cap, level, axis, dim, sizes, sel, pivots, top_rows, cg, err)
    assert int(err[0]) == 0
    nat.top_fixup(buf, cap, dim, level, axis, next_axis, pivots, cg, next_bins, node_f, hn)
    pv = pivots.cpu().numpy().view(np.uint64)
    ids = np.arange(1, n + 1, dtype=np.uint32)
    nodes_np = node_c.numpy()
    for j in range(nl):
        h = nl - 1 + j
        mask = (nodes_np == h) if level > 0 else np.ones(n, bool)
        if sizes[j] == 0:
            assert pv[h] == np.uint64(0xFFFFFFFFFFFFFFFF)
            continue
        keys = np.sort(composite_u64(x.numpy()[mask, axis], ids[mask]))
        assert pv[h] == keys[sizes[j] // 2], f"node {h}: wrong pivot"
        i = int(pv[h] & np.uint64(0xFFFFFFFF)) - 1
        tr = top_rows.cpu()[h]
        assert torch.equal(tr[:dim], x[i]) and int(tr[dim].view(torch.int32)) == i + 1
        c = cg.cpu().view(-1, dim, 2)
        assert float(c[2 * h + 1, axis, 1]) == float(x[i, axis]) and float(c[2 * h + 2, axis, 0]) == float(x[i, axis])
    # every point routed below its pivot, and the next level's histogram, as the host path does it
    nl2 = 2 * nl
    params2 = np.stack([np.array(make_params(cells[nl2 - 1 + j, next_axis, 0], cells[nl2 - 1 + j, next_axis, 1],
                                             next_bins)) for j in range(nl2)]).astype(np.float32)
    hc2 = _HostOps.route_hist(rows, dim, node_c, level + 1, pv, axis, next_axis, params2, next_bins)
    assert torch.equal(node_c.to(torch.int32), node_f.cpu()), "fused routing differs from the host routing"
    assert torch.equal(hc2, hn.cpu()[: nl2 * next_bins]), "fused next-level histogram differs"


@pytest.mark.parametrize("P,dim", [(2, 3), (4, 3), (8, 3), (8, 5)])
def test_pack_matches_host(gpu_device, P, dim):
    n = 100_000
    L = P.bit_length() - 1
    x = pk.generate_problem(P, dim, n)
    rows = _to_rows(x, None, 1)
    piv = _pivots(x, n, dim, L, P)
    nat = ops.native()
    node_c = torch.zeros(n, dtype=torch.int64)
    node_g = torch.zeros(n, dtype=torch.int32, device=gpu_device)
    xg = x.to(gpu_device)
    piv_g = torch.from_numpy(piv.view(np.int64).copy()).to(gpu_device)
    cells_g = torch.from_numpy(np.tile(np.array([-100, 100], np.float32), 2 * P * dim)).to(gpu_device)
    for l in range(L):
        nl = 1 << l
        pr = np.tile(np.array(make_params(-100, 100, 8192 // nl), dtype=np.float32), (nl, 1))
        _HostOps.route_hist(rows, dim, node_c, l, piv, (l - 1) % dim, l % dim, pr, 8192 // nl)
        hg = torch.zeros(8192, dtype=torch.int32, device=gpu_device)
        nat.top_route_hist(xg, None, 1, node_g, l, piv_g, (l - 1) % dim, l % dim, cells_g, 8192 // nl, hg)
    sc, cc = _HostOps.pack(rows, dim, node_c, L, piv, (L - 1) % dim)
    # top_pack takes the nodes as the (fused) top levels leave them: routed to the leaves
    node_g = node_c.to(torch.int32).to(gpu_device)
    out = torch.empty((n, dim + 1), dtype=torch.float32, device=gpu_device)
    counts = torch.empty(4 * P, dtype=torch.int64, device=gpu_device)
    err = torch.zeros(4, dtype=torch.int32, device=gpu_device)
    scratch = torch.empty(nat.top_pack_scratch_bytes(n, P), dtype=torch.uint8, device=gpu_device)
    node_keep = node_g.clone()
    node_keep2 = node_g.clone()
    nat.top_pack(xg, None, 1, node_g, L, out, 0, None, counts, err, scratch)
    cg = counts.cpu().view(P, 4)
    assert torch.equal(cc, cg[:, 0]) and int(cg[:, 1].abs().sum()) == 0
    k = int(cc.sum())
    assert torch.equal(sc.view(torch.int32), out[:k].cpu().view(torch.int32)), "pack must be stable by destination"

    # planar output (SoA planes of a padded stride): the same rows, column by column
    stride = n + 61
    planes = torch.full((dim * stride,), -7.0, dtype=torch.float32, device=gpu_device)
    nat.top_pack(xg, None, 1, node_keep2, L, planes, stride, None, counts, err, scratch)
    pl = planes.cpu().view(dim, stride)
    assert torch.equal(pl[:, :k].t().contiguous(), sc[:, :dim])

    # compact exchange: coordinates only + destination bitmaps; ids rebuilt on the receiver side
    words = (n + 31) // 32
    bm = torch.full((P, words), -1, dtype=torch.int32, device=gpu_device)
    outc = torch.empty((n, dim), dtype=torch.float32, device=gpu_device)
    nat.top_pack(xg, None, 1, node_keep, L, outc, 0, bm, counts, err, scratch)
    assert torch.equal(outc[:k].cpu(), sc[:, :dim])
    dest = node_keep.cpu().to(torch.int64) - (P - 1)
    bits = ((bm.cpu().to(torch.int64) & 0xFFFFFFFF)[:, :, None] >> torch.arange(32)) & 1
    bits = bits.reshape(P, -1)
    for d in range(P):
        assert torch.equal(bits[d, :n].bool(), dest == d) and int(bits[d, n:].sum()) == 0
    # the receiver: every source is this same rank here, with its own id base
    bases = [1 + 1000 * s for s in range(P)]
    off = [0] + np.cumsum(cc.tolist())[:-1].tolist()
    rows_per = cc.tolist()
    # bitmap of source s for receiver d: here receiver d == s's row of the bitmap block
    recv_bm = torch.cat([bm[d, :words] for d in range(P)])
    ids = torch.full((k,), -1, dtype=torch.int32, device=gpu_device)
    scr = torch.empty(nat.ids_from_bitmaps_scratch_bytes(words, P), dtype=torch.uint8, device=gpu_device)
    err.zero_()
    nat.ids_from_bitmaps(recv_bm, off, rows_per, [d * words for d in range(P)], [words] * P, bases, ids, scr, err)
    want = torch.cat([torch.nonzero(dest == d).flatten() + bases[d] for d in range(P)]).to(torch.int32)
    assert int(err.cpu()[0]) == 0
    assert torch.equal(ids.cpu(), want)


def test_explicit_ids(gpu_device):
    """Explicit id arrays route ties by id exactly like implicit ones (level 0 of the fused top
    levels: histogram, select, staging, pivot, fix-up), and the pack counts the two leaves."""
    n, dim = 20_000, 2
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 4, (n, dim), generator=g).float()  # massive ties
    ids = torch.randperm(n, generator=g).to(torch.int32) + 10
    rows = torch.cat([x, ids.view(torch.float32)[:, None]], 1)
    keys = composite_u64(x[:, 0].numpy(), ids.numpy().view(np.uint32))
    piv = np.array([np.sort(keys)[n // 2]], dtype=np.uint64)
    node_c = torch.zeros(n, dtype=torch.int64)
    _HostOps.pack(rows, dim, node_c, 1, piv, 0)
    nat = ops.native()
    xg, ig = x.to(gpu_device), ids.to(gpu_device)
    node_g = torch.zeros(n, dtype=torch.int32, device=gpu_device)
    cells = torch.tensor([-1.0, 5.0, -1.0, 5.0] * 3, dtype=torch.float32, device=gpu_device)
    hist = torch.zeros(8192, dtype=torch.int32, device=gpu_device)
    nat.top_route_hist(xg, ig, 0, node_g, 0, torch.zeros(1, dtype=torch.int64, device=gpu_device), 0, 0, cells, 8192,
                       hist)
    sel = torch.zeros(128, dtype=torch.int32, device=gpu_device)
    err = torch.zeros(4, dtype=torch.int32, device=gpu_device)
    cap = n
    buf = torch.empty(nat.top_middle_words(dim, cap), dtype=torch.float32, device=gpu_device)
    nat.top_select(hist, 0, 8192, [n], sel, err, None, buf)
    nat.top_collect_route(xg, ig, 0, node_g, 0, 0, 1, cells, 8192, 4096, sel, buf, cap, None)
    pivots = torch.full((2,), -1, dtype=torch.int64, device=gpu_device)
    top_rows = torch.zeros((2, dim + 1), dtype=torch.float32, device=gpu_device)
    nat.top_pivot(buf, 1, cap, 0, 0, dim, [n], sel, pivots, top_rows, cells, err)
    nat.top_fixup(buf, cap, dim, 0, 0, 1, pivots, cells, 4096, node_g, None)
    assert int(err[0]) == 0 and int(pivots[0]) == int(piv.view(np.int64)[0])
    assert torch.equal(node_c.to(torch.int32), node_g.cpu())
    out = torch.empty((n, dim + 1), dtype=torch.float32, device=gpu_device)
    counts = torch.empty(8, dtype=torch.int64, device=gpu_device)
    scratch = torch.empty(nat.top_pack_scratch_bytes(n, 2), dtype=torch.uint8, device=gpu_device)
    nat.top_pack(xg, ig, 0, node_g, 1, out, 0, None, counts, err, scratch)
    assert counts.cpu()[0::4].tolist() == [n // 2, n - n // 2 - 1]


def test_build_rows_equals_build(gpu_device):
    x = pk.generate_problem(4, 3, 200_000)
    ids = torch.arange(200_000, dtype=torch.int32) * 3 + 7
    b = ops.GpuTreeBuilder(200_000, 3, 2)
    rows = torch.cat([x, ids.view(torch.float32)[:, None]], 1).to(gpu_device)
    tp, ti = b.build_rows(rows)
    cp, ci = ops.build_cpu(x, ids, "exact", 2, 4)
    assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("P", [2, 8])
def test_pack_empty_rank_zeroes_bitmaps(gpu_device, P):
    """A rank with no rows (N < P) still sends one bitmap word per leaf: the pack must write it
    (zero), whatever the buffer held before, so the receiver's id rebuild sees no stray bits."""
    L = P.bit_length() - 1
    nat = ops.native()
    x = torch.empty((0, 3), dtype=torch.float32, device=gpu_device)
    node = torch.empty(0, dtype=torch.int32, device=gpu_device)
    outc = torch.empty((1, 3), dtype=torch.float32, device=gpu_device)
    counts = torch.empty(4 * P, dtype=torch.int64, device=gpu_device)
    err = torch.zeros(4, dtype=torch.int32, device=gpu_device)
    scratch = torch.empty(max(1, nat.top_pack_scratch_bytes(0, P)), dtype=torch.uint8, device=gpu_device)
    bm = torch.full((P, 1), -1, dtype=torch.int32, device=gpu_device)  # poisoned: every bit set
    nat.top_pack(x, None, 1, node, L, outc, 0, bm, counts, err, scratch)
    torch.cuda.synchronize()
    assert int(bm.abs().sum()) == 0, bm
    assert int(counts.cpu().view(P, 4)[:, 0].sum()) == 0
