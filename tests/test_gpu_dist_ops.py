"""The global decomposition's HIP kernels (csrc/gpu/dist_ops.hip) against the torch reference
ops that the multi-process CPU tests validate end to end. Single GPU: ranks are not needed to
check the per-rank kernels; the 8-GPU path is exercised by the driver's scaling run."""
import numpy as np
import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd.parallel.geometry import composite_u64, make_params
from parallel_kd_tree_amd.parallel.global_tree import _Backend, _to_rows

pytestmark = pytest.mark.gpu


def _setup(n, dim, level, seed=1):
    x = pk.generate_problem(seed, dim, n)
    rows = _to_rows(x, None, 1)
    nodes = 1 << level
    first = nodes - 1
    # fake pivots: medians of random subsets per heap node (exact composite keys of points)
    rng = np.random.default_rng(seed)
    piv = np.zeros(max(2 * nodes - 1, 1), dtype=np.uint64)
    for h in range(first):
        i = int(rng.integers(0, n))
        ax = ((h + 1).bit_length() - 1) % dim
        piv[h] = composite_u64(x[i:i + 1, ax].numpy(), np.array([i + 1], dtype=np.uint32))[0]
    return x, rows, piv


@pytest.mark.parametrize("level,dim", [(0, 3), (1, 3), (2, 3), (3, 2), (2, 8)])
def test_route_hist_matches_cpu(gpu_device, level, dim):
    n = 50_000
    x, rows, piv = _setup(n, dim, level)
    nodes = 1 << level
    bins = 8192 // nodes
    params = np.stack([np.array(make_params(-100.0 + j, 100.0 - j, bins)) for j in range(nodes)]).astype(np.float32)
    cpu, gpu = _Backend(torch.device("cpu")), _Backend(gpu_device)
    axis, prev = level % dim, (level - 1) % dim
    # route down to `level` one level at a time on both backends
    node_c = torch.zeros(n, dtype=torch.int64)
    node_g = torch.zeros(n, dtype=torch.int32, device=gpu_device)
    rows_g = rows.to(gpu_device)
    for l in range(level + 1):
        nl = 1 << l
        b = 8192 // nl
        pr = np.stack([np.array(make_params(-100.0 + j, 100.0 - j, b)) for j in range(nl)]).astype(np.float32)
        hc = cpu.route_hist(rows, dim, node_c, l, piv, (l - 1) % dim, l % dim, pr, b)
        hg = gpu.route_hist(rows_g, dim, node_g, l, piv, (l - 1) % dim, l % dim, pr, b)
        assert torch.equal(hc, hg.cpu()), f"histogram mismatch at level {l}"
        assert torch.equal(node_c.to(torch.int32), node_g.cpu()), f"routing mismatch at level {l}"
    bstar = np.array([int(torch.argmax(hc[j * bins:(j + 1) * bins])) for j in range(nodes)])
    mc = cpu.collect_middle(rows, dim, node_c, level, axis, params, bins, bstar)
    mg = gpu.collect_middle(rows_g, dim, node_g, level, axis, params, bins, bstar).cpu()
    key = lambda m: sorted(map(tuple, m.view(torch.int32).tolist()))
    assert key(mc) == key(mg)


@pytest.mark.parametrize("P,dim", [(2, 3), (4, 3), (8, 3), (8, 5)])
def test_pack_matches_cpu(gpu_device, P, dim):
    n = 100_000
    L = P.bit_length() - 1
    x, rows, piv = _setup(n, dim, L, seed=P)
    cpu, gpu = _Backend(torch.device("cpu")), _Backend(gpu_device)
    # nodes at level L-1: route from the root with the fake pivots
    node_c = torch.zeros(n, dtype=torch.int64)
    node_g = torch.zeros(n, dtype=torch.int32, device=gpu_device)
    rows_g = rows.to(gpu_device)
    for l in range(L):
        nl = 1 << l
        pr = np.tile(np.array(make_params(-100, 100, 8192 // nl), dtype=np.float32), (nl, 1))
        cpu.route_hist(rows, dim, node_c, l, piv, (l - 1) % dim, l % dim, pr, 8192 // nl)
        gpu.route_hist(rows_g, dim, node_g, l, piv, (l - 1) % dim, l % dim, pr, 8192 // nl)
    sc, cc = cpu.pack(rows, dim, node_c, L, piv, (L - 1) % dim, P)
    sg, cg = gpu.pack(rows_g, dim, node_g, L, piv, (L - 1) % dim, P)
    assert torch.equal(cc, cg.cpu())
    assert torch.equal(sc.view(torch.int32), sg.cpu().view(torch.int32)), "pack must be stable by destination"


def test_build_rows_equals_build(gpu_device):
    from parallel_kd_tree_amd import ops
    x = pk.generate_problem(4, 3, 200_000)
    ids = torch.arange(200_000, dtype=torch.int32) * 3 + 7
    b = ops.GpuTreeBuilder(200_000, 3, 2)
    rows = torch.cat([x, ids.view(torch.float32)[:, None]], 1).to(gpu_device)
    tp, ti = b.build_rows(rows)
    cp, ci = ops.build_cpu(x, ids, "exact", 2, 4)
    assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)
