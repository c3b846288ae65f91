"""4-level tail (build_global.hip, k_tail3<..., LEV = 4>): at dims 4..8, where one more tail level
turns the plan's trailing pair + triple passes into triples only (100 M x 8D: 2 triples + 2 pairs
-> 3 triples), the last 4 levels of each segment are built by one workgroup in LDS. The tree must
equal the CPU exact tree slot for slot (sizes over the 12 Ki and 16 Ki rows-per-segment shapes,
depth0, explicit ids, ties), and equal the 3-level-tail build (PKD_TAIL4=0) bit for bit."""
import importlib

import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops

pytestmark = pytest.mark.gpu


def _tail_levels(b):
    return sum("tail" in line for line in b.describe().split("\n"))


def _build(x, dev, depth0=0, ids=None):
    b = ops.GpuTreeBuilder(x.shape[0], x.shape[1], depth0, 0)
    tp, ti = b.build(x.to(dev), None if ids is None else ids.to(dev))
    torch.cuda.synchronize()
    return b, tp, ti


@pytest.mark.parametrize("n,dim,depth0,with_ids", [(1_250_000, 4, 0, False), (1_500_001, 5, 3, True),
                                                   (2_000_000, 8, 0, True), (1_750_000, 7, 1, False),
                                                   (8_500_000, 6, 0, False), (10_000_000, 8, 2, False)])
def test_tail4_equals_cpu_exact(gpu_device, n, dim, depth0, with_ids):
    x = pk.generate_problem(n + dim, dim, n)
    ids = torch.randperm(n, generator=torch.Generator().manual_seed(n)).to(torch.int32) * 2 + 1 if with_ids else None
    b, tp, ti = _build(x, gpu_device, depth0, ids)
    assert _tail_levels(b) == 4, b.describe()
    assert b.read_error() == 0, (b.read_error_detail(), b.describe())
    cp, ci = ops.build_cpu(x, ids, "exact", depth0, 8)
    assert torch.equal(ti.cpu(), ci), "GPU tree differs from the CPU exact tree"
    assert torch.equal(tp.cpu(), cp)


@pytest.mark.parametrize("vals", [2, 40])
def test_tail4_ties(gpu_device, vals):
    """Few distinct values: the tail's medians fall inside runs of equal keys (ids decide)."""
    torch.manual_seed(vals)
    x = torch.randint(0, vals, (2_000_000, 6)).float()
    b, tp, ti = _build(x, gpu_device)
    assert _tail_levels(b) == 4, b.describe()
    cp, ci = ops.build_cpu(x, None, "exact", 0, 8)
    if b.read_error() == 0:
        assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)
    tp2, ti2, _ = ops.build_gpu_checked(x.to(gpu_device), None, 0, 0)
    torch.cuda.synchronize()
    assert torch.equal(ti2.cpu(), ci) and torch.equal(tp2.cpu(), cp)


def test_tail4_matches_three_level_tail(gpu_device, monkeypatch):
    """The same 12 M x 8D build with the 4-level tail and with it off: identical trees."""
    x = pk.generate_slice(8, 8, 0, 12_000_000, device=gpu_device)
    b4, tp4, ti4 = _build(x, gpu_device)
    assert _tail_levels(b4) == 4, b4.describe()
    monkeypatch.setenv("PKD_AB", "1")
    monkeypatch.setenv("PKD_TAIL4", "0")
    importlib.import_module("parallel_kd_tree_amd.ops.build")._builders.clear()
    b3, tp3, ti3 = _build(x, gpu_device)
    assert _tail_levels(b3) == 3, b3.describe()
    assert b4.read_error() == 0 and b3.read_error() == 0
    assert torch.equal(ti4, ti3) and torch.equal(tp4, tp3)
    importlib.import_module("parallel_kd_tree_amd.ops.build")._builders.clear()
