"""Sampled triples (build_global.hip, k_g3_*): a triple's pivots of levels l and l+1 come from a
per-segment sample, the rows the estimate cannot place are staged and resolved exactly. The tree
must equal the CPU exact tree slot for slot (sizes, dims 2..8, depth0, explicit ids, sorted input,
duplicates); a band that misses its median is reported (error bit 0x20), never silent, and the
checked entry points rebuild unsampled. The knobs below push the sampled triples down to small
builds (they start at 128 segments of >= 256 Ki rows by default)."""
import importlib

import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture
def g3_small(monkeypatch):
    monkeypatch.setenv("PKD_AB", "1")  # A/B knobs below
    monkeypatch.setenv("PKD_G3_MIN_SEGS", "4")
    monkeypatch.setenv("PKD_G3_MIN_N", "0")
    monkeypatch.setenv("PKD_G3_MAX_DIM", "8")
    monkeypatch.setenv("PKD_G3_MIN_ROWS", "4096")
    monkeypatch.setenv("PKD_G3_SAMPLE", "8192")
    importlib.import_module("parallel_kd_tree_amd.ops.build")._builders.clear()
    yield
    importlib.import_module("parallel_kd_tree_amd.ops.build")._builders.clear()


def _build(x, dev, depth0=0, ids=None):
    b = ops.GpuTreeBuilder(x.shape[0], x.shape[1], depth0, 0)
    tp, ti = b.build(x.to(dev), None if ids is None else ids.to(dev))
    torch.cuda.synchronize()
    return b, tp, ti


def _same_as_cpu(x, dev, depth0=0, ids=None):
    b, tp, ti = _build(x, dev, depth0, ids)
    assert " g3" in b.describe() and b.sampled, b.describe()
    assert b.read_error_detail()[0] == 0, (b.read_error_detail(), b.describe())
    cp, ci = ops.build_cpu(x, ids, "exact", depth0, 8)
    assert torch.equal(ti.cpu(), ci), "GPU tree differs from the CPU exact tree"
    assert torch.equal(tp.cpu(), cp)
    return b


@pytest.mark.parametrize("multi", ["1", "1024"])  # resolve: one workgroup per node / K blocks per node
@pytest.mark.parametrize("n,dim,depth0", [(2_000_000, 3, 0), (1_500_001, 2, 1), (1_000_003, 5, 0),
                                          (800_000, 8, 2), (3_000_000, 4, 3), (2_500_000, 7, 0),
                                          (1_000_000, 6, 5)])
def test_g3_equals_cpu_exact(gpu_device, g3_small, monkeypatch, n, dim, depth0, multi):
    monkeypatch.setenv("PKD_G3_MULTI_BELOW", multi)
    b = _same_as_cpu(pk.generate_problem(n + 7 * dim, dim, n), gpu_device, depth0)
    lvl, segs = b.g3_report()
    assert sum(s[0] for s in segs) > 0 and not any(s[24] for s in segs)
    for s in segs:  # every row is certain or staged; the staged ones were all inserted
        assert sum(s[8:16]) + sum(s[16:24]) + 7 == s[0] or s[0] == 0, s


# k_g3_part stores: from registers / LDS tile in 1 / 2 parts; rows of >= 6 columns: 4 or 8 per thread
@pytest.mark.parametrize("stage,wide", [("0", "4"), ("1", "4"), ("2", "4"), ("2", "8")])
@pytest.mark.parametrize("n,dim,depth0", [(2_000_000, 3, 0), (1_000_003, 5, 1), (900_001, 6, 0), (800_000, 8, 2)])
def test_g3_ballot_ranks_staged_stores(gpu_device, g3_small, monkeypatch, n, dim, depth0, stage, wide):
    """The ballot-rank form of the pass (the default from 64 M points) with its stores staged
    through LDS in zone order: the same exact tree."""
    monkeypatch.setenv("PKD_PART3_ATOMIC", "0")
    monkeypatch.setenv("PKD_G3_STAGE", stage)
    monkeypatch.setenv("PKD_WIDE_KI", wide)
    ids = torch.randperm(n, generator=torch.Generator().manual_seed(n)).to(torch.int32) + 3
    _same_as_cpu(pk.generate_problem(n + 11 * dim, dim, n), gpu_device, depth0, ids)


def test_g3_explicit_ids(gpu_device, g3_small):
    n = 2_000_000
    x = pk.generate_problem(78, 3, n)
    ids = torch.randperm(n, dtype=torch.int64).to(torch.int32) * 3 + 11
    _same_as_cpu(x, gpu_device, 0, ids)


def test_g3_sorted_and_constant_axis(gpu_device, g3_small):
    x = pk.generate_problem(19, 3, 2_000_000)
    _same_as_cpu(x[torch.argsort(x[:, 1])].contiguous(), gpu_device)  # sorted on a triple's axis
    y = pk.generate_problem(20, 3, 2_000_000)
    y[:, 2] = -3.0                                                      # a constant axis
    b, tp, ti = _build(y, gpu_device)
    _check_or_rebuilt(b, y, gpu_device, tp, ti)


def _check_or_rebuilt(b, x, dev, tp, ti, depth0=0):
    """A sampled build either succeeds exactly or reports a miss; the checked path is exact."""
    err = b.read_error()
    cp, ci = ops.build_cpu(x, None, "exact", depth0, 8)
    if err == 0:
        assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)
    else:
        assert err & ops.GpuTreeBuilder.TOP_BAND_MISS, err  # (later levels may flag the garbage too)
    tp2, ti2, _ = ops.build_gpu_checked(x.to(dev), None, 0, depth0)
    torch.cuda.synchronize()
    assert torch.equal(ti2.cpu(), ci) and torch.equal(tp2.cpu(), cp)


@pytest.mark.parametrize("multi", ["1", "1024"])
@pytest.mark.parametrize("vals", [3, 200, 100_000])
def test_g3_duplicates(gpu_device, g3_small, monkeypatch, vals, multi):
    """Few distinct values: bands hold whole runs of equal keys (a region may overflow: then the
    miss is reported and the checked build is exact)."""
    monkeypatch.setenv("PKD_G3_MULTI_BELOW", multi)
    torch.manual_seed(vals)
    x = torch.randint(0, vals, (2_000_000, 3)).float()
    b, tp, ti = _build(x, gpu_device)
    _check_or_rebuilt(b, x, gpu_device, tp, ti)


@pytest.mark.parametrize("multi", ["1", "1024"])
def test_g3_band_miss_detected_and_rebuilt(gpu_device, g3_small, monkeypatch, multi):
    """Bands far too narrow (z = 0.01): the build must REPORT the miss (bit 0x20), complete
    without a fault, and KDTree.build must rebuild it exactly."""
    monkeypatch.setenv("PKD_G3_Z", "0.01")
    monkeypatch.setenv("PKD_G3_MULTI_BELOW", multi)
    x = pk.generate_problem(23, 3, 2_000_000)
    b, tp, ti = _build(x, gpu_device)
    assert b.read_error() & ops.GpuTreeBuilder.TOP_BAND_MISS
    importlib.import_module("parallel_kd_tree_amd.ops.build")._builders.clear()
    t = pk.KDTree.build(x.to(gpu_device))
    t.check()
    cp, ci = ops.build_cpu(x, None, "exact", 0, 8)
    assert torch.equal(t.tree_ids.cpu(), ci)


@pytest.mark.parametrize("z", ["6", "0.01"])
def test_g3_from_columns_keeps_them(gpu_device, g3_small, monkeypatch, z):
    """build_columns (the distributed leaves' layout): a sampled-triple build runs on a copy, so
    the caller's columns survive for a rebuild after a miss."""
    monkeypatch.setenv("PKD_G3_Z", z)
    n, dim, depth0 = 2_000_000, 3, 2
    x = pk.generate_problem(31, dim, n)
    ids = torch.randperm(n, generator=torch.Generator().manual_seed(5)).to(torch.int32) + 1
    b = ops.GpuTreeBuilder(n, dim, depth0, 0)
    assert b.sampled and not b.sampled_top, b.describe()
    cols = torch.zeros((dim + 1, b.column_stride), dtype=torch.float32, device=gpu_device)
    cols[:dim, :n] = x.t().to(gpu_device)
    cols[dim, :n] = ids.to(gpu_device).view(torch.float32)
    keep = cols.clone()
    tp, ti = b.build_columns(cols)
    torch.cuda.synchronize()
    assert torch.equal(cols, keep), "a sampled-triple build clobbered the caller's columns"
    cp, ci = ops.build_cpu(x, ids, "exact", depth0, 8)
    if z == "6":
        assert b.read_error() == 0
    else:
        assert b.read_error() & ops.GpuTreeBuilder.TOP_BAND_MISS
        fb = ops.GpuTreeBuilder(n, dim, depth0, 0, allow_top=False)
        assert not fb.sampled
        tp, ti = fb.build_columns(cols)
        torch.cuda.synchronize()
        assert fb.read_error() == 0
    assert torch.equal(ti.cpu(), ci) and torch.equal(tp.cpu(), cp)


def test_g3_default_40m_equals_unsampled(gpu_device):
    """Default knobs at 40 M points: the triple at level 7 samples; the tree equals the build
    with every sampling off, slot for slot."""
    x = pk.generate_slice(4, 3, 0, 40_000_000, device=gpu_device)
    b = ops.GpuTreeBuilder(x.shape[0], 3, 0, 0)
    assert " g3" in b.describe(), b.describe()
    tp, ti = b.build(x, None, 1)
    b0 = ops.GpuTreeBuilder(x.shape[0], 3, 0, 0, allow_top=False)
    assert not b0.sampled
    tp0, ti0 = b0.build(x, None, 1)
    torch.cuda.synchronize()
    assert b.read_error() == 0 and b0.read_error() == 0
    assert torch.equal(ti, ti0) and torch.equal(tp, tp0)


@pytest.mark.parametrize("multi", ["1", "1024"])
def test_g3_across_second_stage_levels(gpu_device, g3_small, monkeypatch, multi):
    """Levels whose median bucket would take a second-stage histogram (the 1 B build's levels 4-7)
    still sample their triples: level l's bucket rows are ranked exactly among the staged rows,
    levels l+1 and l+2 need no histogram at all (PKD_STAGE2_MIN pushes the second stage down to
    this size)."""
    monkeypatch.setenv("PKD_STAGE2_MIN", "4")
    monkeypatch.setenv("PKD_G3_MULTI_BELOW", multi)
    b = _same_as_cpu(pk.generate_problem(99, 3, 2_000_000), gpu_device)
    assert " stage2" in b.describe(), b.describe()
