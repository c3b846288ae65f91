"""MFMA candidate filter of the batched brute force (query.hip, namespace mf): bf16 matrix-core
distances with a rigorous error bound select candidates, which are rescored with the exact
sequential fp32 sum. The packed (d2, id) answers must be bit-identical to the VALU brute force
(PKD_BRUTE_MFMA=0) and to a host float32 sequential sum, including ties and the overflow
fallback (more candidates than the list holds)."""
import numpy as np
import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops

pytestmark = pytest.mark.gpu


def _both(pts, q, monkeypatch, ids=None, id_base=0):
    monkeypatch.setenv("PKD_BRUTE_MFMA", "1")
    a = ops.nn_gpu(pts, ids, q, "brute", id_base=id_base)
    monkeypatch.setenv("PKD_BRUTE_MFMA", "0")
    b = ops.nn_gpu(pts, ids, q, "brute", id_base=id_base)
    torch.cuda.synchronize()
    return a.cpu(), b.cpu()


def _host_exact(pts, q, id_base=0):
    """Sequential float32 sum over the coordinates in order, separately rounded (numpy float32
    ops are IEEE single): the reference's distance loop; minimum (d2, id)."""
    p = pts.cpu().numpy().astype(np.float32)
    out = []
    for qi in q.cpu().numpy().astype(np.float32):
        acc = np.zeros(p.shape[0], np.float32)
        for i in range(p.shape[1]):
            t = p[:, i] - qi[i]
            acc = acc + t * t
        m = acc.min()
        j = int(np.flatnonzero(acc == m)[0])
        out.append((float(m), j + id_base))
    return out


@pytest.mark.parametrize("n,dim,nq", [(50_000, 128, 100), (33_333, 32, 16), (20_001, 256, 130), (9_000, 64, 40)])
def test_mfma_equals_exact(gpu_device, monkeypatch, n, dim, nq):
    x = pk.generate_problem(n + dim, dim, n + nq).to(gpu_device)
    a, b = _both(x[:n].contiguous(), x[n:].contiguous(), monkeypatch, id_base=1)
    assert torch.equal(a, b)


def test_mfma_equals_host_sequential_sum(gpu_device, monkeypatch):
    n, dim, nq = 20_000, 128, 20
    x = pk.generate_problem(5, dim, n + nq)
    a, _ = _both(x[:n].to(gpu_device), x[n:].to(gpu_device), monkeypatch, id_base=1)
    d2, ids = ops.unpack(a)
    for k, (m, j) in enumerate(_host_exact(x[:n], x[n:], id_base=1)):
        assert float(d2[k]) == m and int(ids[k]) == j


def test_mfma_explicit_ids(gpu_device, monkeypatch):
    n, dim, nq = 40_000, 64, 50
    x = pk.generate_problem(8, dim, n + nq).to(gpu_device)
    ids = (torch.randperm(n, generator=torch.Generator().manual_seed(2)).to(torch.int32) + 11).to(gpu_device)
    a, b = _both(x[:n].contiguous(), x[n:].contiguous(), monkeypatch, ids=ids)
    assert torch.equal(a, b)


def test_mfma_ties_overflow_fallback(gpu_device, monkeypatch):
    """Every point identical: all are tied candidates, the list overflows, the gated exact
    brute force answers (smallest id among the ties)."""
    n, dim, nq = 10_000, 64, 32
    pts = torch.full((n, dim), 3.25, device=gpu_device)
    q = pk.generate_problem(1, dim, nq).to(gpu_device)
    a, b = _both(pts, q, monkeypatch, id_base=5)
    assert torch.equal(a, b)
    assert torch.all(ops.unpack(a)[1] == 5)


def test_mfma_far_cluster(gpu_device, monkeypatch):
    """Points in a tight cluster far from the origin: the bound is wide, candidates overflow or
    not -- either way the answer is exact."""
    n, dim, nq = 30_000, 32, 24
    g = torch.Generator().manual_seed(4)
    pts = (1.0e4 + torch.rand((n, dim), generator=g)).to(gpu_device)
    q = (1.0e4 + torch.rand((nq, dim), generator=g)).to(gpu_device)
    a, b = _both(pts, q, monkeypatch)
    assert torch.equal(a, b)
