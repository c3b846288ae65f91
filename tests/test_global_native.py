"""Native global decomposition (csrc/cpu/global_builder.cpp).

CPU: the exchange planner (split sizes per round and peer, collective-consistent geometry
checks, overflow retry signal) against the implicit-tree geometry.
GPU: the whole native builder with P ranks as threads sharing one card through the loopback
communicator (the P > 1 orchestration of kdtree_dist --decomp global without P GPUs): the
assembled tree is slot for slot the single-GPU / CPU exact tree."""
import random

import pytest
import torch

import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops
from parallel_kd_tree_amd.parallel.geometry import segment


def _counts(n_total, P, R, seed):
    """A consistent count matrix [P][R * P][4]: every leaf's rows split at random over the sources."""
    rng = random.Random(seed)
    c = [[[0, 0, 7 + src, 1000 + src] for _ in range(R * P)] for src in range(P)]
    for q in range(P):
        for j in range(R):
            want = segment(n_total, (P + q) * R - 1 + j)[1]
            cuts = sorted(rng.randint(0, want) for _ in range(P - 1))
            parts = [b - a for a, b in zip([0] + cuts, cuts + [want])]
            for src in range(P):
                c[src][j * P + q][0] = parts[src]
    return c


@pytest.mark.parametrize("P,R", [(1, 1), (1, 4), (2, 2), (4, 1), (8, 2)])
def test_native_plan(native, P, R):
    n = 100_003
    c = _counts(n, P, R, P * 10 + R)
    flat = [v for src in c for slot in src for v in slot]
    for me in range(P):
        rc, ins, outs, starts = native.global_plan(flat, P, R, me, n)
        assert rc == 0
        for j in range(R):
            assert ins[j] == [c[me][j * P + p][0] for p in range(P)]
            assert outs[j] == [c[p][j * P + me][0] for p in range(P)]
            assert starts[j + 1] - starts[j] == sum(ins[j])
            assert sum(outs[j]) == segment(n, (P + me) * R - 1 + j)[1]


def test_native_plan_errors(native):
    n, P, R = 5000, 4, 1
    c = _counts(n, P, R, 1)
    c[2][1][1] = 1  # a middle bucket overflowed on rank 2: every rank sees it and retries
    flat = [v for src in c for slot in src for v in slot]
    assert all(native.global_plan(flat, P, R, me, n)[0] == 1 for me in range(P))
    c = _counts(n, P, R, 2)
    c[0][1][0] += 1  # rank 0 claims one row too many for rank 1: every rank raises
    flat = [v for src in c for slot in src for v in slot]
    for me in range(P):
        with pytest.raises(RuntimeError, match="would receive"):
            native.global_plan(flat, P, R, me, n)


@pytest.mark.gpu
@pytest.mark.parametrize("P,k,n,dim", [(1, 0, 100_000, 3), (1, 2, 200_001, 3), (2, -1, 300_000, 3), (4, 0, 250_000, 3),
                                       (4, 1, 120_000, 5), (8, 0, 400_003, 3), (8, 1, 90_000, 2), (4, 0, 7, 3),
                                       (2, 0, 20_000_000, 3), (2, 3, 300_000, 3), (8, 2, 500_000, 3),
                                       (4, 2, 1_000_000, 8), (8, 0, 5, 3), (2, 1, 1, 3), (8, 1, 20, 2)])
def test_native_global_loopback(gpu_device, native, P, k, n, dim):
    x = pk.generate_problem(P + k + 3, dim, n)
    tp, ti, err, scale = native.global_loopback(x, P, k)
    assert err == 0
    # the middle-bucket all-gather slots held every bucket: no overflow retry (uniform data)
    assert scale == 1 or n < 1000
    cp, ci = ops.build_cpu(x, None, "exact", 0, 8)
    assert torch.equal(ti, ci + 1), "native global tree differs from the exact tree"
    assert torch.equal(tp, cp)
