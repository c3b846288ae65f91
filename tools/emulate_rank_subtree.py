#!/usr/bin/env python3
"""CPU emulation of k_subtree_rank (csrc/gpu/build_subtree.hip): same per-level decisions
(bucket ranking on an axis' first use, compressed-rank bitmaps afterwards, same widths and
mode switches), checked against the exact CPU builder. Debug aid, not used by the package."""
import sys

import numpy as np


def orderable(x):
    b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return np.where(b & 0x80000000, (~b) & 0xFFFFFFFF, b | 0x80000000)


def pow2_ceil(v):
    return 1 if v <= 1 else 1 << (int(v) - 1).bit_length()


def emulate(pts, ids, depth_base, NM=2048):
    n, dim = pts.shape
    lsub = n.bit_length()
    keep = dim < lsub
    crank = np.zeros((dim, n), np.int64)
    lo = np.zeros(n, np.int64); nn = np.full(n, n, np.int64); sg = np.zeros(n, np.int64)
    fin = np.full(n, -1, np.int64)
    modes = []
    for t in range(lsub):
        axis = (depth_base + t) % dim
        S = 1 << t
        Wt = 0
        if keep and t >= dim:
            wbits = n >> (t - dim + 1)
            words = pow2_ceil((wbits + 31) // 32)
            if words <= 64 and S * words <= NM:
                Wt = words
        live = np.nonzero(nn)[0]
        rank = np.zeros(n, np.int64)
        if Wt:
            modes.append(f"b{Wt}")
            c = crank[axis]
            for p in live:
                same = live[sg[live] == sg[p]]
                assert len(set(c[same].tolist())) == len(same), "compressed ranks collide"
                assert c[p] < Wt * 32, "compressed rank exceeds bitmap width"
                rank[p] = int(np.sum(c[same] < c[p]))
        else:
            modes.append("h")
            ok = orderable(pts[:, axis])
            for p in live:
                same = live[sg[live] == sg[p]]
                rank[p] = int(np.sum((ok[same] < ok[p]) | ((ok[same] == ok[p]) & (ids[same] < ids[p]))))
        for p in live:
            mid = nn[p] // 2
            r = rank[p]
            if r == mid:
                fin[lo[p] + mid] = p
                nn[p] = 0
                continue
            if r < mid:
                sg[p] = 2 * sg[p]; nn[p] = mid; nc = r
            else:
                sg[p] = 2 * sg[p] + 1; lo[p] += mid + 1; nn[p] -= mid + 1; nc = r - mid - 1
            crank[axis, p] = nc
    assert (fin >= 0).all()
    return fin, modes


def main():
    sys.path.insert(0, ".")
    import torch
    from parallel_kd_tree_amd import ops
    rng = np.random.default_rng(0)
    for n, dim, db in [(1526, 3, 16), (2048, 3, 0), (1000, 2, 5), (777, 4, 3), (300, 8, 1), (5, 3, 2), (1, 3, 0),
                       (2047, 1, 0)]:
        pts = rng.uniform(-1, 1, size=(n, dim)).astype(np.float32)
        pts[::7, 0] = 0.25  # ties
        ids = rng.permutation(n).astype(np.uint32) + 3
        fin, modes = emulate(pts, ids, db)
        cp, ci = ops.build_cpu(torch.from_numpy(pts), torch.from_numpy(ids.view(np.int32)), "exact", db, 1)
        ok = np.array_equal(ids[fin].view(np.int32), ci.numpy())
        print(n, dim, db, "OK" if ok else "MISMATCH", " ".join(modes))
        assert ok


if __name__ == "__main__":
    main()
