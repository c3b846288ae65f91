#!/usr/bin/env python3
"""Step through level 0 of the distributed top levels on one rank (the ops of dist_ops.hip) and print
the selected median bucket, the collected middle rows and the pivot kernel's verdict."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parallel_kd_tree_amd as pk
from parallel_kd_tree_amd import ops
nat = ops.native()
n, dim = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000, 3
dev = torch.device("cuda:0")
x = pk.generate_slice(42, dim, 0, n, device=dev)
box = torch.full((2 * dim,), 0xFFFFFFFF, dtype=torch.int64, device=dev)
nat.top_bbox(x, box)
cells = torch.zeros(15 * dim * 2, dtype=torch.float32, device=dev)
nat.top_root_cell(box, dim, cells)
ref_lo, ref_hi = x.min(0).values, x.max(0).values
print("cell", cells[: 2 * dim].view(dim, 2).tolist(), "true", ref_lo.tolist(), ref_hi.tolist())
node = torch.zeros(n, dtype=torch.int32, device=dev)
pivots = torch.full((7,), -1, dtype=torch.int64, device=dev)
hist = torch.zeros(8192, dtype=torch.int32, device=dev)
nat.top_route_hist(x, None, 1, node, 0, pivots, 0, 0, cells, 8192, hist)
err = torch.zeros(4, dtype=torch.int32, device=dev)
sel = torch.zeros(128, dtype=torch.int32, device=dev)
nat.top_select(hist, 0, 8192, [n], sel, err)
print("hist sum", int(hist.sum()), "max", int(hist.max()), "sel", sel[:4].tolist(), "err", err.tolist())
cap = 4580
words = nat.top_middle_words(dim, cap)
buf = torch.zeros(words, dtype=torch.float32, device=dev)
nat.top_collect(x, None, 1, node, 0, 0, cells, 8192, sel, buf, cap)
print("collected header", buf[:4].view(torch.int32).tolist())
top_rows = torch.zeros(7, dim + 1, dtype=torch.float32, device=dev)
nat.top_pivot(buf, 1, cap, 0, 0, dim, [n], sel, pivots, top_rows, cells, err)
torch.cuda.synchronize()
print("pivot", hex(int(pivots[0]) & 0xFFFFFFFFFFFFFFFF), "err", err.tolist(), "row", top_rows[0].tolist())
