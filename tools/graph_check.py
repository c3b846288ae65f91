#!/usr/bin/env python3
"""Capture one build in a hipGraph (torch.cuda.CUDAGraph), replay it and compare with the eager
build, at several sizes. Usage: graph_check.py N [N ...] (default 100000 1000000 12500000).

The builder enqueues a fixed kernel sequence with no host synchronisation and no allocation
(the workspace and the outputs exist before the capture), so a replay must reproduce the
eager tree bit for bit; after each replay the device error word must be 0 and, for the last
size, the replayed input is changed in place and the replay must follow it."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def check(n: int, dim: int = 3) -> None:
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd.ops import GpuTreeBuilder
    dev = torch.device("cuda", 0)
    x = pk.generate_slice(7, dim, 0, n, device=dev)
    b = GpuTreeBuilder(n, dim)
    ep, ei = torch.empty_like(x), torch.empty(n, dtype=torch.int32, device=dev)
    b.build(x, None, 1, ep, ei)  # eager; also allocates the workspace outside the capture
    torch.cuda.synchronize()
    assert b.read_error() == 0
    gp, gi = torch.empty_like(x), torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # the warm-up launch on the capture stream (torch's recipe)
        b.build(x, None, 1, gp, gi)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.build(x, None, 1, gp, gi)
    gp.zero_()
    gi.zero_()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    err = b.read_error()
    same = torch.equal(gi, ei) and torch.equal(gp, ep)
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    t_graph = (time.perf_counter() - t0) / 10 * 1e3
    t0 = time.perf_counter()
    for _ in range(10):
        b.build(x, None, 1, ep, ei)
    torch.cuda.synchronize()
    t_eager = (time.perf_counter() - t0) / 10 * 1e3
    print(f"n={n}: replay {'==' if same else '!='} eager, err={err}, graph {t_graph:.3f} ms, eager {t_eager:.3f} ms",
          flush=True)
    assert same and err == 0
    # the graph reads the input buffer at replay time
    x.copy_(pk.generate_slice(8, dim, 0, n, device=dev))
    g.replay()
    b.build(x, None, 1, ep, ei)
    torch.cuda.synchronize()
    assert torch.equal(gi, ei) and torch.equal(gp, ep), "replay did not follow the new input"
    del g


if __name__ == "__main__":
    sizes = [int(a) for a in sys.argv[1:]] or [100_000, 1_000_000, 12_500_000]
    for n in sizes:
        check(n)
    print("graph check ok", flush=True)
