"""Problem generation.

``generate_problem`` / ``generate_slice`` reproduce the reference data bit for bit:
``std::mt19937(seed)`` + ``std::uniform_real_distribution<float>(-100, 100)``, row-major,
(Utility.cpp:6-18), including per-rank slices (kdtree_mpi.cpp:19-41) reached by an O(log)
jump-ahead instead of ``discard`` (csrc/cpu/generator.cpp).

``generate_slice(..., device="cuda")`` produces the same bits on the GPU (csrc/gpu/generator.hip):
chunked mt19937 with device-side jump-ahead rounds, no serial walk over the stream.

``uniform_points`` is the fast on-device synthetic generator for benchmarks: a different
random stream, but the same value map (``float(u32) / 2^32`` clamped below 1, ``*200 - 100``)
so values take the same ~22.5 M distinct levels per axis (ties as in the reference data).
"""
from __future__ import annotations

import torch

from ..ops import native


def generate_problem(seed: int, dim: int, num_points: int, threads: int = 0) -> torch.Tensor:
    """Rows 0..num_points-1 of the reference stream (CPU float32 [num_points, dim])."""
    return native().generate(int(seed), int(dim), int(num_points), 0, int(threads))


def generate_slice(seed: int, dim: int, first: int, rows: int, threads: int = 0, device=None) -> torch.Tensor:
    """Rows first..first+rows-1 of the reference stream (on `device` if it is a GPU)."""
    if device is not None and torch.device(device).type == "cuda":
        out = torch.empty((int(rows), int(dim)), dtype=torch.float32, device=device)
        return native().generate_gpu(int(seed), int(first), out)
    return native().generate(int(seed), int(dim), int(rows), int(first), int(threads))


def generate_emulated(seed: int, dim: int, first: int, rows: int) -> torch.Tensor:
    """The device generator's algorithm (chunk plan, jump rounds, twists) run on the host."""
    return native().generate_emulated(int(seed), int(dim), int(rows), int(first))


def u32_to_uniform(u: torch.Tensor, lo: float = -100.0, hi: float = 100.0) -> torch.Tensor:
    """libstdc++ generate_canonical<float> + uniform_real_distribution map (separately rounded)."""
    f = u.to(torch.int64).to(torch.float32) / 4294967296.0
    f = torch.where(f >= 1.0, torch.full_like(f, 0.99999994), f)
    return f * (hi - lo) + lo  # two separate fp32 kernels: no fused multiply-add


def uniform_points(n: int, dim: int, seed: int = 0, device="cuda", chunk: int = 1 << 26) -> torch.Tensor:
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    out = torch.empty((n, dim), dtype=torch.float32, device=device)
    flat = out.view(-1)
    for s in range(0, flat.numel(), chunk):
        e = min(flat.numel(), s + chunk)
        u = torch.randint(0, 1 << 32, (e - s,), generator=g, device=device, dtype=torch.int64)
        flat[s:e] = u32_to_uniform(u)
    return out
