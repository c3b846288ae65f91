"""Exact 1-NN query ops (csrc/gpu/query.hip, csrc/cpu/cpu_tree.cpp).

GPU results are packed int64: ``(float_bits(d2) << 32) | id`` so a plain MIN (also across
ranks) is the lexicographic (distance, id) minimum.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import native

INF_PACKED = (0x7F800000 << 32) | 0xFFFFFFFF


def nn_gpu(points: torch.Tensor, ids: Optional[torch.Tensor], queries: torch.Tensor, method: str = "brute",
           depth0: int = 0, id_base: int = 0, into: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed (d2, id) nearest neighbours of ``queries`` among ``points``.

    method='brute' works on any point array; method='traverse' needs an implicit in-order
    tree (``points``, ``ids`` from a build) whose root is at depth ``depth0``. With ``into``
    the results are MIN-accumulated into an existing packed tensor (forest queries).
    """
    return native().nn(points.contiguous(), ids, int(id_base), queries.contiguous(), method, int(depth0), into)


def unpack(packed: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Packed int64 -> (squared distance float32, id int64)."""
    p = packed.to(torch.int64)
    d2 = (p >> 32).to(torch.int32).view(torch.float32)
    ids = p & 0xFFFFFFFF
    return d2, ids


def finalize(packed: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Packed -> (distance = correctly rounded sqrtf(d2), id). On the GPU this runs a HIP
    kernel: torch's device sqrt is not correctly rounded, the reference's is."""
    if packed.is_cuda:
        d, i = native().nn_finalize(packed.contiguous())
        return d, i
    d2, ids = unpack(packed)
    return sqrt_exact(d2), ids


def sqrt_exact(d2: torch.Tensor) -> torch.Tensor:
    """Correctly rounded fp32 sqrt on the host. torch's CPU sqrt may use a 0.5001-ulp SIMD
    polynomial on some CPUs; numpy uses the hardware sqrt instruction (IEEE exact)."""
    import numpy as np
    return torch.from_numpy(np.sqrt(d2.detach().cpu().to(torch.float32).numpy()))


def nn_cpu(tree_pts: torch.Tensor, queries: torch.Tensor, depth0: int = 0, brute: bool = False):
    """Reference-procedure search on a CPU tree: returns (slot int64, d2 float32)."""
    return tuple(native().search_cpu(tree_pts.contiguous(), queries.to(torch.float32).contiguous(), int(depth0),
                                     bool(brute)))
