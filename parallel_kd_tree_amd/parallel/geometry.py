"""Implicit-tree geometry shared by the decompositions.

Heap numbering: node h at level l = floor(log2(h+1)); children 2h+1, 2h+2. The node owns the
in-order slot range [lo, lo+n); its point sits at slot lo + n//2; left child [lo, lo+n//2),
right child [lo+n//2+1, lo+n).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def segment(n_total: int, h: int) -> Tuple[int, int]:
    """(lo, n) of heap node h in the implicit tree of n_total points."""
    l = (h + 1).bit_length() - 1
    j = h + 1 - (1 << l)
    lo, m = 0, int(n_total)
    for b in range(l - 1, -1, -1):
        if (j >> b) & 1:
            lo = lo + m // 2 + 1
            m = max(0, m - m // 2 - 1)
        else:
            m = m // 2
    return lo, m


def median_slot(n_total: int, h: int) -> int:
    lo, m = segment(n_total, h)
    return lo + m // 2


# ---- exact-order helpers (numpy, host side) ---------------------------------------------
def orderable_u32(x: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return np.where(b & 0x80000000, (~b) & 0xFFFFFFFF, b | 0x80000000).astype(np.uint64)


def composite_u64(key: np.ndarray, ids_u32: np.ndarray) -> np.ndarray:
    """(orderable(key) << 32) | id as uint64 — the exact builder's total order."""
    return (orderable_u32(key) << np.uint64(32)) | np.asarray(ids_u32, dtype=np.uint64)


def make_params(lo: float, hi: float, nb: int) -> Tuple[np.float32, np.float32]:
    """Same fp32 arithmetic as dev::make_params (csrc/gpu/device_utils.hpp)."""
    lo32, hi32 = np.float32(lo), np.float32(hi)
    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        span = np.float32(hi32 - lo32)
        scale = np.float32(np.float32(nb) / span) if span > 0 else np.float32(0.0)
    return lo32, scale
