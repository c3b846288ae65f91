"""Forest decomposition — the reference's MPI design (kdtree_mpi.cpp:170-291), one rank per GPU.

Each rank owns the generation-order slice [local*rank, local*rank+local) (remainder on the
last rank, kdtree_mpi.cpp:208-216), builds an independent tree on it, answers every query
locally, and one MIN reduction combines the answers (kdtree_mpi.cpp:253). The reduction
carries the packed (distance, id), so the result also names the neighbour; ranks with no
points contribute +inf instead of crashing.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..models.kdtree import KDTree
from . import comm
from .global_tree import _local_packed


class ForestTree:
    def __init__(self, local: KDTree, first_row: int, n_total: int):
        self.local = local
        self.first_row = int(first_row)
        self.n_total = int(n_total)

    @classmethod
    def build(cls, points: torch.Tensor, first_row: int, n_total: int, id_base: int = 1, mode: str = "exact",
              threads: int = 1) -> "ForestTree":
        """points: this rank's slice; ids are the global ids first_row + i + id_base."""
        t = KDTree.build(points, id_base=first_row + id_base, mode=mode, threads=threads)
        return cls(t, first_row, n_total)

    def local_error(self) -> int:
        """Device error word of this rank's build (0 = ok, also for CPU trees). Synchronises."""
        e = self.local._err
        return int(e[0].item()) & 0xFFFFFFFF if e is not None else 0

    def local_packed(self, queries: torch.Tensor, method: str = "auto") -> torch.Tensor:
        """Packed (d2, global id) of the nearest point of THIS slice (no communication)."""
        return _local_packed(self.local, queries, method)

    def query_packed(self, queries: torch.Tensor, method: str = "auto") -> torch.Tensor:
        """Packed (d2, global id) of the nearest point over all ranks. Reference-mode forests
        use the reference search on each rank (so results match kdtree_mpi exactly)."""
        return comm.min_packed_(self.local_packed(queries, method).to(comm.device()))


def logical_ranks(ranks: int, world: int, rank: int) -> range:
    """The logical forest ranks a process owns when R logical ranks (the reference's `mpirun
    -np R`, Makefile:36 runs 16) are spread over P processes / GPUs: a contiguous block of
    R / P (the first R % P processes take one more). Each logical rank keeps the reference's
    slicing of the generation order (kdtree_mpi.cpp:204-224) at R, so the forest -- and in
    reference mode its answers, which depend on R -- is the reference's at -np R."""
    if ranks < world:
        raise ValueError(f"--ranks {ranks} < {world} processes")
    q, r = divmod(ranks, world)
    lo = rank * q + min(rank, r)
    return range(lo, lo + q + (1 if rank < r else 0))


def forest_min_packed(trees, queries: torch.Tensor, method: str = "auto") -> torch.Tensor:
    """MIN over this process's forest slices, then over the processes (one reduction)."""
    best = None
    for t in trees:
        p = t.local_packed(queries, method).to(comm.device())
        best = p if best is None else torch.minimum(best, p)
    return comm.min_packed_(best)  # (every process owns at least one logical rank)
