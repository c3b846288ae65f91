"""ONE exact kd-tree over the ranks of the process group, built by the native global builder
(csrc/cpu/global_builder.cpp) on its own RCCL communicator.

The same decomposition as :class:`GlobalTreeBuilder` (top log2(P) levels by allreduced
histograms and all-gathered pivot candidates, compact all-to-all of the points to their
subtree's rank, 2^k pipelined exchange rounds, one local build per leaf), but the whole build
runs in C++: no Python between the collectives, one host synchronisation (the exchange plan).
The reference has no counterpart: its MPI program only builds independent per-rank trees
(kdtree_mpi.cpp:204-253)."""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from . import comm
from .global_tree import DistTree


class NativeGlobalBuilder:
    def __init__(self, n_total: int, dim: int, device: torch.device, pipeline_k: int = -1):
        if device.type != "cuda":
            raise ValueError("the native global builder runs on GPUs (use GlobalTreeBuilder for host tensors)")
        nat = ops.native()
        self.n_total, self.dim, self.device = int(n_total), int(dim), device
        self.P = comm.world() if comm.is_initialized() else 1
        self.rank = comm.rank() if comm.is_initialized() else 0
        uid = nat.rccl_unique_id() if self.rank == 0 else bytes(128)
        if self.P > 1:  # rank 0's communicator id to every rank, over the default process group
            words = np.frombuffer(uid, dtype=np.int64).tolist()
            uid = np.asarray(comm.broadcast_ints(words), dtype=np.int64).tobytes()
        with comm.stdout_to_stderr():  # RCCL's version banner must not reach the protocol / JSON stdout
            self._g = nat.NativeGlobal(self.n_total, self.dim, self.rank, self.P, uid, pipeline_k,
                                       device.index or 0)
        self.depth0 = 0

    @property
    def top_levels(self) -> int:
        return int(self._g.top_levels())

    def build(self, points: torch.Tensor, id_base: int = 1) -> DistTree:
        """This rank's points [n_local, dim] (ids id_base + row); returns this rank's share of
        the global tree (views of the builder's buffers, valid until the next build)."""
        x = points.to(self.device, torch.float32).contiguous()
        self._g.build(x, int(id_base))
        return DistTree(self.n_total, self.dim, 0, self.P, self.rank, self._g.tree_pts(), self._g.tree_ids(),
                        int(self._g.slot_lo()), list(self._g.top_slots()), self._g.top_rows(), {})

    def read_error(self) -> int:
        return int(self._g.read_error())
