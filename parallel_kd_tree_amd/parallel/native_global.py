"""ONE exact kd-tree over the ranks of the process group, built by the native global builder
(csrc/cpu/global_builder.cpp) on its own RCCL communicator.

Top levels by allreduced histograms and all-gathered pivot candidates, one all-to-all round per
top-level leaf of a rank (coordinates as SoA planes straight into the leaf builder's columns,
ids rebuilt from one bit per row and leaf), leaf subtrees built while the next round is in
flight. The whole build runs in C++: no Python between the collectives, one bounded host wait
(the exchange plan). Any number of ranks (<= 64). The reference has no counterpart: its MPI
program only builds independent per-rank trees (kdtree_mpi.cpp:204-253).

Failure detection: every host wait of the builder (and :meth:`sync`) is bounded by
``timeout_s`` (default: ``PKD_COMM_TIMEOUT`` or 300 s) and polls RCCL's asynchronous error
state; a stuck or failed peer aborts the communicator and raises a rank-tagged RuntimeError.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from .. import ops
from . import comm
from .global_tree import DistTree


class NativeGlobalBuilder:
    def __init__(self, n_total: int, dim: int, device: torch.device, pipeline_k: int = -1,
                 timeout_s: float = 0.0):
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
                                       device.index or 0, float(timeout_s))
        self.layout = self._g.layout()
        self.depth0 = 0

    @property
    def top_levels(self) -> int:
        return int(self._g.top_levels())

    def build(self, points: torch.Tensor, id_base: int = 1) -> DistTree:
        """This rank's points [n_local, dim] (ids id_base + row); returns this rank's share of
        the global tree (views of the builder's buffers, valid until the next build)."""
        x = points.to(self.device, torch.float32).contiguous()
        self._g.build(x, int(id_base))
        t = DistTree(self.n_total, self.dim, 0, self.P, self.rank, self._g.tree_pts(), self._g.tree_ids(),
                     int(self._g.slot_lo()), list(self._g.top_slots()), self._g.top_rows(), {}, self.layout)
        t.native = self._g  # routed queries run natively (GlobalBuilder::query)
        return t

    def sync(self) -> None:
        """Bounded wait for the last build (raises instead of hanging on a stuck peer)."""
        self._g.sync()

    def read_error(self) -> int:
        return int(self._g.read_error())

    def set_profile(self, on: bool = True) -> None:
        """hipEvent timing of every phase of the following builds (no host synchronisation)."""
        self._g.set_profile(bool(on))

    def phases(self) -> Dict[str, float]:
        """Per-phase times (ms) and exchange bytes of the last profiled build; synchronises."""
        return dict(self._g.phases())
