"""KDTree — the single-device tree object.

Built by the level-synchronous HIP builder on a GPU tensor or by the native CPU builders on
a CPU tensor. The tree is the implicit in-order array (``tree_pts``, ``tree_ids``): the node
of slot range [lo, lo+n) sits at slot lo + n//2 and splits on axis (depth0 + depth) % dim,
exactly the reference's post-build ``point_list`` layout (kdtree_sequential.cpp:30-70).

Modes
  exact      median under the total order (coordinate, id): unique tree, exact NN, identical
             for any number of GPUs (default).
  reference  the reference's quirky tree (sorts only the first n-1 points of every segment,
             kdtree_sequential.cpp:46-48) and its search procedure (:75-130), which can miss
             the true NN. On the CPU byte-identical to the reference binaries; on the GPU
             (csrc/gpu/build_reference.hip: one segmented radix sort per level) identical
             whenever no two points of a segment tie on its axis -- std::sort is unstable, so
             the order of ties is the C++ library's business.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import ops
from ..utils import io as tio
from .node import Node, Point, tree_height


class KDTree:
    def __init__(self, tree_pts: torch.Tensor, tree_ids: torch.Tensor, depth0: int = 0, mode: str = "exact"):
        if tree_pts.dim() != 2:
            raise ValueError("tree_pts must be [n, dim]")
        self.tree_pts = tree_pts
        self.tree_ids = tree_ids
        self.depth0 = int(depth0)
        self.mode = mode
        self._host = None
        self._err = None  # device copy of the GPU build's error words (exact mode)

    # ------------------------------------------------------------------ construction
    @classmethod
    def build(cls, points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0,
              mode: str = "exact", depth0: int = 0, subtree_max: int = 0, threads: int = 1,
              check_ids: bool = True) -> "KDTree":
        """Build from ``points`` [n, dim]. ``ids`` default to ``id_base + row``; explicit ids
        must be distinct (checked unless ``check_ids=False``). A GPU build is enqueued
        without a host sync; ``check()`` reads its device error word."""
        if points.dim() != 2:
            raise ValueError("points must be [n, dim]")
        points = points.to(torch.float32).contiguous()
        if mode not in ("exact", "reference"):
            raise ValueError("mode must be 'exact' or 'reference'")
        if check_ids:
            ops.check_unique_ids(ids)
        if points.is_cuda and mode == "exact":
            # (a sampled-top build is checked on the host and rebuilt unsampled if a band missed)
            tp, ti, b = ops.build_gpu_checked(points, ids, id_base, depth0, subtree_max)
            t = cls(tp, ti, depth0, mode)
            t._err = b.error_words()  # this build's error words (device copy, stream-ordered)
            return t
        if points.is_cuda:  # reference mode on the GPU (CPU std::sort builder where ties decide)
            tp, ti, _ = ops.build_reference_gpu_checked(points, ids, id_base, depth0)
            return cls(tp, ti, depth0, mode)
        else:
            cpu_ids = ids
            if cpu_ids is None:
                cpu_ids = (torch.arange(points.shape[0], dtype=torch.int64) + id_base).to(torch.int32)
            tp, ti = ops.build_cpu(points.cpu(), cpu_ids, mode, depth0, threads)
            if points.is_cuda:
                tp, ti = tp.to(points.device), ti.to(points.device)
        return cls(tp, ti, depth0, mode)

    def check(self) -> "KDTree":
        """Raise RuntimeError if the GPU build of this tree reported a device error (histogram
        / key disagreement, subtree overflow, ...). Synchronises; a no-op for CPU trees."""
        if self._err is not None:
            err, code, level, value = (int(v) & 0xFFFFFFFF for v in self._err.tolist())
            if err:
                raise RuntimeError(f"GPU kd-tree build failed: error word {err:#x} (code {code}, level {level}, "
                                   f"value {value})")
        return self

    # ------------------------------------------------------------------ properties
    @property
    def n(self) -> int:
        return int(self.tree_pts.shape[0])

    @property
    def dim(self) -> int:
        return int(self.tree_pts.shape[1])

    @property
    def device(self) -> torch.device:
        return self.tree_pts.device

    @property
    def height(self) -> int:
        return tree_height(self.n)

    @property
    def root(self) -> Optional[Node]:
        return Node(self, 0, self.n, 0) if self.n > 0 else None

    def _host_arrays(self):
        if self._host is None:
            self._host = (self.tree_pts.detach().cpu().numpy(), self.tree_ids.detach().cpu().numpy())
        return self._host

    def point_at(self, slot: int) -> Point:
        """The Point of one slot. A GPU tree copies that row only (a Node walk over a 100 M
        point tree never moves the tree to the host); CPU trees are viewed in place."""
        if self.tree_pts.is_cuda and self._host is None:
            row = self.tree_pts[slot].detach().cpu().numpy()
            return Point(self.dim, int(self.tree_ids[slot].item()) & 0xFFFFFFFF, row)
        pts, ids = self._host_arrays()
        return Point(self.dim, int(ids[slot]) & 0xFFFFFFFF, pts[slot])

    def to(self, device) -> "KDTree":
        return KDTree(self.tree_pts.to(device), self.tree_ids.to(device), self.depth0, self.mode)

    # ------------------------------------------------------------------ queries
    def query_packed(self, queries: torch.Tensor, method: str = "auto",
                     into: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Packed (d2, id) int64 per query (GPU). ``method``: auto | brute | traverse. A
        reference-mode tree always answers with the reference's search procedure."""
        if not self.tree_pts.is_cuda:
            raise ValueError("query_packed needs a GPU tree; use query() on CPU trees")
        q = queries.to(self.device, torch.float32).contiguous()
        if self.mode == "reference":
            method = "reference"
        elif method == "auto":
            method = "traverse" if self.dim <= 16 else "brute"
        return ops.nn_gpu(self.tree_pts, self.tree_ids, q, method, self.depth0, 0, into)

    def query(self, queries: torch.Tensor, method: str = "auto") -> Tuple[torch.Tensor, torch.Tensor]:
        """Exact nearest neighbour: (distance float32, id int64) per query row.

        Exact-mode trees return the true NN (ties -> smallest id). Reference-mode trees
        reproduce the reference search (which can miss the NN).
        """
        if self.tree_pts.is_cuda:
            return ops.finalize(self.query_packed(queries, method))
        q = queries.detach().cpu().to(torch.float32).contiguous()
        slots, d2 = ops.nn_cpu(self.tree_pts.cpu().contiguous(), q, self.depth0, brute=(method == "brute"))
        ids = self.tree_ids.cpu().to(torch.int64)[slots] & 0xFFFFFFFF
        # distance printed by the reference: sqrt(distance_squared(query, nn)), computed in fp32
        return ops.query.sqrt_exact(d2), ids

    def nearest_neighbor(self, query: Point) -> Optional[Node]:
        """Reference API (kdtree_sequential.cpp:133-136): the Node of the nearest point."""
        if self.n == 0:
            return None
        q = torch.from_numpy(query.coordinates.reshape(1, -1).copy())
        if self.tree_pts.is_cuda:
            # the id -> slot lookup runs on the device: one comparison pass over tree_ids, and
            # only the slot index crosses to the host (never the tree)
            _, ids = ops.finalize(self.query_packed(q))
            hit = (self.tree_ids == ids[0].to(torch.int32)).nonzero()
            slot = int(hit[0, 0])
        else:
            slots, _ = ops.nn_cpu(self.tree_pts.cpu().contiguous(), q, self.depth0)
            slot = int(slots[0])
        return self._node_of_slot(slot)

    def _node_of_slot(self, slot: int) -> Node:
        lo, n, depth = 0, self.n, 0
        while True:
            m = lo + n // 2
            if slot == m:
                return Node(self, lo, n, depth)
            if slot < m:
                n = n // 2
            else:
                lo, n = m + 1, n - n // 2 - 1
            depth += 1

    # ------------------------------------------------------------------ checks / io
    def invariant_violations(self) -> int:
        """Exact-mode invariant (left < node < right under (key, id) on the node's axis); 0 iff
        it holds. Runs on the tree's device: a HIP kernel for GPU trees (csrc/gpu/query.hip,
        counts violating (point, ancestor) pairs), the recursive checker for CPU trees (counts
        violating node sides)."""
        return int(ops.native().invariant_violations(self.tree_pts.detach().contiguous(),
                                                     self.tree_ids.detach().contiguous(), self.depth0))

    def save(self, path) -> None:
        tio.save_tree(path, self.tree_pts, self.tree_ids, self.depth0, self.mode)

    @classmethod
    def load(cls, path, device="cpu") -> "KDTree":
        tp, ti, depth0, mode = tio.load_tree(path)
        return cls(tp.to(device), ti.to(device), depth0, mode)

    def __repr__(self) -> str:
        return f"KDTree(n={self.n}, dim={self.dim}, mode={self.mode}, device={self.device}, height={self.height})"


# ---------------------------------------------------------------------- reference-style API
def build_tree(points, ids=None, **kw) -> Optional[Node]:
    """Reference API ``Node* build_tree(Point**, int)`` (kdtree_sequential.cpp:68-70)."""
    t = KDTree.build(torch.as_tensor(points, dtype=torch.float32), ids, **kw)
    return t.root


def nearest_neighbor(root: Node, query: Point) -> Optional[Node]:
    """Reference API ``Node* nearest_neighbor(Node*, Point*)`` (kdtree_sequential.cpp:133-136)."""
    return root._tree.nearest_neighbor(query) if root is not None else None


__all__ = ["KDTree", "build_tree", "nearest_neighbor", "Point", "Node"]
