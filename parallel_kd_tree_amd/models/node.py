"""Point / Node facade with the reference API (Node.hpp:9-45, Node.cpp:1-48).

The tree itself is the implicit in-order array (no pointers); ``Node`` objects are created
lazily from (lo, n) slot ranges, so ``root.left.right.point`` works like the reference's
pointer tree without materialising N heap nodes.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np

MAX_PRINT_DIMENSION = 5  # Node.hpp:5


def _fmt(v: float) -> str:
    # std::ostream default float formatting: %g with 6 significant digits
    return format(float(v), ".6g")


class Point:
    """A d-dimensional point with an ID; ``coordinates`` is a float32 view."""

    __slots__ = ("ID", "dimension", "coordinates")

    def __init__(self, dim: int = 0, ID: int = 0, coordinates: Optional[Sequence[float]] = None):
        self.ID = int(ID)
        self.dimension = int(dim)
        self.coordinates = np.asarray(coordinates if coordinates is not None else np.zeros(dim), dtype=np.float32)

    # -- distances: fp32, sequential order, separately rounded (kdtree_sequential.cpp:14-25)
    @staticmethod
    def _d2(a: "Point", b: "Point") -> float:
        if a.dimension != b.dimension:
            raise ValueError("Dimensions do not match!")
        acc = np.float32(0.0)
        for x, y in zip(a.coordinates, b.coordinates):
            t = np.float32(x - y)
            acc = np.float32(acc + np.float32(t * t))
        return float(acc)

    def distance_squared(self, other: "Point") -> float:
        return Point._d2(self, other)

    def distance(self, other: "Point") -> float:
        return float(np.float32(math.sqrt(Point._d2(self, other))))

    @staticmethod
    def compare(a: "Point", b: "Point", axis: int) -> bool:  # Node.cpp:46-48
        return bool(a.coordinates[axis] < b.coordinates[axis])

    def __repr__(self) -> str:  # Node.cpp:16-28, including its ", , ..., " quirk for dim > 5
        s = f"Point(ID={self.ID}, dimension={self.dimension}, coordinates=["
        for d in range(self.dimension - 1):
            s += _fmt(self.coordinates[d]) + ", "
            if d >= MAX_PRINT_DIMENSION - 1:
                s += ", ..., "
                break
        if self.dimension > 0:
            s += _fmt(self.coordinates[self.dimension - 1])
        return s + "])"


class Node:
    """Lazy view of the node owning slot range [lo, lo+n) of an implicit tree."""

    __slots__ = ("_tree", "lo", "n", "depth")

    def __init__(self, tree, lo: int, n: int, depth: int):
        self._tree, self.lo, self.n, self.depth = tree, int(lo), int(n), int(depth)

    @property
    def slot(self) -> int:
        return self.lo + self.n // 2

    @property
    def axis(self) -> int:
        return (self._tree.depth0 + self.depth) % self._tree.dim

    @property
    def point(self) -> Point:
        return self._tree.point_at(self.slot)

    @property
    def left(self) -> Optional["Node"]:
        nl = self.n // 2
        return Node(self._tree, self.lo, nl, self.depth + 1) if nl > 0 else None

    @property
    def right(self) -> Optional["Node"]:
        nr = self.n - self.n // 2 - 1
        return Node(self._tree, self.slot + 1, nr, self.depth + 1) if nr > 0 else None

    def __repr__(self) -> str:
        return f"Node(slot={self.slot}, depth={self.depth}, size={self.n}, point={self.point!r})"


def tree_height(n: int) -> int:
    """ceil(log2(n+1)) — the height of the implicit tree of n points."""
    h = 0
    while n > 0:
        n //= 2
        h += 1
    return h
