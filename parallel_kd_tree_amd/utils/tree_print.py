"""Tree utilities of the reference (Utility.cpp:21-63): ``print_tree``, ``print_head_and_leaves``
and ``free_tree``, on the implicit in-order tree.

The text comes from the native printers (csrc/cpu/cpu_tree.cpp), which use ``std::ostream``
exactly like the reference, so float formatting and the ``", , ..., "`` artifact of
``operator<<(Point)`` for dim > 5 (Node.cpp:16-28) are byte-identical.
"""
from __future__ import annotations

import sys
from typing import TextIO, Union

from ..ops import native


def _tree_of(obj):
    from ..models.kdtree import KDTree
    from ..models.node import Node
    if isinstance(obj, KDTree):
        return obj, 0, obj.n
    if isinstance(obj, Node):
        return obj._tree, obj.lo, obj.n
    raise TypeError("expected a KDTree or a Node")


def tree_string(obj, what: str = "tree") -> str:
    """The reference's dump of a tree (or of the subtree under a Node) as a string."""
    tree, lo, n = _tree_of(obj)
    pts = tree.tree_pts[lo:lo + n].detach().cpu().contiguous()
    ids = tree.tree_ids[lo:lo + n].detach().cpu().contiguous()
    return native().tree_dump(pts, ids, what)


def print_tree(root: Union["KDTree", "Node"], file: TextIO = None) -> None:  # noqa: F821
    """Utility::print_tree: pre-order, ``NODE(@depth=d): Point(...)``, d tabs of indent.
    Depths are relative to ``root`` (print_tree_rec(root, 0))."""
    (file or sys.stdout).write(tree_string(root, "tree"))


def print_head_and_leaves(root: Union["KDTree", "Node"], file: TextIO = None) -> None:  # noqa: F821
    """Utility::print_head_and_leaves: the root, the left-most and the right-most leaf."""
    (file or sys.stdout).write(tree_string(root, "head_and_leaves"))


def free_tree(root) -> None:
    """Utility::free_tree. The implicit tree owns two tensors and no per-node memory; drop
    the references (the caching allocator reuses the HBM)."""
    from ..models.kdtree import KDTree
    if isinstance(root, KDTree):
        root.tree_pts = root.tree_pts.new_empty((0, root.tree_pts.shape[1]))
        root.tree_ids = root.tree_ids.new_empty((0,))
