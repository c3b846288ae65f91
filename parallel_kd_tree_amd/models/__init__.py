"""Tree "models": the single-device KDTree and the distributed forest / global trees."""
from .kdtree import KDTree, build_tree, nearest_neighbor
from .node import Node, Point, tree_height

__all__ = ["KDTree", "build_tree", "nearest_neighbor", "Node", "Point", "tree_height"]
