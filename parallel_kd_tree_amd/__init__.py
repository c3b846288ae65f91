"""parallel_kd_tree_amd — MI355X-native parallel kd-tree (HIP/CDNA4 kernels + RCCL).

Capabilities of Dan-Yeh/Parallel-Kd-Tree (median-split kd-tree with cycling axis, exact 1-NN,
reference data generator and CLI protocol, MPI forest decomposition), re-designed for
gfx950: level-synchronous HIP build on an implicit in-order tree resident in HBM, exact NN
kernels, and forest / global multi-GPU decompositions over RCCL.
"""
from .models import KDTree, Node, Point, build_tree, nearest_neighbor, tree_height
from .utils.generator import generate_problem, generate_slice, uniform_points
from .utils.tree_print import free_tree, print_head_and_leaves, print_tree

__version__ = "0.1.0"

__all__ = ["KDTree", "Node", "Point", "build_tree", "nearest_neighbor", "tree_height", "generate_problem",
           "generate_slice", "uniform_points", "print_tree", "print_head_and_leaves", "free_tree", "__version__"]
