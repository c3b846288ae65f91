// CPU kd-tree on the implicit in-order layout.
//
// * build_exact_cpu      — exact median under the (orderable(key), id) total order; the test
//                          oracle for every GPU path, and the threaded "omp" variant named
//                          in the reference Makefile (Makefile:23-27; source absent there).
// * build_reference_cpu  — reproduces the reference tree exactly, including its
//                          off-by-one sort of the first n-1 points (kdtree_sequential.cpp:46-48,
//                          SURVEY.md F1/Q1).
// * nn_search_cpu        — the reference's recursive NN procedure (kdtree_sequential.cpp:75-136)
//                          on the implicit layout: same visit order, same strict pruning.
// * nn_brute_cpu         — exact brute force with the reference's distance summation order.
#pragma once
#include <cstdint>
#include <ostream>
#include <utility>
#include <vector>

#include "pkdtree/common.hpp"

namespace pkdtree {

// perm[k] = input row placed at in-order slot k. ids may be null (id = row index).
void build_exact_cpu(const float* pts, const u32* ids, i64 n, int dim, int depth0, u32* perm,
                     int threads = 1);
// threads > 1: a segment's two children are built on two threads once it is sorted (same tree
// for any thread count); depth0 shifts the split axes like build_exact_cpu's.
void build_reference_cpu(const float* pts, i64 n, int dim, u32* perm, int threads = 1, int depth0 = 0);
// Threads the CPU builders use when the caller does not say (hardware threads, at most 64).
int default_cpu_threads();

// The reference's std::sort(idx, idx + n) by keys[idx] (a bit-exact parallel replica of libstdc++'s
// introsort: the same permutation, ties included, for any thread count).
void std_sort_replica(const float* keys, u32* idx, i64 n, int threads = 1);

// Hybrid reference mode. gpu_perm: slot -> input row of a GPU reference-mode tree whose build
// reported deciding ties (equal keys at ranks m-2..m+1 of a segment: there the reference's
// unstable std::sort decides) at the segments whose median slots are tied_slots[0, ntied).
// Only what std::sort's order decides is redone on the host, from the reference's own input
// order: every ancestor of a tied segment is sorted (its order is what its children start from)
// and every tied segment's whole subtree is built by build_reference_cpu's recursion; every other
// subtree (no deciding tie at or below it) keeps the GPU's slots, which are exact there. Writes
// the complete slot -> row map to perm and returns the slot ranges (start, count) the host decided
// (the rows the caller must patch into the GPU tree).
std::vector<std::pair<i64, i64>> reference_repair(const float* pts, i64 n, int dim, int depth0, const u32* gpu_perm,
                                                  const u32* tied_slots, size_t ntied, u32* perm, int threads);

// Gather rows/ids through a permutation (tree_pts[k] = pts[perm[k]]).
void gather_rows(const float* pts, const u32* ids, const u32* perm, i64 n, int dim, float* tree_pts,
                 u32* tree_ids);

struct NNResult {
  i64 slot;   // in-order slot of the nearest point (-1 if the tree is empty)
  float d2;   // squared distance computed as distance_squared(point, query)
};

// Reference-semantics traversal (strict '<' everywhere, ties go right).
NNResult nn_search_cpu(const float* tree_pts, i64 n, int dim, int depth0, const float* q);
// Exact brute force: lexicographic (d2, slot) minimum.
NNResult nn_brute_cpu(const float* pts, i64 n, int dim, const float* q);

// Number of violations of the exact-mode invariant: for every node, every element of the
// left subtree is < the node and every element of the right subtree is > the node under
// the (key, id) order on the node's axis. O(n log n).
i64 count_invariant_violations(const float* tree_pts, const u32* tree_ids, i64 n, int dim, int depth0);

// ---- tree utilities (Utility.cpp:21-63, Node.cpp:16-28) on the implicit layout ----------
// operator<<(Point): "Point(ID=.., dimension=.., coordinates=[..])", at most
// MAX_PRINT_DIMENSION (5) leading coordinates, with the reference's ", , ..., " artifact.
void print_point(std::ostream& os, i64 id, const float* coords, int dim);
// print_tree / print_tree_rec: pre-order, one "NODE(@depth=d): <point>" line per node,
// indented by d tabs.
void print_tree(std::ostream& os, const float* tree_pts, const u32* tree_ids, i64 n, int dim);
// print_head_and_leaves: the root and the left-most / right-most leaves.
void print_head_and_leaves(std::ostream& os, const float* tree_pts, const u32* tree_ids, i64 n, int dim);

}  // namespace pkdtree
