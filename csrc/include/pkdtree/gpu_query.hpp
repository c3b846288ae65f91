// Exact 1-NN queries on the GPU.
//
// The reference answers queries with a recursive DFS on heap nodes (nearest,
// kdtree_sequential.cpp:75-136). At d=128 that DFS visits every node, so
// two exact kernels are provided and give identical answers:
//   * brute force: every point against a tile of queries, for high dimension / few queries;
//   * traversal: one thread per query walks the implicit in-order tree with an explicit
//     stack, for low dimension / many queries.
// Results are packed (float_bits(d2) << 32 | id); unsigned MIN is the lexicographic
// (distance, id) minimum, so results from different ranks/trees combine with one MIN
// reduction (the reference's MPI_Reduce(MIN), kdtree_mpi.cpp:253, but carrying the id).
// Distances use the reference's summation order (see common.hpp).
#pragma once
#include <hip/hip_runtime.h>

#include "pkdtree/common.hpp"

namespace pkdtree {

// Initialise `out[q]` to kPackedInf for q < nq (queries then MIN into it).
void nn_init(u64* out, i64 nq, hipStream_t stream);

// pts [n, dim] AoS; ids [n] or nullptr (id = id_base + row). out[q] = min over points.
void nn_brute(const float* pts, const u32* ids, u32 id_base, i64 n, int dim, const float* queries, i64 nq,
              u64* out, hipStream_t stream);

// tree_pts/tree_ids: in-order implicit tree of n points whose root is at depth `depth0`.
void nn_traverse(const float* tree_pts, const u32* tree_ids, i64 n, int dim, int depth0, const float* queries,
                 i64 nq, u64* out, hipStream_t stream);

// The same search for the selected queries only: query sel[i] for i < *sel_count (a device
// word; max_sel >= it bounds the launch). out is indexed by the query number. (Routed queries
// of the distributed tree: each rank searches a query only in the blocks it can matter for.)
void nn_traverse_sel(const float* tree_pts, const u32* tree_ids, i64 n, int dim, int depth0, const float* queries,
                     const u32* sel, const u32* sel_count, i64 max_sel, u64* out, hipStream_t stream);

// The reference's search procedure (kdtree_sequential.cpp:75-130: near side first, far side
// iff axis distance^2 < best, strict improvements only) for reference-mode trees: the same
// visited nodes and the same (possibly non-nearest) answer as the reference. `out` should
// start at kPackedInf (nn_init): the reference starts every search afresh from the root.
void nn_traverse_reference(const float* tree_pts, const u32* tree_ids, i64 n, int dim, int depth0,
                           const float* queries, i64 nq, u64* out, hipStream_t stream);

// Exact-mode invariant checked on the device (a semantic race detector for the partition
// scatters): every slot k walks down from the root of its tree; at each
// ancestor m it must sit on the side its slot says (k < m -> (key, id) below m's, k > m ->
// above) on m's axis. Adds the number of violating (slot, ancestor) pairs to *count.
// O(n log n) work, one thread per slot.
void check_tree(const float* tree_pts, const u32* tree_ids, i64 n, int dim, int depth0, unsigned long long* count,
                hipStream_t stream);

// dst[q] = min(dst[q], src[q]) (combining searches that must each start afresh, e.g. the
// reference's procedure on several forest trees of one process)
void nn_min_into(const u64* src, u64* dst, i64 nq, hipStream_t stream);

// packed -> (sqrt(d2) correctly rounded, id)
void nn_finalize(const u64* packed, i64 nq, float* dist, i64* ids, hipStream_t stream);

}  // namespace pkdtree
