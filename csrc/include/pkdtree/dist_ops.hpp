// Device ops of the distributed ("global") decomposition.
//
// The reference only has a forest decomposition (every rank builds an independent tree on
// its slice, kdtree_mpi.cpp:204-253). The global mode builds ONE tree over all ranks: the top
// log2(P) levels are split with allreduced histograms (exact medians under the (key, id)
// order, found by gathering the few points of the median bucket), every point is then sent to
// the rank that owns its top-level leaf with a single all-to-all, and each GPU builds its
// subtree locally. These kernels are the per-rank pieces; communication is done by the caller
// (torch.distributed over RCCL).
//
// Rows are (dim + 1) floats: the coordinates followed by the id bits.
#pragma once
#include <hip/hip_runtime.h>

#include "pkdtree/common.hpp"

namespace pkdtree {

constexpr u32 kTopDone = 0xffffffffu;  // node index of a point that became a top-tree pivot

// One top level: (a) if level > 0, route each point below the pivot of its node from the
// previous level (node = 2*node+1 / 2*node+2 in heap order; the pivot itself -> kTopDone);
// (b) histogram the level's axis into hist[(node - first_node) * bins + b] using the node's
// bucket params (lo, scale). hist must be zeroed by the caller.
//   pivots: composite keys (orderable(key) << 32 | id) of every decided top node (heap order)
//   prev_axis: split axis of the previous level (ignored at level 0)
void top_route_hist(const float* rows, i64 n, int dim, u32* node, int level, const u64* pivots, int prev_axis,
                    int axis, const float* params /* [nodes][2] lo, scale */, int bins, u32* hist,
                    hipStream_t stream);

// Compacts the rows of points whose bucket (same function as top_route_hist) equals
// bstar[node]: out_rows [cap][dim+1], out_count[0] = number found (may exceed cap: caller
// retries with a larger buffer).
void top_collect_middle(const float* rows, i64 n, int dim, const u32* node, int level, int axis,
                        const float* params, int bins, const u32* bstar, float* out_rows, i64 cap,
                        unsigned long long* out_count, hipStream_t stream);

// Final routing below the last top level + counting sort of rows by destination leaf
// (dest = node - (P - 1)): out_rows [n_kept][dim+1] grouped by destination, counts [P].
// Pivot points are dropped. `scratch` holds 2 * blocks * P u32 (see top_pack_scratch).
size_t top_pack_scratch_bytes(i64 n, int P);
void top_pack(const float* rows, i64 n, int dim, u32* node, int levels, const u64* pivots, int last_axis, int P,
              float* out_rows, u32* counts, void* scratch, hipStream_t stream);

}  // namespace pkdtree
