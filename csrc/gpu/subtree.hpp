// LDS subtree kernel (internal header shared by the global builder).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "pkdtree/common.hpp"

namespace pkdtree {

// Default LDS subtree capacity for a dimension (two workgroups per CU), and the largest
// one that fits at all (one workgroup per CU).
int subtree_capacity(int dim);
int subtree_capacity_max(int dim);

// Builds every segment of one level completely: segment k of the level is heap node
// heap0 + k with (seg_lo, seg_n); rows are read from SoA columns `cols` (stride ncol,
// column dim = ids) and the in-order result is written to out_pts / out_ids.
// `cells` holds the heap-indexed cell [h][dim][2] of every segment root (bucket ranges).
void launch_subtree(const float* cols, i64 ncol, int dim, const i64* seg_lo, const i64* seg_n, const float* cells,
                    i64 heap0, i64 segs, int depth_base, int nmax, float* out_pts, u32* out_ids, u32* err,
                    hipStream_t stream);

// Diagnostic: per-phase s_memtime report of the last subtree launch (PKD_SUBTREE_STAMPS=1).
std::string subtree_stamp_report();

}  // namespace pkdtree
