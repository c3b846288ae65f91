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
// narrow_idcol >= 0: the columns are narrow (column narrow_idcol = ids, narrow_idcol + 1 =
// input row index); the subtree's keys and the output rows come from the AoS input `in_rows`
// (row stride in_rs floats).
void launch_subtree(const float* cols, i64 ncol, int dim, const i64* seg_lo, const i64* seg_n, const float* cells,
                    i64 heap0, i64 segs, int depth_base, int nmax, float* out_pts, u32* out_ids, u32* err,
                    hipStream_t stream, int narrow_idcol = -1, const float* in_rows = nullptr, i64 in_rs = 0);

// Largest segment the narrow-column subtree kernel takes (two workgroups per CU), 0 if none.
int subtree_capacity_narrow(int dim);

// Diagnostic: per-phase s_memtime report of the last subtree launch (PKD_SUBTREE_STAMPS=1).
std::string subtree_stamp_report();

}  // namespace pkdtree
