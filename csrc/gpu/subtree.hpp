// LDS subtree kernel (internal header shared by the global builder).
#pragma once
#include <hip/hip_runtime.h>

#include "pkdtree/common.hpp"

namespace pkdtree {

// Largest segment the LDS subtree kernel can hold for a dimension.
int subtree_capacity(int dim);

// Builds every segment of one level completely: segment k of the level is heap node
// heap0 + k with (seg_lo, seg_n); rows are read from SoA columns `cols` (stride ncol,
// column dim = ids) and the in-order result is written to out_pts / out_ids.
void launch_subtree(const float* cols, i64 ncol, int dim, const i64* seg_lo, const i64* seg_n, i64 heap0,
                    i64 segs, int depth_base, int nmax, float* out_pts, u32* out_ids, hipStream_t stream);

}  // namespace pkdtree
