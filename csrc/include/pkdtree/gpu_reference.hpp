// Reference-mode tree on the GPU (the reference's own build, kdtree_sequential.cpp:30-66): every
// subrange sorts only its first n - 1 points on the node's axis. See build_reference.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "pkdtree/common.hpp"

namespace pkdtree {

class ReferenceBuilder {
 public:
  ReferenceBuilder(i64 n, int dim, int depth0 = 0);
  size_t workspace_bytes() const { return ws_bytes_; }
  int sorted_levels() const { return levels_; }
  // pts [n, dim] AoS (device), ids [n] or nullptr (id = id_base + row). Writes the in-order
  // tree to out_pts / out_ids. Enqueued on `stream`; no host synchronisation.
  void build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids, void* workspace,
             hipStream_t stream) const;

 private:
  i64 n_;
  int dim_, depth0_, levels_ = 0;
  size_t off_perm_[2] = {0, 0}, off_key_[2] = {0, 0}, off_lo_ = 0, off_n_ = 0, off_tmp_ = 0, tmp_bytes_ = 0,
         ws_bytes_ = 0;
};

}  // namespace pkdtree
