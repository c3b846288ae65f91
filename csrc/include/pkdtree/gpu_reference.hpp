// Reference-mode tree on the GPU (the reference's own build, kdtree_sequential.cpp:30-66): every
// subrange sorts only its first n - 1 points on the node's axis. See build_reference.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "pkdtree/common.hpp"

namespace pkdtree {

class ReferenceBuilder {
 public:
  ReferenceBuilder(i64 n, int dim, int depth0 = 0);
  size_t workspace_bytes() const { return ws_bytes_; }
  int sorted_levels() const { return levels_; }
  // Levels sorted by device-wide segmented radix passes (segments larger than the LDS finish);
  // the rest run inside one workgroup per segment.
  int global_levels() const { return lfin_; }
  // pts [n, dim] AoS (device), ids [n] or nullptr (id = id_base + row). Writes the in-order
  // tree to out_pts / out_ids. Enqueued on `stream`; no host synchronisation.
  void build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids, void* workspace,
             hipStream_t stream) const;

  // One segment-aligned tile of a sort pass (host-computed from the implicit tree geometry).
  struct Tile {
    u32 pos0;         // first sortable position of the tile
    u32 len;          // sortable rows in the tile (<= 4096)
    u32 seg_lo;       // start of the tile's segment
    u32 rows_before;  // sortable rows of the level's earlier segments
    u32 ent0;         // 256 * (first tile of the segment)
    u32 tseg;         // tiles of the segment
    u32 trel;         // this tile's index inside its segment
    u32 pad;
  };

 private:
  i64 n_;
  int dim_, depth0_, levels_ = 0, lfin_ = 0;
  std::vector<Tile> tiles_;           // every global level's tiles, level after level
  std::vector<i64> level_tile0_;      // first tile of level l (size lfin_ + 1)
  i64 max_tiles_ = 0;
  size_t off_perm_[2] = {0, 0}, off_key_[2] = {0, 0}, off_tiles_ = 0, off_cnt_ = 0, off_sums_ = 0, ws_bytes_ = 0;
};

}  // namespace pkdtree
