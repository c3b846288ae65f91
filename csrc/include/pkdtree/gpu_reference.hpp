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
  // Levels selected device-wide (segments larger than the LDS finish); the rest run inside
  // one workgroup per segment.
  int global_levels() const { return lfin_; }
  // pts [n, dim] AoS (device), ids [n] or nullptr (id = id_base + row). Writes the in-order
  // tree to out_pts / out_ids. Enqueued on `stream`; no host synchronisation.
  void build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids, void* workspace,
             hipStream_t stream) const;
  // Segments of the last build whose tree was decided by equal keys (adjacent ranks m-2/m-1,
  // m-1/m or m/m+1 of a segment's sorted rows, m = n/2): there the reference's unstable
  // std::sort decides, so the tree may differ from the reference binary's; 0 = identical for
  // certain. Synchronises `stream`.
  u32 read_ties(const void* workspace, hipStream_t stream) const;
  // Median slots of the tied segments (at most kTieSlots of them; read_ties() counts them all).
  // Synchronises `stream`.
  static constexpr u32 kTieSlots = 1u << 18;
  std::vector<u32> read_tie_slots(const void* workspace, hipStream_t stream) const;

 private:
  struct RefLevel {
    i64 segs;
    int bins, bps, hbps;  // histogram buckets per segment, partition / histogram blocks per segment
  };
  i64 n_, ncol_ = 0;
  int dim_, depth0_, levels_ = 0, lfin_ = 0;
  bool rows_ = false;  // dim <= 8: rows move as SoA columns (else a permutation, keys gathered)
  int part_blocks_ = 16384;  // PKD_REF_BLOCKS: most blocks of a level's partition pass (one 2048-row chunk per block
                             // up to 33 M rows: 10 M x 3D 2.76 -> 2.64 ms against 2048 blocks)
  bool fin_rank_ = true;  // row-path LDS finish by rank propagation (PKD_REF_FIN=0: k_rr_finish, rows move)
  std::vector<RefLevel> plan_;
  size_t off_perm_[2] = {0, 0}, off_keys_ = 0, off_midc_ = 0, off_hist_ = 0, off_segs_ = 0, off_words_ = 0,
         off_hpart_ = 0, ws_bytes_ = 0;
};

// Writes input row rows[k] (coordinates from pts [*, dim], id ids[row] or id_base + row) to tree
// slot slots[k] for k < count (device arrays): the host-decided slots of a repaired tree.
void reference_patch(const float* pts, const u32* ids, u32 id_base, int dim, const u32* slots, const u32* rows,
                     i64 count, float* out_pts, u32* out_ids, hipStream_t stream);

// out [n][levels] (device) = the split key of every tree level: out[r][d] = pts[r][(depth0 + d) % dim].
// For levels <= dim this is all a host reference build of the tree reads (its axis at depth d is
// column d with depth0 0 and `levels` columns): high-dimensional inputs travel as ~20 columns, not dim.
void reference_level_keys(const float* pts, i64 n, int dim, int depth0, int levels, float* out, hipStream_t stream);

}  // namespace pkdtree
