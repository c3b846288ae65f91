// Level-synchronous kd-tree builder for MI355X (gfx950).
//
// Replaces the reference's recursive std::sort build (build_tree_rec,
// kdtree_sequential.cpp:30-66; O(N log^2 N) pointer chasing) with:
//   * global levels — while segments are larger than the LDS subtree capacity, every level
//     is one streaming pass over HBM: a per-segment linear-bucket histogram (computed in
//     the previous pass) picks the bucket holding the median, a 3-way partition moves each
//     point to its left / middle / right zone and histograms the next level's axis in
//     the same pass, and a tiny refine kernel ranks the few middle-bucket points exactly
//     under the (key, id) order to place the median;
//   * an LDS subtree kernel — one workgroup per remaining segment builds all of its
//     remaining levels in the 160 KiB LDS and writes the final in-order rows.
// Output is the implicit in-order tree: slot k holds the point of the node
// whose segment median sits at k; no pointers, no per-node allocation.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "pkdtree/common.hpp"

namespace pkdtree {

struct BuildOptions {
  int subtree_max = 0;   // max segment handled by the LDS kernel (0 = auto from dim)
  int depth0 = 0;        // depth of the root (subtrees of a distributed tree start deeper)
  // Split build allowed (side HIP streams for large builds). The distributed builder turns it
  // off for its leaf builds: their streams plus its communication stream would exceed the
  // hardware queues (GPU_MAX_HW_QUEUES = 4), and RCCL's kernels would queue behind partitions.
  bool allow_split = true;
  // Sampled levels allowed: the top levels (builds of >= Tuning::top_min_n points, from AoS input
  // or from caller-owned SoA columns such as the distributed builder's received leaves) and the
  // sampled triples. A band miss (error bit top4_band_miss_bit(), GpuBuilder::sampled() builds
  // only) is redone by a builder with allow_top = false.
  bool allow_top = true;
};

// Value of an A/B knob (PKD_* variable that only exists to rerun a measured sweep): the variable
// is honoured only under PKD_AB=1, so a stray setting cannot silently change the build. Without
// PKD_AB=1 a set knob is ignored with a one-time note on stderr, and nullptr is returned.
const char* ab_knob(const char* name);

// Knobs of the builder (PKD_* environment variables, README "Tuning"), read ONCE when a builder
// is constructed -- never while a build is being enqueued. The defaults are the measured best on
// MI355X (profiles/ holds the sweeps). Public: PKD_SPLIT, PKD_TOP and the diagnostic traces;
// every other field is an A/B knob (ab_knob, PKD_AB=1).
struct Tuning {
  bool implicit_ids = true;   // PKD_IMPLICIT_IDS=0: the prep writes generated ids
  bool narrow = true;         // PKD_NARROW=0: full columns at high dims
  bool pairs = true;          // PKD_PAIR=0: one level per row-moving pass
  bool triples = true;        // PKD_TRIPLE=0: at most two levels per row-moving pass
  int triple_from = 3;        // PKD_TRIPLE_FROM: first level a triple may start at (8+ segments)
  int atomic_ranks = -1;      // PKD_PART_ATOMIC: pair scatter ranks zones by LDS atomics (1) or
  int atomic_ranks3 = -1;     //   wave ballots (0); PKD_PART3_ATOMIC the same for triples; -1: by n
  bool prefix = true;         // PKD_PART_PREFIX=0: counting pass instead of prefix placement
  bool tail = true;           // PKD_TAIL=0: the last three global levels by pairs / triples instead of k_tail3
  bool tail4 = true;          // PKD_TAIL4=0: never a 4-level tail (it replaces two pairs by a triple at 8-D)
  int tail4_min_dim = 4;      // PKD_TAIL4_MIN_DIM: lowest dim a 4-level tail may be planned at (>= 3)
  bool tail_pipe = true;      // PKD_TAIL_PIPE=0: k_tail3 moves its columns one at a time (load, stage, store)
  int g3_stage = 2;           // k_g3_part stores through an LDS tile of 2 (1) parts; 0: from registers
  bool part3_stage = true;    // PKD_PART3_STAGE=0: k_partition3 (ballot ranks) stores from registers
  int wide_ki = 4;            // PKD_WIDE_KI: k_g3_part / k_partition3 rows per thread at >= 6 columns (8: staged in
                              //   4 parts; won before the XCD mapping (6D 16.59 -> 16.23 ms), loses after it: 100M
                              //   5D 11.87 vs 12.18, 8D 16.45 vs 16.69 with 8; profiles/r6_wide_subtree_ab.txt)
  bool xcd_map = true;        // PKD_XCD_MAP=0: row-moving passes map block b to segment b / bps (not one XCD per segment)
  int tail_slim12 = 2;  // PKD_TAIL_SLIM12: 12-item k_tail3 registers: 0 all keys + ids (spills 52 B/lane at 3-D),
                        //   1 two key sets (no ids), 2 two key sets + ids (no spill; 100M x 3D 8.46 ms either way)
  bool split = true;          // PKD_SPLIT=0: one-stream build
  bool split_trace = false;   // PKD_SPLIT_TRACE=1: part timeline on stderr (synchronises)
  int colgroup = 0;           // PKD_COLGROUP: columns per load round of wide rows (0: by dim)
  int hist_div = 2;           // PKD_HIST_DIV: first-level histogram on 1/hist_div of the blocks
  int scan_div = 0;           // PKD_SCAN_DIV: key sweeps on 1/scan_div of the blocks (0: ~1024 blocks)
  int pair_bins = 2048;       // PKD_PAIR_BINS: bins of a level a paired pass fuses
  i64 level_blocks = 0;       // PKD_LEVEL_BLOCKS: top-level partition grid (0: by n)
  i64 stage2_min = 2048;      // PKD_STAGE2_MIN: second-stage histogram above this median bucket
  int split_level = 2, split_parts = 4, split_streams = 4;  // PKD_SPLIT_LEVEL / _PARTS / _STREAMS
  i64 split_min_n = i64(64) << 20;                          // PKD_SPLIT_MIN_N
  i64 split_min_n_3d = i64(512) << 20;  // PKD_SPLIT_MIN_N_3D (dims <= 3; PKD_SPLIT_MIN_N when only that is set):
                                        // since k_tail3 a 100 M x 3D split build is ~1% slower than one stream,
                                        // 1 B x 3D 0.4% faster, 100 M x 8D 1.5-6% faster (r3_ab_split_s3.txt)
  i64 split_min(int dim) const { return dim <= 3 ? split_min_n_3d : split_min_n; }
  // Sampled top levels (csrc/gpu/top4.hpp): levels 0..3 from an estimated band per node, one
  // scatter pass from the AoS input, exact fix-up of the staged band rows.
  bool top = true;            // PKD_TOP=0: levels 0..3 by the exact pairs
  i64 top_min_n = 10000000;  // PKD_TOP_MIN_N: smallest build that samples its top levels (8 M: 1.18 ms sampled vs 1.16 paired; 12.5 M: 1.49 vs 1.58)
  int top_sample_log2 = 0;    // PKD_TOP_SAMPLE: log2 of the sample rows (0: by size, 2^20 at 100 M)
  // z: a miss is detected and rebuilt unsampled (+1 build), so z only has to make that rare:
  // P(|N(0,1)| > 6) = 2e-9 per node x 15 nodes; 100M x 3D top staging 6% -> 4% of the rows.
  float top_z = 6.0f;         // PKD_TOP_Z: band half-width in sample-rank standard deviations
  int top_blocks = 0;         // PKD_TOP_BLOCKS: scatter grid (0: by size)
  int top_diag = 0;           // PKD_TOP_DIAG: timing diagnostics of the scatter (no tree; top4::Tune::diag)
  // Sampled triples (build_global.hip, k_g3_*): a triple's pivots of levels l and l+1 estimated
  // from a sample instead of two key sweeps, made exact over the staged band rows.
  // 100M x 3D (profiles/r5_g3_ab.txt): 9.147 ms exact, 8.946 sampled at level 7 (781 k-row
  // segments, 8% of the rows staged); sampling the level-10 triple too (98 k rows) costs more
  // than its sweeps (9.233), as does the level-7 triple of 12.5 M (1.447 vs 1.433).
  bool g3 = true;             // PKD_G3=0: every triple by its exact key sweeps
  int g3_min_segs = 16;       // PKD_G3_MIN_SEGS: first triple level that samples (segments; below
                              //   128 the fix-up of levels l+1, l+2 runs on several blocks per node)
  i64 g3_min_rows = 262144;   // PKD_G3_MIN_ROWS: smallest segment a sampled triple starts from
  i64 g3_min_n = i64(32) << 20;  // PKD_G3_MIN_N: smallest build that samples triples (12.5 M: 1.406 ms
                                 //   without, 1.434 with the 16-segment level-4 triple sampled)
  int g3_max_dim = 8;         // PKD_G3_MAX_DIM: widest rows that sample triples (with k_g3_part's
                              //   stores through LDS, 100M: 4D 11.76 -> 11.21 ms, 6D 17.17 -> 16.90,
                              //   8D 18.89 -> 18.42; profiles/r6_stage_ab.txt)
  i64 g3_sample = 65536;      // PKD_G3_SAMPLE: sample rows per segment (64-row runs)
  int g3_div_min = 1;         // PKD_G3_DIV_MIN: the sample holds at most 1 / g3_div_min of a segment
  i64 g3_multi_below = 128;   // PKD_G3_MULTI_BELOW: triples of fewer segments resolve on several blocks per node
  i64 g3_sample_blocks = 2048;  // PKD_G3_SAMPLE_BLOCKS: grid of a sample pass (all segments)
  float g3_z = 5.0f;          // PKD_G3_Z: band half-width in sample-rank standard deviations (5: a miss in
                              //   ~1 of 2000 100M builds, i.e. +5 us expected; staged 8.0% -> 6.8%)
  static Tuning from_env();
};

struct LevelPlan {
  int level;        // 0-based global level
  i64 segs;         // 2^level
  i64 nmax;         // largest segment at this level
  int bins;         // histogram bins per segment at this level
  int next_bins;    // bins per segment at level+1 (0 if level+1 is the subtree level)
  int bps;          // partition blocks per segment
  int axis;         // split axis at this level
  bool stage2 = false;  // median bucket split by a second (key-only) histogram pass
  bool pair = false;    // this level and the next are moved by ONE fused partition pass
  bool triple = false;  // this level and the next two are moved by ONE fused partition pass
  bool tail = false;    // this level and the next two: one workgroup per segment (k_tail3)
  bool sampled = false; // built by the sampled top levels (top4::run)
  bool g3 = false;      // a triple whose pivots of this level and the next are sampled (k_g3_*)
  int g3_div = 1;       // its sample: one 64-row run per 64 * g3_div rows
  int g3_sblocks = 1;   // sample blocks per segment
  int g3_k1 = 0, g3_k2 = 0;  // blocks per node of the multi-block resolve of levels +1 / +2 (0: one)
};

struct SplitStreams;  // side HIP streams + fork / join events of a split build

class GpuBuilder {
 public:
  GpuBuilder(i64 n, int dim, BuildOptions opt = {});

  i64 n() const { return n_; }
  i64 column_stride() const { return ncol_; }
  int dim() const { return dim_; }
  int global_levels() const { return lg_; }
  // Levels 0..3 built by the sampled top pass (AoS input builds; see top4.hpp).
  bool sampled_top() const { return top_; }
  // Any level built from a sample (the top levels or a sampled triple): a build's error word
  // may then carry top4_band_miss_bit(), and the build must be redone with allow_top = false.
  bool sampled() const { return top_ || g3_; }
  // Diagnostic: per top node {band rows, rank inside the median's fine bin, rows staged at
  // the node} of the last build on `workspace` (synchronises).
  std::vector<u32> top_band_report(const void* workspace, hipStream_t stream) const;
  // Diagnostic: the last sampled triple of the last build on `workspace` (synchronises): its
  // level, then per segment {rows, rows staged per tag 0..6, certain rows per great-grandchild
  // 0..7, staged rows inserted per great-grandchild 0..7, bad} (25 words). Empty without one.
  std::vector<u32> g3_report(const void* workspace, hipStream_t stream) const;
  int subtree_max() const { return nsub_; }
  // Split build (0 parts: off): from level split_level() on, the 2^split_level segments are
  // built as split_parts() independent parts on split_streams() HIP streams.
  int split_level() const { return split_level_; }
  int split_parts() const { return split_parts_; }
  int split_streams() const { return split_streams_; }
  const std::vector<LevelPlan>& levels() const { return levels_; }
  size_t workspace_bytes() const { return ws_bytes_; }
  std::string describe() const;

  // pts: [n, dim] AoS fp32 on the device; ids: [n] u32 or nullptr (id = id_base + row).
  // Writes the in-order tree to out_pts [n, dim] and out_ids [n]. The input is not
  // modified. Enqueued on `stream`; no host synchronisation, no allocation (graph-safe).
  void build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids,
             void* workspace, hipStream_t stream) const;

  // Rows of dim+1 floats: coordinates then the id bits (the distributed exchange format).
  void build_rows(const float* rows, float* out_pts, u32* out_ids, void* workspace, hipStream_t stream) const;

  // Same, but the input already sits in SoA columns inside the workspace (column c of
  // row r at cols[c*n + r], column dim = ids); used by the distributed path which
  // receives points straight into that layout.
  float* soa_input(void* workspace) const;
  // Sticky error word of the last build (0 = ok); synchronises the stream. Debug aid.
  // detail (optional, 3 words): first failure code, level, value.
  u32 read_error(const void* workspace, hipStream_t stream, u32* detail = nullptr) const;
  // Folds the last build's error word into the device words acc[0..2] (OR of the words, builds
  // with an error, builds with the miss bit), ordered after the build on `stream`: a benchmark
  // checks EVERY timed build without a host round trip per build.
  void accumulate_error(const void* workspace, u32* acc, hipStream_t stream) const;
  // Device address of that error word (valid until the workspace's next build).
  const u32* error_word(const void* workspace) const {
    return reinterpret_cast<const u32*>(static_cast<const char*>(workspace) + off_err_);
  }
  void build_from_soa(float* out_pts, u32* out_ids, void* workspace, hipStream_t stream) const;
  // Same, from caller-owned SoA columns (column c of row r at cols[c * column_stride() + r],
  // column dim = ids; 256-B aligned, (dim + 1) * column_stride() floats). The columns are
  // CLOBBERED: they serve as one of the build's two ping-pong buffers, so no AoS -> SoA pass
  // and no copy into the workspace is needed. The distributed builder receives its exchange
  // straight into such columns. Needs dim <= 8 (the full-column layout).
  // root_cell (optional, device [dim][2] floats): a box holding every point (the distributed
  // builder's top-level cell of the leaf); it replaces the bounding-box pass over the columns.
  void build_columns(float* cols, float* out_pts, u32* out_ids, void* workspace, hipStream_t stream,
                     const float* root_cell = nullptr) const;

 private:
  void prep_and_run(const float* pts, int rs, bool ids_in_row, const u32* ids, u32 id_base, float* out_pts,
                    u32* out_ids, void* workspace, hipStream_t stream) const;
  // implicit_ids: the prep left the id column unwritten (ids = id_base + input row); the
  // first pair's kernels synthesise them.
  // in_rows != nullptr: narrow columns (the lg_ global levels' keys, ids, input row index);
  // full rows are gathered from the AoS input `in_rows` (stride in_rs floats).
  // cols_a != nullptr: replaces the workspace's first column buffer (the input of the first pass).
  // first_level > 0: levels [0, first_level) are already built (the sampled top levels): their
  // cells, the first level's histogram parameters and the error word are set.
  void run_top(const float* pts, const float* in_cols, const u32* ids, u32 id_base, float* out_pts, u32* out_ids,
               char* ws, hipStream_t stream) const;
  void run_levels(float* out_pts, u32* out_ids, char* ws, hipStream_t stream, bool implicit_ids = false,
                  u32 id_base = 0, const float* in_rows = nullptr, i64 in_rs = 0, float* cols_a = nullptr,
                  int first_level = 0, bool root_ready = false) const;
  // Side streams for a split build on the current device (nullptr: run unsplit, e.g. when
  // the streams do not exist yet and `stream` is being captured into a graph).
  SplitStreams* split_streams_for(hipStream_t stream) const;

  i64 n_;
  i64 ncol_ = 0;  // column stride of the SoA working buffers (n rounded up to 64)
  int dim_;
  BuildOptions opt_;
  Tuning tune_;
  int lg_ = 0;      // number of global levels
  int nsub_ = 0;    // LDS subtree capacity
  std::vector<LevelPlan> levels_;     // the plan (from level 4 when the top levels are sampled)
  std::vector<LevelPlan> levels_nt_;  // top_ only: the plan of the entry points that start at level 0
  i64 heap_nodes_ = 0;  // nodes of levels 0..lg_
  int max_bins_ = 0;
  i64 max_hist_ = 0;
  i64 max_hist2_ = 0;
  bool narrow_ = false;  // high-dim: narrow columns + key-slot subtree (capacity nsub_ sized for it)
  int tail_ = -1;        // first of the last tail_lev_ global levels, built by k_tail3 (-1: none)
  int tail_items_ = 0;   // rows per thread of its 1024-thread workgroups
  int tail_lev_ = 3;     // levels of the tail: 4 where that leaves whole triples between the top and it (8-D)
  int scan_div_ = 1;     // the key sweeps run on 1 / scan_div_ of a level's partition blocks
  bool top_ = false;     // levels 0..3 by the sampled top pass (AoS input builds)
  mutable u32 top_salt_ = 0;  // per-build salt of the sample positions: a miss is never input-determined
  size_t off_top_ = 0;
  bool g3_ = false;           // some triple is sampled
  mutable u32 g3_salt_ = 0;
  size_t off_stage_ = 0, off_g3_ = 0, off_g3_hist_ = 0;  // staging columns, per-segment state, sample histograms
  size_t off_g3_nodes_ = 0, off_g3_mhist_ = 0, off_g3_cand_ = 0;  // multi-block resolve
  // workspace offsets
  size_t off_cols_a_ = 0, off_cols_b_ = 0, off_seg_lo_ = 0, off_seg_n_ = 0, off_state_ = 0,
         off_params_ = 0, off_cells_ = 0, off_hist0_ = 0, off_hist1_ = 0, off_bbox_ = 0, off_err_ = 0, off_hist2_ = 0, off_bcnt_ = 0,
         ws_bytes_ = 0;
  // Split build: from level split_level_ (a pair boundary) on, segment range p of
  // split_parts_ runs its remaining levels and its subtree kernel on stream p % split_streams_,
  // so one part's LDS-bound subtree kernel and small select / pivot launches overlap another
  // part's HBM-bound passes. Each stream has its own histogram set in the workspace.
  int split_level_ = 0, split_parts_ = 0, split_streams_ = 0;
  size_t off_split_ = 0, split_set_bytes_ = 0;
  size_t split_hist_ = 0, split_hist2_ = 0, split_bcnt_ = 0;  // u32 words per set
  std::shared_ptr<SplitStreams> split_;
};

// Error-word bit of the sampled levels (top levels, sampled triples): a band missed its median
// (the build is invalid and must be redone with BuildOptions::allow_top = false).
constexpr u32 top4_band_miss_bit() { return 0x20u; }

// Subtree kernel capacity for a dimension (largest power of two whose LDS image fits).
int default_subtree_max(int dim);

}  // namespace pkdtree
