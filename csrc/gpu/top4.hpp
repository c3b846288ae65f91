// Sampled top levels: the first four levels of the exact tree in ONE row-moving pass.
//
// The level-synchronous builder needs each level's exact (key, id) median before it can move
// rows, so levels 0..3 used to cost two paired scatter passes plus five key sweeps and
// second-stage histograms that exist only to make each pivot exact before its scatter
// (profiles/r3_100Mx3_timeline_s3.txt). Here the pivots are ESTIMATED first and made exact
// afterwards ("sample -> splitters -> exact fix-up", SURVEY.md §5.8, inside one GPU):
//   sample    a stratified random sample of rows (one per stride window, random offset) is
//             read from the AoS input; a 4-level tree is built over the sample with 16-bit
//             histograms, giving every node a band [a, b] of keys that holds the node's true
//             median with overwhelming probability (z standard deviations of the sample rank
//             plus margin for the estimated routing of the sample);
//   scatter   every row is read ONCE from the AoS input: a row that is certain at all four
//             levels (key < a: left, key > b: right) goes straight to its level-4 segment,
//             whose size is known exactly; a row inside some band goes to a staging arena
//             with the tag of that node. The pass writes the SoA columns the later levels
//             read, so it also replaces the AoS -> SoA prep;
//   resolve   per level, over the staged rows only: counts give the median's rank inside the
//             band, a 16-bit histogram of the band's (key, id) composites finds its bin, the
//             bin's rows are collected and radix-selected: the exact median. Staged rows are
//             routed by it to the next level;
//   insert    staged rows fill the remaining slots of their level-4 segments.
// A band that misses its median (~2e-9 per node at the default z = 6 for any input order, since
// the sample positions are random; always on duplicate-heavy data whose median arenas are too
// large to stream) is DETECTED (counts do not bracket the median rank) and reported in the error
// word (bit kErrBit); every later kernel of the build then returns at once (dev::build_failed)
// and callers rebuild unsampled. Ties are exact: bands are inclusive key ranges and the median is
// selected on the composite key.
// Replaces build_tree_rec's top four levels of std::sort (kdtree_sequential.cpp:30-66).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "device_utils.hpp"
#include "pkdtree/common.hpp"

namespace pkdtree {
namespace top4 {

constexpr int kLevels = 4;
constexpr int kNodes = 15;      // heap nodes of levels 0..3
constexpr int kCells = 16;      // level-4 segments
constexpr int kHeap = 31;       // heap nodes 0..30 (levels 0..4)
constexpr u32 kErrBit = 0x20u;  // error-word bit of the sampled top levels

struct Geom {       // host-computed segment geometry of the heap nodes of levels 0..4
  i64 lo[kHeap];
  i64 n[kHeap];
  int axis[kLevels + 1];  // split axis of levels 0..4
  int dim;
};

struct IO {
  const float* pts;   // [n, dim] AoS input, or nullptr: SoA input columns below
  const float* in_cols = nullptr;  // dim coordinate columns + the id column, stride in_ncol (must
  i64 in_ncol = 0;                 // not alias cols / stage)
  const u32* ids;     // [n] or nullptr (id = id_base + row); AoS input only
  u32 id_base;
  i64 n;
  float* cols;        // SoA output columns (dim coords + ids), stride ncol: level-4 segments
  float* stage;       // SoA staging columns (same layout), at least n rows
  i64 ncol;
  float* out_pts;     // the tree: the 15 medians are written here; out_ids doubles as the
  u32* out_ids;       // staging tags until then (both are free before the later levels)
  float* cells;       // heap-indexed [h][dim][2]: nodes 0..30 written
  dev::BucketParams* params;  // params of the level-4 nodes (heap 15..30) written
  int bins4;          // histogram bins of level 4
  u32* err;           // the builder's sticky error words [4]
  void* ws;           // workspace_bytes() bytes, 256-B aligned
};

struct Tune {
  int sample_log2 = 0;  // sample rows = 2^sample_log2 (capped at n / 4); 0: by size (2^20 at 100 M)
  float z = 6.0f;        // band half-width in sample-rank standard deviations (the builder passes Tuning::top_z)
  int scatter_blocks = 0;  // 0: by size
  // Diagnostics (PKD_TOP_DIAG; timing only, the tree is NOT built): 1 stop after the scatter,
  // 2 the same with the scatter's reservation atomics replaced by in-range tile offsets, 3 also
  // without the scatter's global stores.
  int diag = 0;
  u32 salt = 0;  // sample positions are a hash of (row window, salt): the builder varies it per build
};

size_t workspace_bytes();
void run(const Geom& g, const IO& io, const Tune& t, hipStream_t stream);

// Diagnostic (tests, tools): band statistics of the last build on this workspace, per node:
// {band rows, rank of the median inside the band, staged rows at the node}; synchronises.
void band_report(const void* ws, hipStream_t stream, u32 (*out)[3]);

}  // namespace top4
}  // namespace pkdtree
