// Host-side geometry and planning of the global decomposition (global_builder.hpp): who owns
// which part of the tree, and the exchange plan. Pure host C++ with no HIP dependency, so it is
// unit-tested on the CPU and run under AddressSanitizer / UndefinedBehaviorSanitizer
// (csrc/tests/sanitize_main.cpp). The reference's counterpart is the slice arithmetic of
// kdtree_mpi.cpp:204-224, whose N < P case crashes.
#pragma once

#include <vector>

#include "pkdtree/common.hpp"

namespace pkdtree {

constexpr int kTopBins = 8192;  // nodes * bins per top level of the distributed histograms (LDS)

// Host-side geometry and planning (pure functions, unit-tested on the CPU).
namespace global_plan {
// (lo, n) of heap node h in the implicit tree of n_total points.
void segment(i64 n_total, i64 h, i64* lo, i64* n);
// Middle-bucket rows a rank may contribute at `level` (identical on every rank).
i64 middle_cap(i64 n_total, int P, int level, int scale);

// Which rank owns which part of the tree. The top LL levels have T = 2^LL leaves (heap nodes
// T - 1 + t); rank r owns leaves [leaf_lo[r], leaf_lo[r + 1]). A rank's share of the in-order
// tree is the contiguous slot range of its leaves plus the top nodes between them; the top
// nodes between two ranks' leaves ("boundary" nodes, owner -1) sit outside every share.
// LL: pipeline_k >= 0 gives ceil(log2 P) + pipeline_k; -1 picks 1 extra level at P = 2 (the
// exchange over one xGMI link is worth overlapping), 0 at other powers of two and 2 for other
// P (leaf runs of 4-6 keep the ranks within ~12-25% of an equal share); LL <= 6.
struct Layout {
  int P = 1, LL = 0, T = 1, R = 1;       // ranks, top levels, leaves, rounds (max leaves per rank)
  std::vector<int> leaf_lo;              // [P + 1]
  std::vector<i64> leaf_slot, leaf_n;    // [T] in-order slot range of each leaf
  std::vector<i64> top_slot;             // [T - 1] heap order; -1: empty node
  std::vector<int> top_owner;            // [T - 1] rank whose share holds it, -1: boundary
  std::vector<i64> share_lo, share_n;    // [P] slot range of each rank's share
};
Layout make_layout(i64 n_total, int P, int pipeline_k);
int top_levels_for(int P, int pipeline_k);
// A rank's share as complete subtrees ("blocks": dyadic runs of its leaves) and the top nodes
// between consecutive blocks. Block: offset in the share, points, depth of its root, heap node.
struct Block {
  i64 off, n;
  int depth;
  i64 heap;
};
void share_blocks(const Layout& lay, int r, std::vector<Block>* blocks, std::vector<i64>* between_heap);

// Exchange plan from the all-gathered per-leaf counts [P][T][4] (rows, err, id base, n_local).
// Returns 0 (ok), 1 (a middle bucket overflowed: retry with larger slots) or throws on
// inconsistent geometry. Round j carries leaf leaf_lo[q] + j of every rank q that has one.
struct Plan {
  std::vector<std::vector<i64>> send_rows, send_off;  // [R][P] rows to peer q in round j, and where
  std::vector<std::vector<i64>> recv_rows;             // [R][P] rows from peer p in round j
  std::vector<i64> leaf_start;                          // [T + 1] my pack buffer's leaf offsets
  std::vector<i64> src_base, src_n;                     // [P] id base and local rows of every rank
};
int make_plan(const std::vector<i64>& counts, const Layout& lay, int me, Plan* plan);
}  // namespace global_plan

}  // namespace pkdtree
