// Device ops of the distributed ("global") decomposition.
//
// The reference only has a forest decomposition (every rank builds an independent tree on
// its slice, kdtree_mpi.cpp:204-253). The global mode builds ONE tree over all ranks: the top
// log2(P) levels are split with allreduced histograms (exact medians under the (key, id)
// order, found by gathering the few points of the median bucket), every point is then sent to
// the rank that owns its top-level leaf with a single all-to-all, and each GPU builds its
// subtree locally. These kernels are the per-rank pieces; communication is done by the caller
// (torch.distributed over RCCL). Every per-level decision (median bucket, exact pivot,
// children cells) is computed on the device from the collective outputs, so the top levels
// run without a single host round trip; only the all-to-all split sizes are read back.
//
// Input points are the caller's [n][dim] f32 rows; ids are either an explicit u32 array or
// implicit (id_base + row). Rows sent by the all-to-all are (dim + 1) floats: the coordinates
// followed by the id bits.
#pragma once
#include <hip/hip_runtime.h>

#include "pkdtree/common.hpp"
#include "pkdtree/global_plan.hpp"  // kTopBins

namespace pkdtree {

constexpr u32 kTopDone = 0xffffffffu;  // node index of a point that became a top-tree pivot
constexpr int kTopMaxNodes = 32;       // nodes per top level (P <= 64)
constexpr int kTopMaxRanks = 64;       // ranks whose middle rows one pivot block walks

struct TopPoints {
  const float* pts;  // [n][dim]
  const u32* ids;    // [n] or nullptr: id = id_base + row
  i64 n;
  int dim;
  u32 id_base;
};

// Global sizes of the nodes of one top level (heap nodes 2^l - 1 ...), known on the host
// from the implicit-tree geometry.
struct TopSizes {
  i64 n[kTopMaxNodes];
};

// Per-rank bounding box, encoded for ONE allreduce(MIN) over int64: box[c] = orderable(lo_c),
// box[dim + c] = ~orderable(hi_c) (both < 2^32). The caller fills box with 0xffffffff first.
// Device-side fills (kernels, so no host staging and graph-capturable): n 64-bit words of v;
// the [slots][4] count matrix of top_pack with its id-base / n_local columns set.
void fill_u64(void* p, i64 n, u64 v, hipStream_t stream);
// Several independent fills in ONE launch (each launch of a tiny kernel costs ~5 us on the
// chain): segment i = n[i] 64-bit words of v[i] at p[i]; count <= kFillSegs.
constexpr int kFillSegs = 8;
struct FillSegs {
  u64* p[kFillSegs];
  i64 n[kFillSegs];
  u64 v[kFillSegs];
  int count = 0;
  void add(void* ptr, i64 words, u64 value) {
    p[count] = static_cast<u64*>(ptr);
    n[count] = words;
    v[count] = value;
    ++count;
  }
};
void fill_u64_multi(const FillSegs& f, hipStream_t stream);
void fill_u32(void* p, i64 n, u32 v, hipStream_t stream);
void top_counts_init(i64* counts, int slots, i64 id_base, i64 n_local, hipStream_t stream);

void top_bbox(const TopPoints& p, i64* box, hipStream_t stream);
// cells[0] ([dim][2] lo/hi) from the reduced box.
void top_root_cell(const i64* box, int dim, float* cells, hipStream_t stream);

// One top level: (a) if level > 0, route each point below the pivot of its node from the
// previous level (heap order: 2h+1 / 2h+2; the pivot itself -> kTopDone) and store the node;
// at level 0 every point is at the root and `node` is not read; (b) histogram the level's
// axis into hist[(node - first) * bins + b] with the node's cell (cells, heap-indexed
// [h][dim][2]) as bucket range. hist must be zeroed by the caller.
void top_route_hist(const TopPoints& p, u32* node, int level, const u64* pivots, int prev_axis, int axis,
                    const float* cells, int bins, u32* hist, hipStream_t stream);

// Per node of the level: the bucket b* holding the element of rank size/2 and the counts
// below / inside it. sel[j] = {b*, count_less, count_mid, 0}. err |= 2 on inconsistent sums.
// Also zeroes zero_hist (the next level's histogram, kTopBins words; may be null) and the
// 16-B header of the level's staging buffer (may be null).
void top_select(const u32* hist, int level, int bins, const TopSizes& sizes, u32* sel, u32* err, u32* zero_hist,
                u32* zero_hdr, hipStream_t stream);

// Median-bucket staging fused with the next level's routing and histogram (one pass per top
// level): points outside their node's median bucket go to their child now (node[i]) and count
// into hist_next (nullptr at the last top level); points inside it are staged in buf =
// [4 header words: count, 0, 0, 0][cap][dim + 3] floats (coordinates, id bits, node, input
// row); count may exceed cap (the pivot kernel flags it). A node's histogram is bucketed over
// its parent's cell (the root's own at level 0), which top_route_hist at level 0 matches.
size_t top_middle_words(int dim, i64 cap);
void top_collect_route(const TopPoints& p, u32* node, int level, int axis, int next_axis, const float* cells,
                       int bins, int next_bins, const u32* sel, float* buf, i64 cap, u32* hist_next,
                       hipStream_t stream, bool radix = false);
// After the level's pivots: routes this rank's staged rows (buf from top_collect_route) below
// their node's pivot and counts them into hist_next (may be null).
void top_fixup(const float* buf, i64 cap, int dim, int level, int axis, int next_axis, const u64* pivots,
               const float* cells, int next_bins, u32* node, u32* hist_next, hipStream_t stream);

// Exact pivots of one level from the all-gathered middle buffers (P consecutive buffers of
// top_middle_words(dim, cap) words): per node, the element of rank size/2 - count_less among
// the gathered middles (radix select over (orderable(key) << 32 | id)). Writes pivots[h],
// top_rows[h] (dim + 1 floats) and the children cells. err |= 1 if a buffer overflowed.
void top_pivot(const float* gathered, int P, i64 cap, int level, int axis, int dim, const TopSizes& sizes,
               const u32* sel, u64* pivots, float* top_rows, float* cells, u32* err, hipStream_t stream);

// Counting sort of rows by top-level leaf (dest = node - (T - 1), T = 2^levels leaves <= 64;
// node[] as the top levels left it, kTopDone rows -- the pivots -- dropped; levels == 0: every
// row at leaf 0 and node[] unread). Output grouped by leaf (stable):
//   * col_stride == 0: rows out[k][row_stride], row_stride = dim + 1 (coordinates, id bits) or
//     dim (compact: coordinates only);
//   * col_stride  > 0: SoA planes, coordinate c of output row k at out[c * col_stride + k]
//     (the receiver's builder takes columns directly, no AoS -> SoA pass).
// counts [T][4] int64 = (rows for leaf, err word, 2 words left to the caller). With `bitmaps`
// ([T][bitmap_words] u32, bitmap_words >= ceil(n / 32)) the leaf of every row is also written
// as one bit per (leaf, row) -- from the scatter's own ballots: the compact exchange sends the
// coordinates plus n / 8 bytes per leaf instead of ids, and the receiver rebuilds the ids.
size_t top_pack_scratch_bytes(i64 n, int T);
void top_pack(const TopPoints& p, const u32* node, int levels, float* out, int row_stride, i64 col_stride,
              u32* bitmaps, i64 bitmap_words, i64* counts, const u32* err, void* scratch, hipStream_t stream);
// top_pack in two steps: the per-leaf counts (written to `counts`; the scatter offsets stay in
// `scratch`), then the scatter. The global builder starts the counts' all-gather and host
// read-back between them, so the host's exchange planning overlaps the scatter.
void top_pack_count(const TopPoints& p, const u32* node, int levels, i64* counts, const u32* err, void* scratch,
                    hipStream_t stream);
void top_pack_scatter(const TopPoints& p, const u32* node, int levels, float* out, int row_stride, i64 col_stride,
                      u32* bitmaps, i64 bitmap_words, const void* scratch, hipStream_t stream);

// Copies top-tree rows (dim + 1 floats: coordinates, id bits; heap order) into output slots:
// out_pts[slot[i]] / out_ids[slot[i]] = top_rows[heap[i]] for i < count (<= 64).
struct TopPlacement {
  int count;
  int heap[64];
  i64 slot[64];
};
void top_place_rows(const float* top_rows, int dim, const TopPlacement& pl, float* out_pts, u32* out_ids,
                    hipStream_t stream);

// *dst |= *src (device words): collects the error words of builds that share a workspace.
void or_error_word(const u32* src, u32* dst, hipStream_t stream);

// Receiver of the compact exchange: rows from source s occupy [off[s], off[s] + cnt[s]) of
// the receive buffer in increasing source-row order, so the k-th row from s has the id
// base[s] + (position of the k-th set bit of s's bitmap, words [bm_off[s], bm_off[s] +
// words[s]) of `bitmaps`). err |= 8 if a bitmap's popcount differs from cnt[s].
constexpr int kBmMaxSources = 64;
struct BmSources {
  i64 off[kBmMaxSources];
  i64 cnt[kBmMaxSources];
  i64 bm_off[kBmMaxSources];
  i64 words[kBmMaxSources];
  u32 base[kBmMaxSources];
};
size_t ids_from_bitmaps_scratch_bytes(i64 max_words, int P);
void ids_from_bitmaps(const u32* bitmaps, int P, const BmSources& src, u32* ids, void* scratch, u32* err,
                      hipStream_t stream);

// ---- the median by distributed radix rounds (duplicate-heavy / skewed data) -------------
// When a median bucket outgrows the all-gather slots, the builder switches to this mode: the
// bucket's rows stay at their node (top_collect_route radix=true), and 8 rounds of a per-node
// 256-bin digit histogram of the (key, id) composite (top_radix_hist) + an all-reduce(SUM) +
// top_radix_sel fix the exact median one byte at a time; its row comes from the one rank that
// holds it by an all-reduce(MIN) of (dim + 1) i64 words per node (top_radix_row, INT64_MAX
// elsewhere); top_radix_pivot sets pivots, top rows and children cells, top_radix_fixup routes
// the bucket's rows. Memory O(nodes x 256) instead of P x (bucket rows).
struct TopRadix {
  u64 prefix;  // composite bits fixed so far
  u32 rank;    // rank of the median among the rows matching the prefix
  u32 active;  // node has points
};
void top_radix_init(const u32* sel, const TopSizes& sizes, int level, TopRadix* rs, hipStream_t stream);
void top_radix_hist(const TopPoints& p, const u32* node, int level, int axis, const TopRadix* rs, int pass,
                    u32* hist, hipStream_t stream);
void top_radix_sel(u32* hist, int level, int pass, TopRadix* rs, u32* err, hipStream_t stream);
void top_radix_row(const TopPoints& p, const u32* node, int level, int axis, const TopRadix* rs, i64* rowbuf,
                   hipStream_t stream);
void top_radix_pivot(const i64* rowbuf, const TopRadix* rs, int level, int axis, int dim, u64* pivots,
                     float* top_rows, float* cells, u32* err, hipStream_t stream);
void top_radix_fixup(const TopPoints& p, u32* node, int level, int axis, int next_axis, const u64* pivots,
                     const float* cells, int next_bins, u32* hist_next, hipStream_t stream);

// ---- routed queries on the distributed tree ---------------------------------------------
// A rank's blocks (complete subtrees of its share with points): which top-level leaf belongs
// to which block, and each block's root heap node.
constexpr int kRqMaxBlocks = 64;
struct RqBlocks {
  int nb;                      // blocks
  int LL, T;                   // top levels, leaves
  int depth0;
  int leaf_block[64];          // [T]: index of the block holding leaf t, -1: another rank's
  i64 heap[kRqMaxBlocks];      // root heap node of block b
};
// Home routing: every query descends the top tree (q[axis] >= pivot: right, the search's own
// near side) to its leaf; a query whose leaf is in block b is appended to lists[b * Q ..] with
// counts[b] (device words, zeroed by the caller); home[q] = b or -1.
void rq_home(const float* queries, i64 Q, int dim, const float* top_rows, const RqBlocks& bl, u32* lists,
             u32* counts, int* home, hipStream_t stream);
// Reach routing: query q is appended to block b (b != home[q]) when the box of b (the top
// pivots above its root, [lo, hi] per axis, closed) is within q's best distance so far:
// gap^2 <= d2 * (1 + 1e-5) (conservative against the fp32 sequential distance sums).
void rq_reach(const float* queries, i64 Q, int dim, const float* top_rows, const RqBlocks& bl, const u64* best,
              const int* home, u32* lists, u32* counts, hipStream_t stream);

}  // namespace pkdtree
