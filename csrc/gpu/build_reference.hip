// Reference-mode builder on the GPU: the reference's own (quirky) tree.
//
// build_tree_rec (kdtree_sequential.cpp:30-66, kdtree_mpi.cpp:60-100) sorts only the FIRST
// n - 1 points of every subrange on the node's axis (:46-48), takes list[n/2] as the median
// and recurses on [0, n/2) and [n/2 + 1, n): the last point of a subrange keeps its slot, so
// the tree violates the kd invariant and depends on array positions, not only
// on point sets. Level-synchronous reproduction: at level l every segment [lo, lo + n) sorts
// rows [lo, lo + n - 1) by the level's axis and leaves row lo + n - 1 in place. One device
// radix sort per level does all segments at once on the 64-bit key (segment start << 32 |
// orderable(axis key)); the segment's last row gets the largest key of its segment, medians
// (finished slots) are singleton segments keyed by their own position, so nothing crosses a
// segment boundary. Rows never move: only a u32 permutation is sorted; the output rows are
// gathered once at the end.
//
// The radix sort is stable (ties keep their previous order) while std::sort is not, so the
// tree equals the reference's exactly when no two points of a segment share a key on its
// axis -- always true for tie-free data, usually true for the reference
// generator at small N. Exact mode (gpu_build.hpp) is the fast path; this one costs one sort
// of N keys per level (~log2 N sorts).
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <stdexcept>

#include "device_utils.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {

namespace {

constexpr int kBlock = 256;

int grid_for(i64 n) { return int(std::min<i64>(8192, std::max<i64>(1, (n + kBlock - 1) / kBlock))); }

__global__ __launch_bounds__(kBlock) void k_ref_init(u32* __restrict__ perm, u32* __restrict__ seg_lo,
                                                     u32* __restrict__ seg_n, i64 n) {
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += i64(gridDim.x) * kBlock) {
    perm[p] = u32(p);
    seg_lo[p] = 0;
    seg_n[p] = u32(n);
  }
}

// sort key of the row at position p for this level's sort
__global__ __launch_bounds__(kBlock) void k_ref_keys(const float* __restrict__ pts, int dim, int axis,
                                                     const u32* __restrict__ perm, const u32* __restrict__ seg_lo,
                                                     const u32* __restrict__ seg_n, i64 n, u64* __restrict__ keys) {
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += i64(gridDim.x) * kBlock) {
    const u32 lo = seg_lo[p], m = seg_n[p];
    u64 k;
    if (m <= 1) k = u64(p) << 32;                                   // finished slot: stays
    else if (u64(p) == u64(lo) + m - 1) k = (u64(lo) << 32) | 0xffffffffull;  // the unsorted last row
    else k = (u64(lo) << 32) | orderable(pts[i64(perm[p]) * dim + axis]);
    keys[p] = k;
  }
}

// segments of the next level: [lo, mid) | mid | (mid, lo + m)
__global__ __launch_bounds__(kBlock) void k_ref_split(u32* __restrict__ seg_lo, u32* __restrict__ seg_n, i64 n) {
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += i64(gridDim.x) * kBlock) {
    const u32 lo = seg_lo[p], m = seg_n[p];
    if (m <= 1) continue;
    const u32 mid = lo + m / 2;
    if (u32(p) < mid) {
      seg_n[p] = m / 2;
    } else if (u32(p) == mid) {
      seg_lo[p] = mid;
      seg_n[p] = 1;
    } else {
      seg_lo[p] = mid + 1;
      seg_n[p] = m - m / 2 - 1;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_ref_gather(const float* __restrict__ pts, const u32* __restrict__ ids,
                                                       u32 id_base, int dim, const u32* __restrict__ perm, i64 n,
                                                       float* __restrict__ out_pts, u32* __restrict__ out_ids) {
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += i64(gridDim.x) * kBlock) {
    const i64 r = perm[p];
    for (int c = 0; c < dim; ++c) out_pts[p * dim + c] = pts[r * dim + c];
    out_ids[p] = ids ? ids[r] : id_base + u32(r);
  }
}

int bitlen(u64 v) {
  int b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}

size_t align_up(size_t v) { return (v + 255) / 256 * 256; }

size_t sort_temp_bytes(i64 n) {
  size_t b = 0;
  PKD_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, b, static_cast<const u64*>(nullptr), static_cast<u64*>(nullptr),
                                          static_cast<const u32*>(nullptr), static_cast<u32*>(nullptr), size_t(n), 0,
                                          64));
  return b;
}

}  // namespace

ReferenceBuilder::ReferenceBuilder(i64 n, int dim, int depth0) : n_(n), dim_(dim), depth0_(depth0) {
  if (dim <= 0) throw std::invalid_argument("pkdtree: dim must be > 0");
  if (n < 0 || n >= (i64(1) << 32)) throw std::invalid_argument("pkdtree: n must be in [0, 2^32)");
  levels_ = 0;
  while ((n_ >> levels_) >= 2) ++levels_;  // the largest segment of level l has n >> l rows
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + std::max<size_t>(bytes, 1));
    return o;
  };
  const size_t nn = size_t(std::max<i64>(n_, 1));
  off_perm_[0] = take(nn * 4);
  off_perm_[1] = take(nn * 4);
  off_key_[0] = take(nn * 8);
  off_key_[1] = take(nn * 8);
  off_lo_ = take(nn * 4);
  off_n_ = take(nn * 4);
  tmp_bytes_ = sort_temp_bytes(n_);
  off_tmp_ = take(tmp_bytes_);
  ws_bytes_ = off;
}

void ReferenceBuilder::build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids,
                             void* workspace, hipStream_t stream) const {
  if (n_ == 0) return;
  char* ws = static_cast<char*>(workspace);
  u32* perm[2] = {reinterpret_cast<u32*>(ws + off_perm_[0]), reinterpret_cast<u32*>(ws + off_perm_[1])};
  u64* key[2] = {reinterpret_cast<u64*>(ws + off_key_[0]), reinterpret_cast<u64*>(ws + off_key_[1])};
  u32* seg_lo = reinterpret_cast<u32*>(ws + off_lo_);
  u32* seg_n = reinterpret_cast<u32*>(ws + off_n_);
  const int g = grid_for(n_);
  k_ref_init<<<g, kBlock, 0, stream>>>(perm[0], seg_lo, seg_n, n_);
  PKD_LAUNCH_CHECK();
  const int end_bit = 32 + bitlen(u64(n_));  // segment starts < n
  int cur = 0;
  for (int l = 0; l < levels_; ++l) {
    const int axis = (depth0_ + l) % dim_;
    k_ref_keys<<<g, kBlock, 0, stream>>>(pts, dim_, axis, perm[cur], seg_lo, seg_n, n_, key[0]);
    PKD_LAUNCH_CHECK();
    size_t tb = tmp_bytes_;
    PKD_HIP_CHECK(rocprim::radix_sort_pairs(ws + off_tmp_, tb, key[0], key[1], perm[cur], perm[cur ^ 1], size_t(n_), 0,
                                            end_bit, stream));
    cur ^= 1;
    k_ref_split<<<g, kBlock, 0, stream>>>(seg_lo, seg_n, n_);
    PKD_LAUNCH_CHECK();
  }
  k_ref_gather<<<g, kBlock, 0, stream>>>(pts, ids, id_base, dim_, perm[cur], n_, out_pts, out_ids);
  PKD_LAUNCH_CHECK();
}

}  // namespace pkdtree
