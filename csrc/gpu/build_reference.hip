// Reference-mode builder on the GPU: the reference's own (quirky) tree.
//
// build_tree_rec (kdtree_sequential.cpp:30-66, kdtree_mpi.cpp:60-100) sorts only the FIRST
// n - 1 points of every subrange on the node's axis (:46-48), takes list[n/2] as the median
// and recurses on [0, n/2) and [n/2 + 1, n): the last point of a subrange keeps its slot, so
// the tree violates the kd invariant and depends on array positions, not only
// on point sets. Level-synchronous reproduction on a u32 permutation (rows never move; the
// output rows are gathered once at the end):
//   * levels whose segments exceed the LDS finish (kFinCap rows): a segmented LSD radix sort of
//     every segment's first n - 1 positions on the level's 32-bit orderable key, four 8-bit
//     passes. Tiles never cross a segment (host-computed from the implicit geometry), so a pass
//     is: per-tile digit histograms laid out segment by segment, digit-major inside a segment
//     (k_rs_hist); ONE exclusive scan over them gives every (segment, digit, tile) its output
//     offset (k_scan_*); a stable scatter ranks each wave's items by ballot matching of the
//     digit bits (k_rs_scatter). The last position of every segment and the finished medians
//     are never touched, and four passes bring the result back into the same buffer.
//   * then one workgroup per segment (<= kFinCap rows) finishes all remaining levels in LDS:
//     per level every sortable row's rank inside its sub-segment is counted against the other
//     rows (stable: position breaks ties), rows move to their ranks, sub-segments split.
// The sorts are stable (ties keep their previous order) while std::sort is not, so the tree
// equals the reference's exactly when no two points of a segment share a key on its axis --
// always true for tie-free data, usually true for the reference generator at
// small N. Exact mode (gpu_build.hpp) is the fast path; this one is a parity mode.
#include <algorithm>
#include <stdexcept>

#include "device_utils.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {

namespace {

constexpr int kBlock = 256;
constexpr int kTile = 4096;      // sortable rows per radix tile (4 waves x 16 x 64)
constexpr int kFinCap = 2048;    // largest segment the LDS finish takes
constexpr int kScanChunk = kBlock * 16;

int grid_for(i64 n) { return int(std::min<i64>(8192, std::max<i64>(1, (n + kBlock - 1) / kBlock))); }

__global__ __launch_bounds__(kBlock) void k_ref_init(u32* __restrict__ perm, i64 n) {
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += i64(gridDim.x) * kBlock) perm[p] = u32(p);
}

using Tile = ReferenceBuilder::Tile;

// sort keys of the level's sortable positions (every tile's rows)
__global__ __launch_bounds__(kBlock) void k_ref_keys(const float* __restrict__ pts, int dim, int axis,
                                                     const u32* __restrict__ perm, const Tile* __restrict__ tiles,
                                                     u32* __restrict__ keys) {
  const Tile t = tiles[blockIdx.x];
  for (u32 e = threadIdx.x; e < t.len; e += kBlock) {
    const u32 p = t.pos0 + e;
    keys[p] = orderable(pts[i64(perm[p]) * dim + axis]);
  }
}

// per-tile digit histogram -> cnt[ent0 + digit * tseg + trel]
__global__ __launch_bounds__(kBlock) void k_rs_hist(const u32* __restrict__ keys, const Tile* __restrict__ tiles,
                                                    int shift, u32* __restrict__ cnt) {
  __shared__ u32 h[256];
  const Tile t = tiles[blockIdx.x];
  h[threadIdx.x] = 0;
  __syncthreads();
  for (u32 e = threadIdx.x; e < t.len; e += kBlock) atomicAdd(&h[(keys[t.pos0 + e] >> shift) & 255u], 1u);
  __syncthreads();
  cnt[size_t(t.ent0) + size_t(threadIdx.x) * t.tseg + t.trel] = h[threadIdx.x];
}

// exclusive scan of n words in place: chunk sums, a scan of the sums, chunk scans + base
__global__ __launch_bounds__(kBlock) void k_scan_sums(const u32* __restrict__ v, i64 n, u32* __restrict__ sums) {
  __shared__ u32 red[kBlock / 64];
  const i64 c0 = i64(blockIdx.x) * kScanChunk;
  u32 s = 0;
  for (int k = 0; k < 16; ++k) {
    const i64 i = c0 + i64(k) * kBlock + threadIdx.x;
    if (i < n) s += v[i];
  }
  s = dev::wave_incl_scan(s);
  if (dev::lane() == 63) red[threadIdx.x / 64] = s;
  __syncthreads();
  if (threadIdx.x == 0) sums[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// one block: exclusive scan of m block sums (m <= kBlock * 16)
__global__ __launch_bounds__(kBlock) void k_scan_top(u32* __restrict__ sums, int m) {
  __shared__ u32 ws[kBlock / 64];
  u32 loc[16];
  u32 s = 0;
  for (int k = 0; k < 16; ++k) {
    const int i = threadIdx.x * 16 + k;
    loc[k] = i < m ? sums[i] : 0u;
    s += loc[k];
  }
  const u32 incl = dev::wave_incl_scan(s);
  if (dev::lane() == 63) ws[threadIdx.x / 64] = incl;
  __syncthreads();
  u32 base = 0;
  for (int w = 0; w < int(threadIdx.x / 64); ++w) base += ws[w];
  u32 run = base + incl - s;
  for (int k = 0; k < 16; ++k) {
    const int i = threadIdx.x * 16 + k;
    if (i < m) sums[i] = run;
    run += loc[k];
  }
}

__global__ __launch_bounds__(kBlock) void k_scan_apply(u32* __restrict__ v, i64 n, const u32* __restrict__ sums) {
  __shared__ u32 ws[kBlock / 64];
  const i64 c0 = i64(blockIdx.x) * kScanChunk;
  u32 loc[16];
  u32 s = 0;
  for (int k = 0; k < 16; ++k) {  // thread t owns 16 consecutive words
    const i64 i = c0 + i64(threadIdx.x) * 16 + k;
    loc[k] = i < n ? v[i] : 0u;
    s += loc[k];
  }
  const u32 incl = dev::wave_incl_scan(s);
  if (dev::lane() == 63) ws[threadIdx.x / 64] = incl;
  __syncthreads();
  u32 base = sums[blockIdx.x];
  for (int w = 0; w < int(threadIdx.x / 64); ++w) base += ws[w];
  u32 run = base + incl - s;
  for (int k = 0; k < 16; ++k) {
    const i64 i = c0 + i64(threadIdx.x) * 16 + k;
    if (i < n) v[i] = run;
    run += loc[k];
  }
}

// stable scatter of one tile: wave w owns tile rows [w * 1024, (w + 1) * 1024); item i of lane
// l is row w * 1024 + i * 64 + l, so (w, i, l) is the input order. Lanes with equal digits are
// matched by 8 ballots; a digit's running count per wave lives in LDS.
__global__ __launch_bounds__(kBlock) void k_rs_scatter(const u32* __restrict__ kin, const u32* __restrict__ vin,
                                                       u32* __restrict__ kout, u32* __restrict__ vout,
                                                       const Tile* __restrict__ tiles, int shift,
                                                       const u32* __restrict__ off) {
  __shared__ u32 wc[kBlock / 64][256];
  const Tile t = tiles[blockIdx.x];
  const int w = threadIdx.x / 64, ln = dev::lane();
  for (int d = threadIdx.x; d < 4 * 256; d += kBlock) (&wc[0][0])[d] = 0u;
  __syncthreads();
  const u64 lt = (u64(1) << ln) - 1ull;
  u32 kk[16], vv[16], rk[16];
  for (int i = 0; i < 16; ++i) {
    const u32 e = u32(w) * 1024u + u32(i) * 64u + u32(ln);
    const bool valid = e < t.len;
    const u32 key = valid ? kin[t.pos0 + e] : 0u;
    kk[i] = key;
    vv[i] = valid ? vin[t.pos0 + e] : 0u;
    const u32 d = (key >> shift) & 255u;
    u64 m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const u64 bb = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    u32 base = 0;
    if (valid) base = wc[w][d];
    rk[i] = base + u32(__popcll(m & lt));
    if (valid && (m & lt) == 0ull) wc[w][d] = base + u32(__popcll(m));  // the group's first lane
  }
  __syncthreads();
  {  // wave prefix per digit
    const int d = threadIdx.x;
    u32 s = 0;
    for (int ww = 0; ww < kBlock / 64; ++ww) {
      const u32 c = wc[ww][d];
      wc[ww][d] = s;
      s += c;
    }
  }
  __syncthreads();
  for (int i = 0; i < 16; ++i) {
    const u32 e = u32(w) * 1024u + u32(i) * 64u + u32(ln);
    if (e >= t.len) continue;
    const u32 d = (kk[i] >> shift) & 255u;
    const u32 pos = t.seg_lo + (off[size_t(t.ent0) + size_t(d) * t.tseg + t.trel] - t.rows_before) + wc[w][d] + rk[i];
    kout[pos] = kk[i];
    vout[pos] = vv[i];
  }
}

// (lo, n) of segment j of level l of the implicit tree over n rows
__device__ __forceinline__ void seg_geometry(i64 n, int l, i64 j, i64* lo_out, i64* n_out) {
  i64 lo = 0, m = n;
  for (int b = l - 1; b >= 0; --b) {
    if ((j >> b) & 1) {
      lo = lo + m / 2 + 1;
      m = m - m / 2 - 1;
    } else {
      m = m / 2;
    }
    if (m < 0) m = 0;
  }
  *lo_out = lo;
  *n_out = m;
}

// One workgroup per segment of level lf (<= kFinCap rows): every remaining level in LDS.
__global__ __launch_bounds__(kBlock) void k_ref_finish(const float* __restrict__ pts, int dim, int depth0,
                                                       u32* __restrict__ perm, i64 n, int lf, int levels) {
  __shared__ u32 P[2][kFinCap], K[kFinCap];
  __shared__ unsigned short SL[kFinCap], SN[kFinCap];
  i64 lo = 0, m = 0;
  seg_geometry(n, lf, blockIdx.x, &lo, &m);
  if (m <= 1) return;
  const int M = int(m);
  for (int p = threadIdx.x; p < M; p += kBlock) {
    P[0][p] = perm[lo + p];
    SL[p] = 0;
    SN[p] = (unsigned short)M;
  }
  int cur = 0;
  __syncthreads();
  for (int l = lf; l < levels; ++l) {
    const int axis = (depth0 + l) % dim;
    for (int p = threadIdx.x; p < M; p += kBlock) {
      const int sl = SL[p], sn = SN[p];
      if (sn >= 2 && p != sl + sn - 1) K[p] = orderable(pts[i64(P[cur][p]) * dim + axis]);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < M; p += kBlock) {
      const int sl = SL[p], sn = SN[p];
      int dst = p;
      if (sn >= 2 && p != sl + sn - 1) {
        const u32 kp = K[p];
        int r = 0;
        for (int q = sl; q < sl + sn - 1; ++q) {
          const u32 kq = K[q];
          r += (kq < kp || (kq == kp && q < p)) ? 1 : 0;
        }
        dst = sl + r;
      }
      P[cur ^ 1][dst] = P[cur][p];
    }
    __syncthreads();
    cur ^= 1;
    for (int p = threadIdx.x; p < M; p += kBlock) {  // sub-segments of the next level
      const int sl = SL[p], sn = SN[p];
      if (sn <= 1) continue;
      const int mid = sl + sn / 2;
      if (p < mid) {
        SN[p] = (unsigned short)(sn / 2);
      } else if (p == mid) {
        SL[p] = (unsigned short)mid;
        SN[p] = 1;
      } else {
        SL[p] = (unsigned short)(mid + 1);
        SN[p] = (unsigned short)(sn - sn / 2 - 1);
      }
    }
    __syncthreads();
  }
  for (int p = threadIdx.x; p < M; p += kBlock) perm[lo + p] = P[cur][p];
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

size_t align_up(size_t v) { return (v + 255) / 256 * 256; }

void host_geometry(i64 n, int l, i64 j, i64* lo_out, i64* n_out) {
  i64 lo = 0, m = n;
  for (int b = l - 1; b >= 0; --b) {
    if ((j >> b) & 1) {
      lo = lo + m / 2 + 1;
      m = m - m / 2 - 1;
    } else {
      m = m / 2;
    }
    if (m < 0) m = 0;
  }
  *lo_out = lo;
  *n_out = m;
}

}  // namespace

ReferenceBuilder::ReferenceBuilder(i64 n, int dim, int depth0) : n_(n), dim_(dim), depth0_(depth0) {
  if (dim <= 0) throw std::invalid_argument("pkdtree: dim must be > 0");
  if (n < 0 || n >= (i64(1) << 32)) throw std::invalid_argument("pkdtree: n must be in [0, 2^32)");
  levels_ = 0;
  while ((n_ >> levels_) >= 2) ++levels_;  // the largest segment of level l has n >> l rows
  // global levels: while the largest segment exceeds the LDS finish
  lfin_ = 0;
  while (lfin_ < levels_ && (n_ >> lfin_) > kFinCap) ++lfin_;
  level_tile0_.push_back(0);
  for (int l = 0; l < lfin_; ++l) {
    const i64 segs = i64(1) << l;
    u32 rows_before = 0;
    for (i64 j = 0; j < segs; ++j) {
      i64 lo = 0, m = 0;
      host_geometry(n_, l, j, &lo, &m);
      if (m < 2) continue;
      const i64 sortable = m - 1;  // the last row of the segment keeps its slot
      const u32 ts = u32((sortable + kTile - 1) / kTile);
      const u32 t0 = u32(tiles_.size() - size_t(level_tile0_.back()));
      for (u32 k = 0; k < ts; ++k) {
        Tile t{};
        t.pos0 = u32(lo + i64(k) * kTile);
        t.len = u32(std::min<i64>(kTile, sortable - i64(k) * kTile));
        t.seg_lo = u32(lo);
        t.rows_before = rows_before;
        t.ent0 = 256u * t0;
        t.tseg = ts;
        t.trel = k;
        tiles_.push_back(t);
      }
      rows_before += u32(sortable);
    }
    level_tile0_.push_back(i64(tiles_.size()));
    max_tiles_ = std::max<i64>(max_tiles_, level_tile0_[size_t(l + 1)] - level_tile0_[size_t(l)]);
  }
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + std::max<size_t>(bytes, 1));
    return o;
  };
  const size_t nn = size_t(std::max<i64>(n_, 1));
  off_perm_[0] = take(nn * 4);
  off_perm_[1] = take(nn * 4);
  off_key_[0] = take(nn * 4);
  off_key_[1] = take(nn * 4);
  off_tiles_ = take(tiles_.size() * sizeof(Tile));
  const i64 ents = 256 * max_tiles_;
  off_cnt_ = take(size_t(ents) * 4);
  off_sums_ = take(size_t((ents + kScanChunk - 1) / kScanChunk + 1) * 4);
  if ((ents + kScanChunk - 1) / kScanChunk > i64(kBlock) * 16)
    throw std::invalid_argument("pkdtree: reference builder scan too large");
  ws_bytes_ = off;
}

void ReferenceBuilder::build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids,
                             void* workspace, hipStream_t stream) const {
  if (n_ == 0) return;
  char* ws = static_cast<char*>(workspace);
  u32* perm[2] = {reinterpret_cast<u32*>(ws + off_perm_[0]), reinterpret_cast<u32*>(ws + off_perm_[1])};
  u32* key[2] = {reinterpret_cast<u32*>(ws + off_key_[0]), reinterpret_cast<u32*>(ws + off_key_[1])};
  Tile* tiles = reinterpret_cast<Tile*>(ws + off_tiles_);
  u32* cnt = reinterpret_cast<u32*>(ws + off_cnt_);
  u32* sums = reinterpret_cast<u32*>(ws + off_sums_);
  if (!tiles_.empty())
    PKD_HIP_CHECK(hipMemcpyAsync(tiles, tiles_.data(), tiles_.size() * sizeof(Tile), hipMemcpyHostToDevice, stream));
  const int g = grid_for(n_);
  k_ref_init<<<g, kBlock, 0, stream>>>(perm[0], n_);
  PKD_LAUNCH_CHECK();
  for (int l = 0; l < lfin_; ++l) {
    const int axis = (depth0_ + l) % dim_;
    const Tile* lt = tiles + level_tile0_[size_t(l)];
    const int nt = int(level_tile0_[size_t(l + 1)] - level_tile0_[size_t(l)]);
    if (nt == 0) continue;
    const i64 ents = 256 * i64(nt);
    const int chunks = int((ents + kScanChunk - 1) / kScanChunk);
    k_ref_keys<<<nt, kBlock, 0, stream>>>(pts, dim_, axis, perm[0], lt, key[0]);
    PKD_LAUNCH_CHECK();
    for (int pass = 0; pass < 4; ++pass) {  // 8-bit digits, LSD; four passes end in buffer 0
      const int in = pass & 1, shift = 8 * pass;
      k_rs_hist<<<nt, kBlock, 0, stream>>>(key[in], lt, shift, cnt);
      PKD_LAUNCH_CHECK();
      k_scan_sums<<<chunks, kBlock, 0, stream>>>(cnt, ents, sums);
      PKD_LAUNCH_CHECK();
      k_scan_top<<<1, kBlock, 0, stream>>>(sums, chunks);
      PKD_LAUNCH_CHECK();
      k_scan_apply<<<chunks, kBlock, 0, stream>>>(cnt, ents, sums);
      PKD_LAUNCH_CHECK();
      k_rs_scatter<<<nt, kBlock, 0, stream>>>(key[in], perm[in], key[in ^ 1], perm[in ^ 1], lt, shift, cnt);
      PKD_LAUNCH_CHECK();
    }
  }
  if (lfin_ < levels_) {
    const i64 segs = i64(1) << lfin_;
    k_ref_finish<<<int(segs), kBlock, 0, stream>>>(pts, dim_, depth0_, perm[0], n_, lfin_, levels_);
    PKD_LAUNCH_CHECK();
  }
  k_ref_gather<<<g, kBlock, 0, stream>>>(pts, ids, id_base, dim_, perm[0], n_, out_pts, out_ids);
  PKD_LAUNCH_CHECK();
}

}  // namespace pkdtree
