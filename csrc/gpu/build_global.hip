// Global (HBM-streaming) levels of the level-synchronous kd-tree build + the host plan.
//
// Per global level l (segments = contiguous slot ranges of the implicit tree):
//   k_select    one workgroup per segment: prefix-scan the segment's bucket histogram and
//               pick the bucket b* that holds rank n/2 (exact counts: below / inside b*).
//   k_partition grid over all points: bucket -> zone (left / middle / right of b*), each
//               wave ranks its points per zone with ballots, one atomic per zone reserves a
//               run in the destination, rows are moved SoA (coalesced runs), and the next
//               level's histogram (next axis, child segment) is accumulated in LDS on the
//               fly and flushed once per block.
//   k_refine    one workgroup per segment: ranks the middle zone (typically a handful of
//               points; radix passes on the 64-bit (key,id) composite when it is large)
//               so the exact median lands on slot lo+n/2 and is written to the output.
// Replaces build_tree_rec's per-node std::sort (kdtree_sequential.cpp:30-66).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>
#include <sstream>
#include <vector>

#include "device_utils.hpp"
#include "pkdtree/gpu_build.hpp"
#include "pkdtree/hip_check.hpp"
#include "pkdtree/trace.hpp"
#include "subtree.hpp"
#include "top4.hpp"

namespace pkdtree {

using dev::BucketParams;
using dev::bucket_of;
using dev::make_params;
using dev::mbcnt;

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 16;                  // kItems * 4 waves = 64 (i,wave) groups per chunk
constexpr int kChunk = kBlock * kItems;     // 4096 points per partition chunk
constexpr int kMaxBins = 4096;              // per-segment histogram bins (global levels)
constexpr int kRefineCap = 2048;            // middle zone handled in LDS by one workgroup
constexpr int kRadixBits = 11;
constexpr i64 kLevelBlocks = 2048;          // partition-type grids of the top levels (large builds)
constexpr int kPairBins = 2048;             // bins of a level whose histogram a paired pass fuses (4 children)
constexpr int kTripleBins = 1024;           // bins of a level whose histogram a triple's scatter fuses (8 children)
constexpr int kRadixBins = 1 << kRadixBits;

struct SegState {
  u32 bstar;
  u32 cnt_less;
  u32 cnt_mid;
  u32 stage2;                 // 1: the median bucket is split again by a second histogram
  u32 cur[4];                 // zone cursors (relative to segment start)
  unsigned long long mid_min;  // composite (key,id) range of the middle zone
  unsigned long long mid_max;
  u32 sbstar;                 // stage 2: sub-bucket holding the median
  float p2lo, p2scale;        // stage 2: bucketing of the median bucket's value range
  u32 pad2;
  unsigned long long pivot;   // paired levels: composite key of the median (set by k_pivot*)
};

constexpr int kBins2 = 4096;  // stage-2 sub-buckets

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------------------
// Zero-fill of the per-build counters (error word, histograms). A plain kernel rather than
// hipMemsetAsync: it is an ordinary node under hipGraph capture, and one launch of ours costs
// less than the runtime's fill kernel.
__global__ __launch_bounds__(kBlock) void k_zero(u32* __restrict__ p, i64 n) {
  const i64 stride = i64(gridDim.x) * kBlock;
  for (i64 i = i64(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) p[i] = 0u;
}

void zero_u32(void* p, i64 n, hipStream_t stream) {
  if (n <= 0) return;
  const int grid = int(std::min<i64>(1024, (n + kBlock - 1) / kBlock));
  k_zero<<<grid, kBlock, 0, stream>>>(static_cast<u32*>(p), n);
  PKD_LAUNCH_CHECK();
}

// Geometry: heap-ordered (lo, n) of every segment of levels 0..L (node h: children 2h+1,
// 2h+2). Deterministic from n, so it is computed on the device once per build.
__global__ void k_geometry(i64* __restrict__ seg_lo, i64* __restrict__ seg_n, i64 heap_nodes, i64 n) {
  const i64 h = i64(blockIdx.x) * blockDim.x + threadIdx.x;
  if (h >= heap_nodes) return;
  const int l = 63 - __builtin_clzll(u64(h + 1));
  const i64 j = h + 1 - (i64(1) << l);
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
  seg_lo[h] = lo;
  seg_n[h] = m;
}

// Bounding boxes are reduced without global atomics: every prep block writes one partial row
// part[block][2 * dim] (orderable min | max), k_bbox_reduce folds them. (Same-address atomics
// from thousands of waves serialise in L2 and cost hundreds of microseconds.)
constexpr int kMaxBoxParts = 4096;
constexpr int kPrepRows = 64;  // rows per LDS transpose tile of the runtime-dim prep (one wave per column)

template <int D>
__device__ __forceinline__ void block_box_partial(const u32 (&mn)[D], const u32 (&mx)[D], u32* part) {
  __shared__ u32 red[kBlock / 64][2 * D];
  const int w = threadIdx.x / 64;
#pragma unroll
  for (int c = 0; c < D; ++c) {
    const u32 a = dev::wave_min_u32(mn[c]), b = dev::wave_max_u32(mx[c]);
    if (dev::lane() == 0) {
      red[w][c] = a;
      red[w][D + c] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * D) {
    const int c = threadIdx.x;
    u32 v = red[0][c];
    for (int k = 1; k < kBlock / 64; ++k) v = c < D ? min(v, red[k][c]) : max(v, red[k][c]);
    part[size_t(blockIdx.x) * 2 * D + c] = v;
  }
}

// One block per output word c (column min for c < dim, max above): 2 * dim blocks, so a
// 128-D box (256 words x thousands of partial rows) folds in one pass instead of 256
// sequential block-wide reductions.
__global__ __launch_bounds__(kBlock) void k_bbox_reduce(const u32* __restrict__ part, int nparts, int dim,
                                                        u32* __restrict__ bbox) {
  __shared__ u32 red[kBlock / 64];
  const int c = blockIdx.x;
  const bool is_min = c < dim;
  u32 v = is_min ? 0xffffffffu : 0u;
  for (int q = threadIdx.x; q < nparts; q += kBlock) {
    const u32 x = part[size_t(q) * 2 * dim + c];
    v = is_min ? min(v, x) : max(v, x);
  }
  v = is_min ? dev::wave_min_u32(v) : dev::wave_max_u32(v);
  if (dev::lane() == 0) red[threadIdx.x / 64] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 r = red[0];
    for (int k = 1; k < kBlock / 64; ++k) r = is_min ? min(r, red[k]) : max(r, red[k]);
    bbox[c] = r;
  }
}

// ---------------------------------------------------------------------------------------
// AoS input -> SoA working columns (+ ids column) and the bounding box (orderable u32).
// D > 0: one thread per row, the row's D loads issued before its D column stores (each
// column store is fully coalesced) and the box reduced in registers; D == 0: runtime dim.
template <int D>
__global__ __launch_bounds__(kBlock) void k_prep(const float* __restrict__ pts, const u32* __restrict__ ids,
                                                 u32 id_base, float* __restrict__ cols, i64 n, int dim,
                                                 u32* __restrict__ bbox, int rs, int ids_in_row, i64 ncol) {
  extern __shared__ __align__(16) u32 sbox[];  // [2*dim]
  const i64 stride = i64(gridDim.x) * kBlock;
  u32* idcol = reinterpret_cast<u32*>(cols + i64(dim) * ncol);
  if (D > 0) {
    constexpr int DD = D > 0 ? D : 1;
    u32 mn[DD], mx[DD];
#pragma unroll
    for (int c = 0; c < DD; ++c) {
      mn[c] = 0xffffffffu;
      mx[c] = 0u;
    }
    for (i64 r = i64(blockIdx.x) * kBlock + threadIdx.x; r < n; r += stride) {
      float v[DD];
#pragma unroll
      for (int c = 0; c < DD; ++c) v[c] = pts[r * rs + c];
      const u32 id = ids_in_row ? __float_as_uint(pts[r * rs + DD]) : (ids ? ids[r] : id_base + u32(r));
#pragma unroll
      for (int c = 0; c < DD; ++c) {
        cols[i64(c) * ncol + r] = v[c];
        const u32 k = orderable(v[c]);
        mn[c] = min(mn[c], k);
        mx[c] = max(mx[c], k);
      }
      idcol[r] = id;
    }
    block_box_partial<DD>(mn, mx, bbox);
    return;
  }
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) sbox[c] = (c < dim) ? 0xffffffffu : 0u;
  __syncthreads();
  const i64 total = n * i64(dim);
  for (i64 f = i64(blockIdx.x) * kBlock + threadIdx.x; f < total; f += stride) {
    const i64 r = f / dim;
    const int c = int(f - r * dim);
    const float v = pts[r * rs + c];
    cols[i64(c) * ncol + r] = v;
    const u32 k = orderable(v);
    atomicMin(&sbox[c], k);
    atomicMax(&sbox[dim + c], k);
  }
  for (i64 r = i64(blockIdx.x) * kBlock + threadIdx.x; r < n; r += stride)
    idcol[r] = ids_in_row ? __float_as_uint(pts[r * rs + dim]) : (ids ? ids[r] : id_base + u32(r));
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) bbox[size_t(blockIdx.x) * 2 * dim + c] = sbox[c];
}

// Runtime dim (> 8): tiles of kPrepRows rows are transposed through LDS, so both the row
// loads (contiguous rows) and the column stores (kPrepRows consecutive floats per column) are
// coalesced; the box is reduced per (wave, column) with one LDS atomic pair. (k_prep<0>
// stores one float per thread with a column stride between lanes: 10x slower at 128-D.)
// narrow (narrow columns): coordinate c is written only if it is the key of a global
// level j < narrow_k (axis (depth0 + j) % dim, so column j), then the id column (narrow_k) and
// the input row index (narrow_k + 1); the box still covers every coordinate.
__global__ __launch_bounds__(kBlock) void k_prep_tiled(const float* __restrict__ pts, const u32* __restrict__ ids,
                                                       u32 id_base, float* __restrict__ cols, i64 n, int dim,
                                                       u32* __restrict__ bbox, int rs, int ids_in_row, i64 ncol,
                                                       int narrow, int narrow_k, int depth0) {
  extern __shared__ __align__(16) u32 sbox[];  // [2*dim] box | [dim][kPrepRows + 1] tile
  u32* idcol = reinterpret_cast<u32*>(cols + i64(narrow ? narrow_k : dim) * ncol);
  auto out_col = [&](int c) { return narrow ? (c - depth0 % dim + dim) % dim : c; };
  const int ncol_out = narrow ? narrow_k : dim;
  u32* sb = sbox;                                           // [2 * dim]
  float* tile = reinterpret_cast<float*>(sbox + 2 * dim);   // [dim][kPrepRows + 1]
  constexpr int TR = kPrepRows;
  // dim dividing the block (16, 32, 64, 128, 256): every load of a thread is column tid % dim, so
  // the box is kept in two registers and reduced once per block (a wave reduction per 64 elements
  // of the transpose cost more than the copy: 500 k x 128D prep 0.20 ms for 256 MB)
  const bool regbox = kBlock % dim == 0;
  u32 bmn = 0xffffffffu, bmx = 0u;
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) sb[c] = (c < dim) ? 0xffffffffu : 0u;
  const int ln = dev::lane();
  for (i64 r0 = i64(blockIdx.x) * TR; r0 < n; r0 += i64(gridDim.x) * TR) {
    const int rows = int(min<i64>(TR, n - r0));
    __syncthreads();  // previous tile consumed (and sb initialised)
    // the tile's loads in flight together (kU per thread) before their LDS stores
    constexpr int kU = 16;
    const int tot = rows * dim;
    for (int k0 = threadIdx.x; k0 < tot; k0 += kBlock * kU) {
      float v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int k = k0 + u * kBlock;
        const int rr = k / dim, c = k - rr * dim;
        v[u] = k < tot ? pts[(r0 + rr) * rs + c] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int k = k0 + u * kBlock;
        const int rr = k / dim, c = k - rr * dim;
        if (k < tot) {
          tile[c * (TR + 1) + rr] = v[u];
          if (regbox) {
            bmn = min(bmn, orderable(v[u]));
            bmx = max(bmx, orderable(v[u]));
          }
        }
      }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < dim * TR; k += kBlock) {  // a wave = 64 rows of one column
      const int c = k / TR, rr = k - c * TR;
      const bool ok = rr < rows;
      const int oc = out_col(c);
      if (regbox && oc >= ncol_out) continue;  // (narrow: only the global levels' key columns)
      const float v = tile[c * (TR + 1) + rr];
      if (ok && oc < ncol_out) cols[i64(oc) * ncol + r0 + rr] = v;
      if (!regbox) {
        const u32 kv = ok ? orderable(v) : 0xffffffffu;
        const u32 mn = dev::wave_min_u32(kv), mx = dev::wave_max_u32(ok ? orderable(v) : 0u);
        if (ln == 0) {
          atomicMin(&sb[c], mn);
          atomicMax(&sb[dim + c], mx);
        }
      }
    }
    for (int rr = threadIdx.x; rr < rows; rr += kBlock) {
      const i64 r = r0 + rr;
      idcol[r] = ids_in_row ? __float_as_uint(pts[r * rs + dim]) : (ids ? ids[r] : id_base + u32(r));
      if (narrow) idcol[ncol + r] = u32(r);
    }
  }
  if (regbox && bmn <= bmx) {
    const int c = int(threadIdx.x) % dim;
    atomicMin(&sb[c], bmn);
    atomicMax(&sb[dim + c], bmx);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) bbox[size_t(blockIdx.x) * 2 * dim + c] = sb[c];
}

// d = 3, contiguous AoS input: a thread moves 4 rows with three 16-B loads and four 16-B
// column stores (x, y, z, id), all fully coalesced; columns are 256-B aligned (ncol % 64 == 0).
__global__ __launch_bounds__(kBlock) void k_prep3v(const float* __restrict__ pts, const u32* __restrict__ ids,
                                                   u32 id_base, float* __restrict__ cols, i64 n, i64 ncol,
                                                   u32* __restrict__ bbox, int write_ids) {
  const i64 nq = n / 4;
  const i64 stride = i64(gridDim.x) * kBlock;
  u32 mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
  const float4* in = reinterpret_cast<const float4*>(pts);
  float4* cx = reinterpret_cast<float4*>(cols);
  float4* cy = reinterpret_cast<float4*>(cols + ncol);
  float4* cz = reinterpret_cast<float4*>(cols + 2 * ncol);
  uint4* ci = reinterpret_cast<uint4*>(cols + 3 * ncol);
  auto upd = [&](int c, float v) {
    const u32 k = orderable(v);
    mn[c] = min(mn[c], k);
    mx[c] = max(mx[c], k);
  };
  // U quads per thread per iteration, all loads issued before any store (the compiler cannot
  // prove the AoS input and the columns disjoint, so it would otherwise serialise them)
  constexpr int U = 4;
  for (i64 t0 = i64(blockIdx.x) * kBlock + threadIdx.x; t0 < nq; t0 += stride * U) {
    float4 a[U], b[U], c[U];
    uint4 id[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 t = t0 + i64(u) * stride;
      const i64 tt = t < nq ? t : t0;
      a[u] = in[3 * tt];
      b[u] = in[3 * tt + 1];
      c[u] = in[3 * tt + 2];
      if (ids) id[u] = reinterpret_cast<const uint4*>(ids)[tt];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 t = t0 + i64(u) * stride;
      if (t >= nq) break;
      // rows: (a.x a.y a.z) (a.w b.x b.y) (b.z b.w c.x) (c.y c.z c.w)
      const float4 x = make_float4(a[u].x, a[u].w, b[u].z, c[u].y);
      const float4 y = make_float4(a[u].y, b[u].x, b[u].w, c[u].z);
      const float4 z = make_float4(a[u].z, b[u].y, c[u].x, c[u].w);
      if (!ids) {
        const u32 b0 = id_base + u32(4 * t);
        id[u] = make_uint4(b0, b0 + 1, b0 + 2, b0 + 3);
      }
      cx[t] = x;
      cy[t] = y;
      cz[t] = z;
      if (write_ids) ci[t] = id[u];
      upd(0, x.x); upd(0, x.y); upd(0, x.z); upd(0, x.w);
      upd(1, y.x); upd(1, y.y); upd(1, y.z); upd(1, y.w);
      upd(2, z.x); upd(2, z.y); upd(2, z.z); upd(2, z.w);
    }
  }
  for (i64 r = 4 * nq + i64(blockIdx.x) * kBlock + threadIdx.x; r < n; r += stride) {  // tail rows
    for (int c = 0; c < 3; ++c) {
      const float v = pts[r * 3 + c];
      cols[i64(c) * ncol + r] = v;
      upd(c, v);
    }
    if (write_ids) reinterpret_cast<u32*>(cols + 3 * ncol)[r] = ids ? ids[r] : id_base + u32(r);
  }
  block_box_partial<3>(mn, mx, bbox);
}

// bbox over SoA columns (distributed path: points arrive already in SoA).
__global__ __launch_bounds__(kBlock) void k_bbox_soa(const float* __restrict__ cols, i64 n, int dim,
                                                     u32* __restrict__ part, i64 ncol) {
  __shared__ u32 red[kBlock / 64][2];
  const i64 stride = i64(gridDim.x) * kBlock;
  for (int c = 0; c < dim; ++c) {
    u32 mn = 0xffffffffu, mx = 0u;
    for (i64 r = i64(blockIdx.x) * kBlock + threadIdx.x; r < n; r += stride) {
      const u32 k = orderable(cols[i64(c) * ncol + r]);
      mn = min(mn, k);
      mx = max(mx, k);
    }
    mn = dev::wave_min_u32(mn);
    mx = dev::wave_max_u32(mx);
    if (dev::lane() == 0) {
      red[threadIdx.x / 64][0] = mn;
      red[threadIdx.x / 64][1] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int k = 1; k < kBlock / 64; ++k) {
        mn = min(red[0][0], red[k][0]);
        mx = max(red[0][1], red[k][1]);
        red[0][0] = mn;
        red[0][1] = mx;
      }
      part[size_t(blockIdx.x) * 2 * dim + c] = red[0][0];
      part[size_t(blockIdx.x) * 2 * dim + dim + c] = red[0][1];
    }
    __syncthreads();
  }
}
__global__ void k_root(const u32* __restrict__ bbox, int dim, float* __restrict__ cells,
                       BucketParams* __restrict__ params, int axis0, int bins0) {
  for (int c = threadIdx.x; c < dim; c += blockDim.x) {
    cells[2 * c] = from_orderable(bbox[c]);
    cells[2 * c + 1] = from_orderable(bbox[dim + c]);
  }
  if (threadIdx.x == 0)
    params[0] = make_params(from_orderable(bbox[axis0]), from_orderable(bbox[dim + axis0]), bins0);
}

// Root cell given by the caller (a box holding every point, e.g. a distributed leaf's cell).
__global__ void k_cell_root(const float* __restrict__ cell, int dim, float* __restrict__ cells,
                            BucketParams* __restrict__ params, int axis0, int bins0) {
  for (int c = threadIdx.x; c < 2 * dim; c += blockDim.x) cells[c] = cell[c];
  if (threadIdx.x == 0) params[0] = make_params(cell[2 * axis0], cell[2 * axis0 + 1], bins0);
}

// ---------------------------------------------------------------------------------------
struct LevelArgs {
  const float* src;      // SoA columns of this level's input (dim coords + ids)
  float* dst;            // SoA columns of this level's output
  i64 ncol;              // column stride (= n)
  int dim;
  const i64* seg_lo;
  const i64* seg_n;
  SegState* state;       // heap-indexed
  BucketParams* params;  // heap-indexed (this level's axis)
  float* cells;          // heap-indexed [h][dim][2]
  i64 heap0;             // heap index of segment 0 of this level
  int bps;               // partition blocks per segment
  int axis;
  int next_axis;
  int bins;
  int next_bins;         // 0 => next level is not a global level (no fused histogram)
  const u32* hist;       // this level's histograms [segs][bins]
  u32* hist_next;        // next level's histograms [2*segs][next_bins]
  float* out_pts;
  u32* out_ids;
  u32* err;              // sticky error word (bit 0: partition overflow, bit 1: refine)
  int block_reserve;     // 1: count the block's zones first and reserve once per block
  int small_done;        // 1: k_refine_small already resolved middle zones of <= 64 points
  u32* hist2;            // stage-2 histograms [segs][kBins2] (levels with stage2)
  int colgroup;          // runtime-dim partition: columns moved per load round (8, 16, 32)
  // Column roles in src/dst. Classic: column c = coordinate c, column dim = id. Narrow
  // (high-dim AoS input): only the keys of the global levels travel (column l = level l's
  // key), then the id and the input row index; full rows are gathered from `in_rows` by
  // index where a median is written out.
  int kcol, nkcol;       // this / the next level's key column
  int idcol;             // id column
  int ncols;             // columns moved per row
  int narrow;            // 1: narrow columns (idcol + 1 holds the input row index)
  const float* in_rows;  // narrow: the AoS input, row stride in_rs floats
  i64 in_rs;
  int id_implicit;       // 1 (first level only): src has no id column, id of column row p = id_base0 + p
  u32 id_base0;
  int xcd;               // 1: the row-moving passes keep a segment's blocks on one XCD (seg_part)
};

// Segment s and part of this block in a (segments x bps) grid, and its index s * bps + part in
// (segment, part) order (per-block arrays are kept in that order). xcd (with a multiple of 8
// segments): blocks are dealt round-robin over the 8 XCDs (block b shares one with b + 8), so
// segment s is given the blocks b = s % 8 (mod 8): every block of a segment runs on one XCD, and
// the cache lines its blocks' zone runs share at their reservation edges are merged in that XCD's
// L2 instead of leaving it as partial writes from two or more L2s (100M x 8D k_g3_part wrote 4.37
// GB per pass for 3.6 GB of rows).
__device__ __forceinline__ void seg_part(int bps, int xcd, i64& s, int& part, i64& bidx) {
  const u32 b = blockIdx.x, nseg = gridDim.x / u32(bps);
  if (xcd && (nseg & 7u) == 0u) {
    const u32 x = b & 7u, q = b >> 3;
    s = i64(x) + 8 * i64(q / u32(bps));
    part = int(q % u32(bps));
  } else {
    s = i64(b / u32(bps));
    part = int(b % u32(bps));
  }
  bidx = s * bps + part;
}

// Id of src column row p (absolute), materialised or implicit (first level of a build whose
// prep skipped the id column).
__device__ __forceinline__ u32 src_id(const LevelArgs& a, i64 p) {
  return a.id_implicit ? a.id_base0 + u32(p) : reinterpret_cast<const u32*>(a.src)[i64(a.idcol) * a.ncol + p];
}
__device__ __forceinline__ float src_col(const LevelArgs& a, int c, i64 p) {
  return (c == a.idcol && a.id_implicit) ? __uint_as_float(a.id_base0 + u32(p)) : a.src[i64(c) * a.ncol + p];
}

// Zone of a point: 0 left of the median bucket, 1 inside (the middle zone), 2 right.
// Stage 2 splits the median bucket once more with its own linear sub-buckets.
__device__ __forceinline__ u32 zone_of(float key, const BucketParams& prm, int bins, u32 bstar, u32 stage2,
                                       const BucketParams& p2, u32 sbstar) {
  const u32 b = bucket_of(key, prm, bins);
  if (b != bstar) return b < bstar ? 0u : 2u;
  if (!stage2) return 1u;
  const u32 sb = bucket_of(key, p2, kBins2);
  return sb < sbstar ? 0u : (sb == sbstar ? 1u : 2u);
}

// Wave-aggregated min / max of the composite keys of the `active` lanes, one pair of
// atomics per wave (all lanes of the wave must call it).
__device__ __forceinline__ void wave_minmax_atomic(bool active, u64 k, unsigned long long* mn,
                                                   unsigned long long* mx) {
  const u64 m = __ballot(active);
  if (!m) return;
  const u64 lo = dev::wave_min_u64(active ? k : ~0ull);
  const u64 hi = dev::wave_max_u64(active ? k : 0ull);
  if (dev::lane() == __ffsll((long long)m) - 1) {
    atomicMin(mn, (unsigned long long)lo);
    atomicMax(mx, (unsigned long long)hi);
  }
}

// Sweep of one or two key columns over rows [lo + b0, lo + b1) with 16-B loads: the aligned
// bulk 4 rows per lane per load (2 loads per column in flight), the up to 3 rows before and
// after it one per lane. f(k0, k1, e) is called for every row (e relative to lo); no wave
// operations inside f (rows are not visited by all lanes together).
template <int NK, class F>
__device__ __forceinline__ void sweep_keys(const float* c0, const float* c1, i64 lo, i64 b0, i64 b1, F&& f) {
  const i64 abs0 = lo + b0, abs1 = lo + b1;
  const i64 A = min(abs1, (abs0 + 3) & ~i64(3));
  const i64 nv = (abs1 - A) >> 2;
  const i64 Bend = A + 4 * nv;
  {
    const int t = int(threadIdx.x);
    const bool head = t < 3 && abs0 + t < A, tail = t >= 3 && t < 6 && Bend + (t - 3) < abs1;
    if (head | tail) {
      const i64 p = head ? abs0 + t : Bend + (t - 3);
      f(c0[p], NK > 1 ? c1[p] : 0.0f, p - lo);
    }
  }
  const float4* v0 = reinterpret_cast<const float4*>(c0 + A);
  const float4* v1 = reinterpret_cast<const float4*>((NK > 1 ? c1 : c0) + A);
  constexpr int U4 = 2;
  for (i64 w0 = 0; w0 < nv; w0 += i64(kBlock) * U4) {
    float4 k[U4], m[U4];
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      const i64 v = w0 + i64(u) * kBlock + threadIdx.x;
      const i64 vi = v < nv ? v : 0;
      k[u] = v0[vi];
      if (NK > 1) m[u] = v1[vi];
    }
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      const i64 v = w0 + i64(u) * kBlock + threadIdx.x;
      if (v >= nv) continue;
      const i64 e = A - lo + 4 * v;
      f(k[u].x, NK > 1 ? m[u].x : 0.0f, e);
      f(k[u].y, NK > 1 ? m[u].y : 0.0f, e + 1);
      f(k[u].z, NK > 1 ? m[u].z : 0.0f, e + 2);
      f(k[u].w, NK > 1 ? m[u].w : 0.0f, e + 3);
    }
  }
}

// Histogram of a level's keys (used for the first global level only; later levels get
// theirs from the fused partition pass).
__global__ __launch_bounds__(kBlock) void k_hist(LevelArgs a, u32* __restrict__ hist) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  extern __shared__ __align__(16) u32 sh[];
  const i64 s = blockIdx.x / a.bps;
  const int part = blockIdx.x % a.bps;
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  for (int b = threadIdx.x; b < a.bins; b += kBlock) sh[b] = 0;
  __syncthreads();
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  const BucketParams p = a.params[h];
  const float* key = a.src + i64(a.kcol) * a.ncol;
  sweep_keys<1>(key, key, lo, b0, b1, [&](float k, float, i64) { atomicAdd(&sh[bucket_of(k, p, a.bins)], 1u); });
  __syncthreads();
  for (int b = threadIdx.x; b < a.bins; b += kBlock) {
    const u32 v = sh[b];
    if (v) atomicAdd(&hist[s * a.bins + b], v);
  }
}

// Block-wide exclusive scan of one value per thread (256 threads).
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32* sh4, u32* total) {
  const int w = threadIdx.x / 64;
  const u32 incl = dev::wave_incl_scan(v);
  if (dev::lane() == 63) sh4[w] = incl;
  __syncthreads();
  u32 off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kBlock / 64; ++k) {
    const u32 t = sh4[k];
    if (k < w) off += t;
    tot += t;
  }
  *total = tot;
  return off + incl - v;
}

__global__ __launch_bounds__(kBlock) void k_select(LevelArgs a) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  __shared__ u32 sh4[4];
  __shared__ u32 found[3];
  const i64 s = blockIdx.x;
  const i64 h = a.heap0 + s;
  const i64 n = a.seg_n[h];
  // Children's histograms are zeroed even for empty segments (their select reads them).
  if (a.next_bins > 0) {
    u32* hn = a.hist_next + (2 * s) * a.next_bins;
    for (int b = threadIdx.x; b < 2 * a.next_bins; b += kBlock) hn[b] = 0;
  }
  if (n <= 0) return;
  const u32 r = u32(n / 2);
  const u32* hs = a.hist + s * a.bins;
  const int per = (a.bins + kBlock - 1) / kBlock;
  const int b0 = min(a.bins, int(threadIdx.x) * per), b1 = min(a.bins, b0 + per);
  if (threadIdx.x == 0) found[0] = 0xffffffffu;  // (the scan's barriers order it before the finder)
  u32 sum = 0;
  for (int b = b0; b < b1; ++b) sum += hs[b];
  u32 total;
  const u32 excl = block_excl_scan(sum, sh4, &total);
  if (r >= excl && r < excl + sum) {
    u32 c = excl;
    for (int b = b0; b < b1; ++b) {
      const u32 v = hs[b];
      if (r < c + v) {
        found[0] = u32(b);
        found[1] = c;
        found[2] = v;
        break;
      }
      c += v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (found[0] == 0xffffffffu) {  // the histogram does not hold the median rank: only after a
      atomicOr(a.err, 2u);           // reported miss or overflow (rebuilt); empty zones keep the
      found[0] = found[1] = found[2] = 0u;  // passes inside the segment
    }
    SegState st;
    st.bstar = found[0];
    st.cnt_less = found[1];
    st.cnt_mid = found[2];
    st.cur[0] = 0;
    st.cur[1] = found[1];
    st.cur[2] = found[1] + found[2];
    st.cur[3] = 0;
    st.mid_min = ~0ull;
    st.mid_max = 0ull;
    st.stage2 = 0;
    st.sbstar = 0;
    st.pad2 = 0;
    {  // stage-2 bucketing of the median bucket's value range
      const BucketParams p = a.params[h];
      const float* cl = a.cells + h * 2 * a.dim;
      float lo2 = cl[2 * a.axis], hi2 = cl[2 * a.axis + 1];
      if (p.scale > 0.0f) {
        lo2 = p.lo + float(st.bstar) / p.scale;
        hi2 = p.lo + float(st.bstar + 1) / p.scale;
      }
      const BucketParams p2 = make_params(lo2, hi2, kBins2);
      st.p2lo = p2.lo;
      st.p2scale = p2.scale;
    }
    a.state[h] = st;
    if (a.next_bins > 0) {
      // Children's bucketing on the next axis. For dim > 1 the child cell on that axis is
      // the parent's; for dim == 1 it is approximated from the bucket edges (any monotone
      // bucketing is correct, this only sets the resolution).
      const float* cell = a.cells + h * 2 * a.dim;
      const float clo = cell[2 * a.next_axis], chi = cell[2 * a.next_axis + 1];
      BucketParams pl = make_params(clo, chi, a.next_bins), pr = pl;
      if (a.next_axis == a.axis) {
        const BucketParams p = a.params[h];
        if (p.scale > 0.0f) {
          const float e_hi = p.lo + float(st.bstar + 1) / p.scale;
          const float e_lo = p.lo + float(st.bstar) / p.scale;
          pl = make_params(clo, fminf(chi, e_hi), a.next_bins);
          pr = make_params(fmaxf(clo, e_lo), chi, a.next_bins);
        }
      }
      a.params[2 * h + 1] = pl;
      a.params[2 * h + 2] = pr;
    }
  }
}

// Stage 2 (top levels): histogram of the median bucket's points over kBins2 sub-buckets.
__global__ __launch_bounds__(kBlock) void k_hist2(LevelArgs a) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  __shared__ u32 sh[kBins2];
  const i64 s = blockIdx.x / a.bps;
  const int part = blockIdx.x % a.bps;
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  for (int b = threadIdx.x; b < kBins2; b += kBlock) sh[b] = 0;
  __syncthreads();
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  const BucketParams p = a.params[h];
  const SegState* st = a.state + h;
  const u32 bstar = st->bstar;
  BucketParams p2;
  p2.lo = st->p2lo;
  p2.scale = st->p2scale;
  const float* key = a.src + i64(a.kcol) * a.ncol;
  sweep_keys<1>(key, key, lo, b0, b1, [&](float k, float, i64) {
    if (bucket_of(k, p, a.bins) == bstar) atomicAdd(&sh[bucket_of(k, p2, kBins2)], 1u);
  });
  __syncthreads();
  for (int b = threadIdx.x; b < kBins2; b += kBlock) {
    const u32 v = sh[b];
    if (v) atomicAdd(&a.hist2[s * kBins2 + b], v);
  }
}

__global__ __launch_bounds__(kBlock) void k_select2(LevelArgs a) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  __shared__ u32 sh4[4];
  __shared__ u32 found[3];
  const i64 s = blockIdx.x;
  const i64 h = a.heap0 + s;
  const i64 n = a.seg_n[h];
  if (n <= 0) return;
  SegState* st = a.state + h;
  const u32 t = u32(n / 2) - st->cnt_less;  // rank inside the median bucket
  const u32* hs = a.hist2 + s * kBins2;
  constexpr int per = kBins2 / kBlock;
  if (threadIdx.x == 0) found[0] = 0xffffffffu;
  u32 sum = 0;
  for (int b = 0; b < per; ++b) sum += hs[threadIdx.x * per + b];
  u32 total;
  const u32 excl = block_excl_scan(sum, sh4, &total);
  if (t >= excl && t < excl + sum) {
    u32 c = excl;
    for (int b = 0; b < per; ++b) {
      const u32 v = hs[threadIdx.x * per + b];
      if (t < c + v) {
        found[0] = u32(threadIdx.x * per + b);
        found[1] = c;
        found[2] = v;
        break;
      }
      c += v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (found[0] == 0xffffffffu) {  // (as in k_select)
      atomicOr(a.err, 2u);
      found[0] = found[1] = found[2] = 0u;
    }
    const u32 cl = st->cnt_less + found[1];
    st->stage2 = 1;
    st->sbstar = found[0];
    st->cnt_less = cl;
    st->cnt_mid = found[2];
    st->cur[0] = 0;
    st->cur[1] = cl;
    st->cur[2] = cl + found[2];
  }
}

// NCOL > 0: rows of NCOL columns (dim + id) are loaded whole into registers before any
// store, so every chunk pays one HBM latency; NCOL == 0: runtime dim, columns are moved one
// at a time (loads of a column batched before its stores). Loads and stores never
// interleave per item: the compiler cannot prove src/dst disjoint and would otherwise
// serialise each load behind the previous store.
template <int NCOL, int KI>
__global__ __launch_bounds__(kBlock) void k_partition(LevelArgs a) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int kItems = KI;
  constexpr int kChunk = kBlock * KI;
  extern __shared__ __align__(16) u32 nh[];  // [2 * next_bins]
  __shared__ u32 gcnt[3][64];
  __shared__ unsigned long long bmin, bmax;  // block's middle-zone key range, flushed once
  const int dim = NCOL > 0 ? NCOL - 1 : a.dim;
  i64 s, bidx;
  int part;
  seg_part(a.bps, a.xcd, s, part, bidx);
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  const bool fuse = a.next_bins > 0;
  if (fuse) {
    for (int b = threadIdx.x; b < 2 * a.next_bins; b += kBlock) nh[b] = 0;
  }
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  SegState* st = a.state + h;
  const u32 bstar = st->bstar;
  const u32 stage2 = st->stage2, sbstar = st->sbstar;
  BucketParams p2;
  p2.lo = st->p2lo;
  p2.scale = st->p2scale;
  const BucketParams prm = a.params[h];
  BucketParams cprm[2] = {{0.f, 0.f}, {0.f, 0.f}};
  if (fuse) {
    cprm[0] = a.params[2 * h + 1];
    cprm[1] = a.params[2 * h + 2];
  }
  const float* __restrict__ src = a.src;
  float* __restrict__ dst = a.dst;
  const i64 nc = a.ncol;
  const int axis = a.axis, naxis = a.next_axis;
  const int w = threadIdx.x / 64;
  const int ln = dev::lane();
  __shared__ u32 bcur[4];
  if (threadIdx.x == 0) {
    bmin = ~0ull;
    bmax = 0ull;
  }
  if (a.block_reserve) {
    // Few segments and many blocks per segment: per-chunk cursor atomics would all hit the
    // same three words. Count this block's zones from the key column first (an extra 4 B
    // read per point, served from the Infinity Cache on the second pass) and reserve once.
    u32 cnt0 = 0, cnt1 = 0;
    const float* kc = src + i64(a.kcol) * nc + lo;
    constexpr int U = 8;
    for (i64 e0 = b0 + threadIdx.x; e0 < b1; e0 += kBlock * U) {
      float k[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const i64 e = e0 + i64(u) * kBlock;
        k[u] = e < b1 ? kc[e] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (e0 + i64(u) * kBlock >= b1) continue;
        const u32 z = zone_of(k[u], prm, a.bins, bstar, stage2, p2, sbstar);
        cnt0 += z == 0 ? 1u : 0u;
        cnt1 += z == 1 ? 1u : 0u;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      cnt0 += __shfl_xor(cnt0, o, 64);
      cnt1 += __shfl_xor(cnt1, o, 64);
    }
    if (ln == 0) {
      gcnt[0][w] = cnt0;
      gcnt[1][w] = cnt1;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
      u32 t0 = 0, t1 = 0;
      for (int k = 0; k < kBlock / 64; ++k) {
        t0 += gcnt[0][k];
        t1 += gcnt[1][k];
      }
      const u32 tz = threadIdx.x == 0 ? t0 : (threadIdx.x == 1 ? t1 : u32(b1 - b0) - t0 - t1);
      bcur[threadIdx.x] = tz ? atomicAdd(&st->cur[threadIdx.x], tz) : 0u;
    }
  }
  __syncthreads();

  // Compile-time rows (NCOL > 0): 16-B loads of 4 consecutive rows of a column per lane from a
  // 16-B aligned chunk start (as k_partition2); item i = 4 g + j, rows outside [b0, b1) masked.
  constexpr bool VEC = NCOL > 0 && KI % 4 == 0;
  const i64 cstart = VEC ? (((lo + b0) & ~i64(3)) - lo) : b0;
  for (i64 c0 = cstart; c0 < b1; c0 += kChunk) {
    constexpr int NR = NCOL > 0 ? NCOL : 1;
    float row[kItems][NR];
    float kk[NCOL > 0 ? 1 : kItems], nkk[NCOL > 0 ? 1 : kItems];
    i64 eitem[kItems];
    if constexpr (VEC) {
#pragma unroll
      for (int g = 0; g < kItems / 4; ++g) {
        const i64 e4 = c0 + (i64(g) * kBlock + threadIdx.x) * 4;
        const i64 p4 = lo + (e4 < b1 ? e4 : cstart);
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          const float4 v = *reinterpret_cast<const float4*>(src + i64(c) * nc + p4);
          row[4 * g + 0][c] = v.x;
          row[4 * g + 1][c] = v.y;
          row[4 * g + 2][c] = v.z;
          row[4 * g + 3][c] = v.w;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) eitem[4 * g + j] = e4 + j;
      }
    } else {
#pragma unroll
      for (int i = 0; i < kItems; ++i) {
        const i64 e = c0 + i * kBlock + threadIdx.x;
        eitem[i] = e;
        const i64 p = lo + (e < b1 ? e : b0);
        if (NCOL > 0) {
#pragma unroll
          for (int c = 0; c < NR; ++c) row[i][c] = src[i64(c) * nc + p];
        } else {
          kk[i] = src[i64(a.kcol) * nc + p];
          nkk[i] = src[i64(a.nkcol) * nc + p];
        }
      }
    }
    u32 zone_pre[kItems];  // (zone << 16) | rank-in-wave
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      const i64 e = eitem[i];
      const bool valid = e >= b0 && e < b1;
      // split-axis and next-axis keys: select chains over the compile-time row (no indexing)
      float key = NCOL > 0 ? row[i][0] : kk[i], nkey = NCOL > 0 ? row[i][0] : nkk[i];
      if (NCOL > 0) {
#pragma unroll
        for (int c = 1; c < NR - 1; ++c) {
          key = (c == axis) ? row[i][c] : key;
          nkey = (c == naxis) ? row[i][c] : nkey;
        }
      }
      u32 z = 3;
      if (valid) z = zone_of(key, prm, a.bins, bstar, stage2, p2, sbstar);
      const u64 m0 = __ballot(z == 0), m1 = __ballot(z == 1), m2 = __ballot(z == 2);
      if (ln == 0) {
        gcnt[0][i * 4 + w] = __popcll(m0);
        gcnt[1][i * 4 + w] = __popcll(m1);
        gcnt[2][i * 4 + w] = __popcll(m2);
      }
      const u64 mz = z == 0 ? m0 : (z == 1 ? m1 : m2);
      zone_pre[i] = (z << 16) | mbcnt(mz);
      if (m1 != 0) {  // rare: track the middle zone's composite key range
        u64 k = 0;
        if (z == 1)  // the id is in the register row when the dim is compile-time
          k = composite_key(key, NCOL > 0 ? __float_as_uint(row[i][NR - 1])
                                          : reinterpret_cast<const u32*>(src)[i64(a.idcol) * nc + lo + e]);
        wave_minmax_atomic(z == 1, k, &bmin, &bmax);
      }
      if (fuse && z < 3 && z != 1) {
        const int child = z == 0 ? 0 : 1;
        atomicAdd(&nh[child * a.next_bins + bucket_of(nkey, cprm[child], a.next_bins)], 1u);
      }
    }
    __syncthreads();
    if (w < 3) {  // wave w scans zone w over the 64 (item, wave) groups in slot order
      const u32 v = ln < kItems * 4 ? gcnt[w][ln] : 0u;
      const u32 incl = dev::wave_incl_scan(v);
      const u32 tot = __shfl(incl, 63, 64);
      u32 base = 0;
      if (a.block_reserve) {
        base = bcur[w];
        if (ln == 0) bcur[w] = base + tot;
      } else {
        if (ln == 0 && tot) base = atomicAdd(&st->cur[w], tot);
        base = __shfl(base, 0, 64);
      }
      gcnt[w][ln] = base + incl - v;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kItems; ++i) {  // zone_pre becomes the destination offset in the segment
      const u32 z = zone_pre[i] >> 16;
      u32 off = 0xffffffffu;
      if (z < 3) {
        off = gcnt[z][i * 4 + w] + (zone_pre[i] & 0xffffu);
        if (i64(off) >= n) {  // impossible unless histogram and keys disagree
          atomicOr(a.err, 1u);
          off = 0xffffffffu;
        }
      }
      zone_pre[i] = off;
    }
    if (NCOL > 0) {
#pragma unroll
      for (int i = 0; i < kItems; ++i) {
        if (zone_pre[i] != 0xffffffffu) {
          const i64 q = lo + zone_pre[i];
#pragma unroll
          for (int c = 0; c < NR; ++c) dst[i64(c) * nc + q] = row[i][c];
        }
      }
    } else {
      // runtime dim: G columns per round, all of a round's loads issued before its stores
      // (one HBM latency per round instead of per column)
      auto move = [&](auto gc) {
        constexpr int G = decltype(gc)::value;
        const int lastc = a.ncols - 1;
        for (int cg = 0; cg <= lastc; cg += G) {
          float v[G][kItems];
#pragma unroll
          for (int j = 0; j < G; ++j)
#pragma unroll
            for (int i = 0; i < kItems; ++i) {
              const i64 e = c0 + i * kBlock + threadIdx.x;
              const int c = cg + j <= lastc ? cg + j : lastc;
              v[j][i] = src[i64(c) * nc + lo + (e < b1 ? e : b0)];
            }
#pragma unroll
          for (int j = 0; j < G; ++j)
#pragma unroll
            for (int i = 0; i < kItems; ++i)
              if (cg + j <= lastc && zone_pre[i] != 0xffffffffu) dst[i64(cg + j) * nc + lo + zone_pre[i]] = v[j][i];
        }
      };
      if (a.colgroup >= 32) move(std::integral_constant<int, 32>{});
      else if (a.colgroup >= 16) move(std::integral_constant<int, 16>{});
      else move(std::integral_constant<int, 8>{});
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && bmin != ~0ull) {
    atomicMin(&st->mid_min, bmin);
    atomicMax(&st->mid_max, bmax);
  }
  if (fuse) {
    u32* hn = a.hist_next + (2 * s) * a.next_bins;
    for (int b = threadIdx.x; b < 2 * a.next_bins; b += kBlock) {
      const u32 v = nh[b];
      if (v) atomicAdd(&hn[b], v);
    }
  }
}

// Bitonic sort of (key, idx) pairs in LDS, cnt <= cap (cap a power of two).
__device__ void block_bitonic(u64* keys, u32* idx, int cnt, int cap) {
  int np = 1;
  while (np < cnt) np <<= 1;
  for (int i = cnt + threadIdx.x; i < np; i += kBlock) {
    keys[i] = ~0ull;
    idx[i] = 0xffffffffu;
  }
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np; i += kBlock) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const u64 ki = keys[i], kl = keys[l];
          if ((ki > kl) == up) {
            keys[i] = kl;
            keys[l] = ki;
            const u32 t = idx[i];
            idx[i] = idx[l];
            idx[l] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  (void)cap;
}

// Adds the next-level histogram contribution of a middle point that ended on `side`.
__device__ __forceinline__ void add_next_hist(const LevelArgs& a, i64 s, i64 h, int side, float nkey) {
  const BucketParams p = a.params[2 * h + 1 + side];
  const u32 nb = bucket_of(nkey, p, a.next_bins);
  atomicAdd(&a.hist_next[(2 * s + side) * a.next_bins + nb], 1u);
}

// CAP: largest middle zone sorted in LDS (keys + indices in dynamic LDS); larger zones are
// first narrowed by radix passes over the composite key.
// A segment's zone counts as the previous pass left them, clamped to the segment: they exceed it
// only after a reported miss or overflow (a tree that is rebuilt), and the refine / pivot passes
// then still read and write inside the segment.
__device__ __forceinline__ void zone_counts(const SegState& st, i64 n, i64* less, i64* mid) {
  const i64 l = min(i64(st.cnt_less), n);
  *less = l;
  *mid = min(i64(st.cnt_mid), n - l);
}

template <int CAP>
__device__ __forceinline__ void refine_body(LevelArgs a, i64 bid) {
  extern __shared__ __align__(16) u64 dynk[];
  u64* keys = dynk;
  u32* idx = reinterpret_cast<u32*>(dynk + CAP);
  __shared__ u32 rh[kRadixBins];
  __shared__ u32 sh4[4];
  __shared__ u32 info[4];
  const int dim = a.dim;
  const i64 s = bid;
  const i64 h = a.heap0 + s;
  const i64 n = a.seg_n[h];
  if (n <= 0) return;
  const i64 lo = a.seg_lo[h];
  const SegState st = a.state[h];
  const i64 nc = a.ncol;
  float* __restrict__ dst = a.dst;           // the middle zone lives here
  float* __restrict__ alt = const_cast<float*>(a.src);  // dead input buffer: staging area
  const bool fuse = a.next_bins > 0;
  if (a.small_done && st.cnt_mid <= 64) return;
  i64 cl = 0, cm = 0;
  zone_counts(st, n, &cl, &cm);
  i64 zlo = lo + cl;
  i64 zc = cm;
  i64 t = n / 2 - cl;
  auto ckey = [&](i64 p) -> u64 {
    const u32 id = reinterpret_cast<const u32*>(dst)[i64(a.idcol) * nc + p];
    return composite_key(dst[i64(a.kcol) * nc + p], id);
  };
  auto copy_row = [&](float* to, i64 q, const float* from, i64 p) {
    for (int c = 0; c < a.ncols; ++c) to[i64(c) * nc + q] = from[i64(c) * nc + p];
  };
  // Whole-block column-major moves of the zone's rows [zlo, zlo + cnt): consecutive threads
  // touch consecutive rows of one column, so every load is independent of the others (a row
  // per thread would chain dim + 1 load/store pairs, ~130 HBM latencies at 128-D).
  constexpr u32 kNoSlot = 0xffffffffu;
  const int ncols = a.ncols;
  // kMoveU elements per thread per round, all loads of a round before its stores (a loop of
  // single load/store pairs would pay one HBM latency per element per thread: at 128-D a
  // 40-row zone is 20 such rounds per move)
  constexpr int kMoveU = 8;
  auto move_cols = [&](float* to, const float* from, int cnt, int mode) {  // 0 scatter, 1 gather, 2 copy
    const int total = cnt * ncols;
    for (int k0 = threadIdx.x; k0 < total; k0 += kBlock * kMoveU) {
      float v[kMoveU];
      u32 dd[kMoveU];
#pragma unroll
      for (int u = 0; u < kMoveU; ++u) {
        const int k = k0 + u * kBlock;
        const int c = k / max(cnt, 1), e = k - c * cnt;
        dd[u] = kNoSlot;
        v[u] = 0.0f;
        if (k < total) {
          const u32 src_e = mode == 1 ? idx[e] : u32(e);
          dd[u] = mode == 0 ? idx[e] : u32(e);
          v[u] = from[i64(c) * nc + zlo + src_e];
        }
      }
#pragma unroll
      for (int u = 0; u < kMoveU; ++u) {
        const int k = k0 + u * kBlock;
        const int c = k / max(cnt, 1);
        if (k < total && dd[u] != kNoSlot) to[i64(c) * nc + zlo + dd[u]] = v[u];
      }
    }
  };
  auto scatter_cols = [&](float* to, const float* from, int cnt) { move_cols(to, from, cnt, 0); };  // to[idx[e]] = from[e]
  auto gather_cols = [&](float* to, const float* from, int cnt) { move_cols(to, from, cnt, 1); };   // to[e] = from[idx[e]]
  auto copy_cols = [&](float* to, const float* from, int cnt) { move_cols(to, from, cnt, 2); };

  // Middle zones above one wave: radix passes over the composite key, 11 bits at a time
  // starting at the highest differing bit, each keeping only the digit bucket that holds
  // rank t (a median bucket of ~1-2k rows needs one pass; a full LDS sort of it would take
  // one workgroup ~66 barrier stages).
  if (zc > 64) {
    const u64 diff = u64(st.mid_min) ^ u64(st.mid_max);
    int hb = diff ? 63 - __builtin_clzll(diff) : 0;
    while (zc > 64) {
      const int shift = hb >= kRadixBits - 1 ? hb - (kRadixBits - 1) : 0;
      const bool coop = zc <= CAP;  // destinations fit the LDS map: move rows column-major
      for (int b = threadIdx.x; b < kRadixBins; b += kBlock) rh[b] = 0;
      if (threadIdx.x == 0) info[0] = 0xffffffffu;
      __syncthreads();
      for (i64 e = threadIdx.x; e < zc; e += kBlock)
        atomicAdd(&rh[u32(ckey(zlo + e) >> shift) & (kRadixBins - 1)], 1u);
      __syncthreads();
      {
        const int per = kRadixBins / kBlock;
        u32 sum = 0;
        for (int b = 0; b < per; ++b) sum += rh[threadIdx.x * per + b];
        u32 total;
        const u32 excl = block_excl_scan(sum, sh4, &total);
        if (u64(t) >= excl && u64(t) < u64(excl) + sum) {
          u32 c = excl;
          for (int b = 0; b < per; ++b) {
            const u32 v = rh[threadIdx.x * per + b];
            if (u64(t) < u64(c) + v) {
              info[0] = u32(threadIdx.x * per + b);
              info[1] = c;
              info[2] = v;
              break;
            }
            c += v;
          }
        }
        __syncthreads();
      }
      const u32 bsel = info[0], cl = info[1], ce = info[2];
      if (bsel == 0xffffffffu || i64(cl) + ce > zc) {  // rank t not in the zone (only after a reported
        if (threadIdx.x == 0) atomicOr(a.err, 2u);    // miss): stop inside the segment
        return;
      }
      if (threadIdx.x == 0) {
        rh[0] = 0;       // reuse as cursors
        rh[1] = cl;
        rh[2] = cl + ce;
      }
      __syncthreads();
      for (i64 e0 = 0; e0 < zc; e0 += kBlock) {
        const i64 e = e0 + threadIdx.x;
        u32 z = 3;
        if (e < zc) {
          const u32 d = u32(ckey(zlo + e) >> shift) & (kRadixBins - 1);
          z = d < bsel ? 0u : (d == bsel ? 1u : 2u);
        }
        u32 dest = 0;
#pragma unroll
        for (u32 zz = 0; zz < 3; ++zz) {
          const u64 m = __ballot(z == zz);
          if (m) {
            const int leader = __ffsll((long long)m) - 1;
            u32 base = 0;
            if (dev::lane() == leader) base = atomicAdd(&rh[zz], u32(__popcll(m)));
            base = __shfl(base, leader, 64);
            if (z == zz) dest = base + mbcnt(m);
          }
        }
        if (z < 3 && dest >= zc) {
          atomicOr(a.err, 2u);
          z = 3;
        }
        if (z < 3) {
          if (coop) idx[e] = dest;  // rows move below, column by column
          else copy_row(alt, zlo + dest, dst, zlo + e);
          if (fuse && z != 1) add_next_hist(a, s, h, z == 0 ? 0 : 1, dst[i64(a.nkcol) * nc + zlo + e]);
        } else if (coop && e < zc) {
          idx[e] = kNoSlot;
        }
      }
      __syncthreads();
      if (coop) {
        scatter_cols(alt, dst, int(zc));
        __syncthreads();
        copy_cols(dst, alt, int(zc));
      } else {
        for (i64 e = threadIdx.x; e < zc; e += kBlock) copy_row(dst, zlo + e, alt, zlo + e);
      }
      __syncthreads();
      zlo += cl;
      zc = ce;
      t -= cl;
      if (shift == 0) break;
      hb = shift - 1;
    }
  }

  // Final ranking of the (small) middle zone.
  const i64 mpos = lo + n / 2;
  constexpr int kInPlaceU = 32;  // zones of up to 32 * kBlock values are permuted in registers
  const bool inplace = zc <= 64 && zc * ncols <= kInPlaceU * kBlock;
  if (zc <= 64) {
    if (threadIdx.x < 64) {
      const int l = dev::lane();
      const bool valid = l < zc;
      const u64 k = valid ? ckey(zlo + l) : ~0ull;
      u32 rank = 0;
      for (int j = 0; j < zc; ++j) rank += dev::shfl_u64(k, j) < k ? 1u : 0u;
      if (valid) idx[l] = rank < zc ? rank : kNoSlot;
    }
    __syncthreads();
    if (inplace) {  // every value of the zone in registers, one barrier, then the permuted stores
      const int cnt = max(int(zc), 1), total = int(zc) * ncols;
      float v[kInPlaceU];
#pragma unroll
      for (int u = 0; u < kInPlaceU; ++u) {
        const int k = int(threadIdx.x) + u * kBlock;
        const int c = k / cnt, e = k - c * cnt;
        v[u] = k < total ? dst[i64(c) * nc + zlo + e] : 0.0f;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kInPlaceU; ++u) {
        const int k = int(threadIdx.x) + u * kBlock;
        const int c = k / cnt, e = k - c * cnt;
        if (k < total && idx[e] != kNoSlot) dst[i64(c) * nc + zlo + idx[e]] = v[u];
      }
    } else {
      scatter_cols(alt, dst, int(zc));
    }
  } else {
    for (i64 e = threadIdx.x; e < zc; e += kBlock) {
      keys[e] = ckey(zlo + e);
      idx[e] = u32(e);
    }
    __syncthreads();
    block_bitonic(keys, idx, int(zc), CAP);
    gather_cols(alt, dst, int(zc));
  }
  __syncthreads();
  if (!inplace) copy_cols(dst, alt, int(zc));
  const float* zb = inplace ? dst : alt;  // the ordered zone (same values in both after the copy)
  __syncthreads();
  // the median row: one column per thread (a single thread would chain dim dependent
  // load/store pairs)
  if (a.narrow) {  // gathered from the input row
    const u32 r = reinterpret_cast<const u32*>(zb)[i64(a.idcol + 1) * nc + zlo + t];
    for (int c = threadIdx.x; c < dim; c += kBlock) a.out_pts[mpos * dim + c] = a.in_rows[i64(r) * a.in_rs + c];
    if (threadIdx.x == 0) a.out_ids[mpos] = reinterpret_cast<const u32*>(zb)[i64(a.idcol) * nc + zlo + t];
  } else {
    for (int c = threadIdx.x; c <= dim; c += kBlock) {
      const float v = zb[i64(c) * nc + zlo + t];
      if (c < dim) a.out_pts[mpos * dim + c] = v;
      else a.out_ids[mpos] = __float_as_uint(v);
    }
  }
  if (fuse)
    for (i64 e = threadIdx.x; e < zc; e += kBlock)
      if (e != t) add_next_hist(a, s, h, e < t ? 0 : 1, zb[i64(a.nkcol) * nc + zlo + e]);
  // Children cells: the split value bounds the split axis.
  const float split = zb[i64(a.kcol) * nc + zlo + t];
  const float* cell = a.cells + h * 2 * dim;
  float* cl_ = a.cells + (2 * h + 1) * 2 * dim;
  float* cr_ = a.cells + (2 * h + 2) * 2 * dim;
  for (int c = threadIdx.x; c < dim; c += kBlock) {
    const float clo = cell[2 * c], chi = cell[2 * c + 1];
    cl_[2 * c] = clo;
    cl_[2 * c + 1] = c == a.axis ? split : chi;
    cr_[2 * c] = c == a.axis ? split : clo;
    cr_[2 * c + 1] = chi;
  }
}

// One wave per segment for the common case of a middle zone of <= 64 points: each lane
// holds one whole row (NCOL = dim + 1 <= 9 registers), ranks its composite key against the
// other lanes with shuffles and writes the row back in place (a wave's stores issue only
// after all of its loads returned, so in-place is safe inside the wave).
template <int NCOL>
__device__ __forceinline__ void refine_small_body(LevelArgs a, i64 segs, i64 bid) {
  constexpr int D = NCOL - 1;
  const i64 s = bid * (kBlock / 64) + threadIdx.x / 64;
  if (s >= segs) return;
  const i64 h = a.heap0 + s;
  const i64 n = a.seg_n[h];
  if (n <= 0) return;
  const SegState st = a.state[h];
  if (st.cnt_mid > 64) return;
  const i64 lo = a.seg_lo[h];
  i64 cl = 0, cm = 0;
  zone_counts(st, n, &cl, &cm);
  const int zc = int(cm);
  const int t = int(n / 2 - cl);
  const i64 zlo = lo + cl;
  const i64 nc = a.ncol;
  const int l = dev::lane();
  const bool valid = l < zc;
  float row[NCOL];
#pragma unroll
  for (int c = 0; c < NCOL; ++c) row[c] = valid ? a.dst[i64(c) * nc + zlo + l] : 0.0f;
  float key = row[0], nkey = row[0];
#pragma unroll
  for (int c = 1; c < D; ++c) {
    key = c == a.axis ? row[c] : key;
    nkey = c == a.next_axis ? row[c] : nkey;
  }
  const u32 id = __float_as_uint(row[D]);
  const u64 k = valid ? composite_key(key, id) : ~0ull;
  u32 rank = 0;
  for (int j = 0; j < zc; ++j) rank += dev::shfl_u64(k, j) < k ? 1u : 0u;
  if (!valid) return;
#pragma unroll
  for (int c = 0; c < NCOL; ++c) a.dst[i64(c) * nc + zlo + rank] = row[c];
  if (int(rank) == t) {
    const i64 mpos = lo + n / 2;
#pragma unroll
    for (int c = 0; c < D; ++c) a.out_pts[mpos * D + c] = row[c];
    a.out_ids[mpos] = id;
    const float* cell = a.cells + h * 2 * D;
    float* cl_ = a.cells + (2 * h + 1) * 2 * D;
    float* cr_ = a.cells + (2 * h + 2) * 2 * D;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      const float clo = cell[2 * c], chi = cell[2 * c + 1];
      cl_[2 * c] = clo;
      cl_[2 * c + 1] = c == a.axis ? key : chi;
      cr_[2 * c] = c == a.axis ? key : clo;
      cr_[2 * c + 1] = chi;
    }
  } else if (a.next_bins > 0) {
    add_next_hist(a, s, h, int(rank) < t ? 0 : 1, nkey);
  }
}

// =====================================================================================
// Paired global levels: levels l and l+1 are moved by ONE scatter pass instead of two.
//   k_scan       keys of l and l+1 only (8 B / row): rows of level l's median bucket are
//                compacted into their middle-zone area of dst (scratch), every other row
//                adds its level-(l+1) key to its child's histogram (fused, LDS);
//   k_pivot*     exact median of level l among the compacted rows (wave ranking, or a radix
//                select over the composite key): written to the output, its composite key
//                kept as the segment's pivot, the other middle rows complete the children's
//                histograms, children cells set;
//   k_select     level l+1 as usual;
//   k_partition2 one read + one write of every row: child (level l, from the bucket or the
//                pivot comparison) and zone inside the child (level l+1) give 6 destination
//                zones; the level-(l+2) histograms of the 4 grandchildren are fused in;
//   k_refine*    level l+1's middle zones as usual.
// Traffic per two levels: 8 + 16 + 16 B / row instead of 2 x (16 + 16).
struct PairArgs {
  int stage2_1;          // level l+1 median buckets split again (k_hist2p + k_select2)
  int bins1;             // level l+1 bins
  int axis2;             // level l+2 axis
  int bins2;             // level l+2 bins (0: l+2 is the subtree level)
  u32* hist2n;           // level l+2 histograms [4 * segs][bins2]
  // Prefix placement (top pairs with a second-stage level l+1): k_hist2p counts each block's
  // rows whose zone is already certain (child known, level-(l+1) bucket != the child's median
  // bucket) per (child, left/right) into bcnt[block][4]; k_block_bases turns them into
  // per-block write offsets bbase[block][4], so k_partition2 needs no counting pass.
  u32* bcnt = nullptr;
  u32* bbase = nullptr;
};

template <int NCOL>
__global__ __launch_bounds__(kBlock) void k_scan(LevelArgs a) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  extern __shared__ __align__(16) u32 nh[];  // [2 * next_bins] + 64 per-lane dummy words
  constexpr int D = NCOL - 1;
  const i64 s = blockIdx.x / a.bps;
  const int part = blockIdx.x % a.bps;
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  const int nb = a.next_bins;
  for (int b = threadIdx.x; b < 2 * nb; b += kBlock) nh[b] = 0;
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  SegState* st = a.state + h;
  const u32 bstar = st->bstar, stage2 = st->stage2, sbstar = st->sbstar;
  BucketParams p2;
  p2.lo = st->p2lo;
  p2.scale = st->p2scale;
  const BucketParams prm = a.params[h];
  const BucketParams cp0 = a.params[2 * h + 1], cp1 = a.params[2 * h + 2];
  const float* __restrict__ src = a.src;
  float* __restrict__ dst = a.dst;
  const i64 nc = a.ncol;
  const float* kc = src + i64(a.axis) * nc + lo;
  const float* nkc = src + i64(a.next_axis) * nc + lo;
  const int ln = dev::lane();
  // Middle rows (the median bucket) are only noted during the sweep (their offsets in LDS);
  // after it the block reserves them once (same-address atomics on the segment cursor from
  // every wave would serialise in L2) and copies them with all threads, so no wave stalls
  // on row loads inside the sweep.
  constexpr int kStage = 512;
  __shared__ u32 sidx[kStage];
  __shared__ u32 mcnt, mbase;
  __shared__ unsigned long long bmin, bmax;
  if (threadIdx.x == 0) {
    mcnt = 0;
    bmin = ~0ull;
    bmax = 0ull;
  }
  __syncthreads();
  // One row: its level-l zone; rows certain to go left / right add their level-(l+1) key to
  // that child's histogram (one LDS atomic, rows of the median bucket and absent rows add 0 to
  // a per-lane dummy word), rows of the median bucket are noted for staging. Every lane of a
  // wave calls it together (ballots).
  const u32 hdummy = u32(2 * nb) + u32(ln);
  auto visit = [&](float kv, float nkv, i64 e, bool valid) {
    const u32 z = valid ? zone_of(kv, prm, a.bins, bstar, stage2, p2, sbstar) : 3u;
    const u32 bl = bucket_of(nkv, cp0, nb), br = u32(nb) + bucket_of(nkv, cp1, nb);
    const u32 hb = z == 0 ? bl : br;
    const bool side = (z == 0) | (z == 2);
    atomicAdd(&nh[side ? hb : hdummy], 1u);
    const u64 m = __ballot(z == 1);
    if (m) {  // rare: note the median bucket's rows
      const int leader = __ffsll((long long)m) - 1;
      u32 base = 0;
      if (ln == leader) base = atomicAdd(&mcnt, u32(__popcll(m)));
      base = __shfl(base, leader, 64);
      const u32 slot = base + mbcnt(m);
      const bool direct = z == 1 && slot >= u32(kStage);
      if (z == 1 && !direct) sidx[slot] = u32(e - b0);
      if (__ballot(direct)) {  // staging full: reserve and copy directly
        u64 ck = 0;
        if (direct) {
          const u32 g = atomicAdd(&st->cur[1], 1u);
          if (i64(g) >= n) {
            atomicOr(a.err, 1u);
          } else {
#pragma unroll
            for (int c = 0; c < NCOL; ++c) dst[i64(c) * nc + lo + g] = src_col(a, c, lo + e);
          }
          ck = composite_key(kv, src_id(a, lo + e));
        }
        wave_minmax_atomic(direct, ck, &bmin, &bmax);
      }
    }
  };
  // The 16-B aligned bulk of the block's rows is read with 16-B loads (4 rows of each key
  // column per load); the up to 3 rows before and after it one per lane, in one extra round.
  const i64 abs0 = lo + b0, abs1 = lo + b1;
  const i64 A = min(abs1, (abs0 + 3) & ~i64(3));
  const i64 nv = (abs1 - A) >> 2;
  const i64 Bend = A + 4 * nv;
  {
    const int t = int(threadIdx.x);
    const bool head = t < 3 && abs0 + t < A, tail = t >= 3 && t < 6 && Bend + (t - 3) < abs1;
    const i64 e = head ? abs0 + t - lo : (tail ? Bend + (t - 3) - lo : 0);
    const bool v = head | tail;
    const float kv = v ? kc[e] : 0.0f, nkv = v ? nkc[e] : 0.0f;
    visit(kv, nkv, e, v);
  }
  const float4* kc4 = reinterpret_cast<const float4*>(src + i64(a.axis) * nc + A);
  const float4* nk4 = reinterpret_cast<const float4*>(src + i64(a.next_axis) * nc + A);
  constexpr int U4 = 2;  // 2 x 16 B per column in flight per thread
  for (i64 v0 = 0; v0 < nv; v0 += kBlock * U4) {
    float4 k[U4], nk[U4];
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      const i64 v = v0 + i64(u) * kBlock + threadIdx.x;
      const i64 vi = v < nv ? v : 0;
      k[u] = kc4[vi];
      nk[u] = nk4[vi];
    }
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      const i64 v = v0 + i64(u) * kBlock + threadIdx.x;
      const bool in = v < nv;
      const i64 e = A - lo + 4 * v;
      visit(k[u].x, nk[u].x, e, in);
      visit(k[u].y, nk[u].y, e + 1, in);
      visit(k[u].z, nk[u].z, e + 2, in);
      visit(k[u].w, nk[u].w, e + 3, in);
    }
  }
  __syncthreads();
  const u32 staged = min(mcnt, u32(kStage));
  if (threadIdx.x == 0) mbase = staged ? atomicAdd(&st->cur[1], staged) : 0u;
  __syncthreads();
  for (u32 r0 = 0; r0 < staged; r0 += kBlock) {  // uniform trip count: every lane reaches the wave ops
    const u32 k2 = r0 + threadIdx.x;
    const bool act = k2 < staged;
    const i64 q = i64(mbase) + k2;
    u64 ck = 0;
    if (act) {
      const i64 e = b0 + sidx[k2];
      float row[NCOL];
#pragma unroll
      for (int c = 0; c < NCOL; ++c) row[c] = src_col(a, c, lo + e);
      if (q >= n) {
        atomicOr(a.err, 1u);
      } else {
#pragma unroll
        for (int c = 0; c < NCOL; ++c) dst[i64(c) * nc + lo + q] = row[c];
      }
      float key = row[0];
#pragma unroll
      for (int c = 1; c < D; ++c) key = c == a.axis ? row[c] : key;
      ck = composite_key(key, __float_as_uint(row[D]));
    }
    wave_minmax_atomic(act, ck, &bmin, &bmax);
  }
  __syncthreads();
  if (threadIdx.x == 0 && bmin != ~0ull) {
    atomicMin(&st->mid_min, bmin);
    atomicMax(&st->mid_max, bmax);
  }
  u32* hn = a.hist_next + (2 * s) * nb;
  for (int b = threadIdx.x; b < 2 * nb; b += kBlock) {
    const u32 v = nh[b];
    if (v) atomicAdd(&hn[b], v);
  }
}

// Median row of a paired level found: output slot, pivot key, children cells.
template <int NCOL>
__device__ __forceinline__ void pivot_found(const LevelArgs& a, i64 h, i64 lo, i64 n, const float* row, u64 ck) {
  constexpr int D = NCOL - 1;
  const i64 mpos = lo + n / 2;
#pragma unroll
  for (int c = 0; c < D; ++c) a.out_pts[mpos * D + c] = row[c];
  a.out_ids[mpos] = __float_as_uint(row[D]);
  a.state[h].pivot = ck;
  float split = row[0];
#pragma unroll
  for (int c = 1; c < D; ++c) split = c == a.axis ? row[c] : split;
  const float* cell = a.cells + h * 2 * D;
  float* cl_ = a.cells + (2 * h + 1) * 2 * D;
  float* cr_ = a.cells + (2 * h + 2) * 2 * D;
#pragma unroll
  for (int c = 0; c < D; ++c) {
    const float clo = cell[2 * c], chi = cell[2 * c + 1];
    cl_[2 * c] = clo;
    cl_[2 * c + 1] = c == a.axis ? split : chi;
    cr_[2 * c] = c == a.axis ? split : clo;
    cr_[2 * c + 1] = chi;
  }
}

// One wave per segment whose median bucket holds <= 64 rows.
template <int NCOL>
__device__ __forceinline__ void pivot_small_body(LevelArgs a, i64 segs, i64 bid) {
  constexpr int D = NCOL - 1;
  const i64 s = bid * (kBlock / 64) + threadIdx.x / 64;
  if (s >= segs) return;
  const i64 h = a.heap0 + s;
  const i64 n = a.seg_n[h];
  if (n <= 0) return;
  const SegState st = a.state[h];
  if (st.cnt_mid > 64) return;
  const i64 lo = a.seg_lo[h];
  i64 cl = 0, cm = 0;
  zone_counts(st, n, &cl, &cm);
  const int zc = int(cm);
  const int t = int(n / 2 - cl);
  const i64 zlo = lo + cl;
  const i64 nc = a.ncol;
  const int l = dev::lane();
  const bool valid = l < zc;
  float row[NCOL];
#pragma unroll
  for (int c = 0; c < NCOL; ++c) row[c] = valid ? a.dst[i64(c) * nc + zlo + l] : 0.0f;
  float key = row[0], nkey = row[0];
#pragma unroll
  for (int c = 1; c < D; ++c) {
    key = c == a.axis ? row[c] : key;
    nkey = c == a.next_axis ? row[c] : nkey;
  }
  const u64 k = valid ? composite_key(key, __float_as_uint(row[D])) : ~0ull;
  u32 rank = 0;
  for (int j = 0; j < zc; ++j) rank += dev::shfl_u64(k, j) < k ? 1u : 0u;
  if (!valid) return;
  if (int(rank) == t) pivot_found<NCOL>(a, h, lo, n, row, k);
  else if (a.next_bins > 0) add_next_hist(a, s, h, int(rank) < t ? 0 : 1, nkey);
}

// One workgroup per segment with a larger median bucket: radix select (11-bit digits) of
// the rank-t composite key, rows read in place (no staging).
template <int NCOL>
__device__ __forceinline__ void pivot_body(LevelArgs a, i64 bid) {
  constexpr int D = NCOL - 1;
  __shared__ u32 rh[kRadixBins];
  __shared__ u32 sh4[4];
  __shared__ u32 info[3];
  const i64 s = bid;
  const i64 h = a.heap0 + s;
  const i64 n = a.seg_n[h];
  if (n <= 0) return;
  const SegState st = a.state[h];
  if (st.cnt_mid <= 64) return;
  const i64 lo = a.seg_lo[h];
  const i64 nc = a.ncol;
  const float* __restrict__ dst = a.dst;
  i64 cl = 0, zc = 0;
  zone_counts(st, n, &cl, &zc);
  const i64 zlo = lo + cl;
  u64 t = u64(n / 2 - cl);
  auto ckey = [&](i64 p) -> u64 {
    float key = dst[p];
#pragma unroll
    for (int c = 1; c < D; ++c) key = c == a.axis ? dst[i64(c) * nc + p] : key;
    return composite_key(key, reinterpret_cast<const u32*>(dst)[i64(D) * nc + p]);
  };
  const u64 diff = u64(st.mid_min) ^ u64(st.mid_max);
  int hb = diff ? 63 - __builtin_clzll(diff) : -1;
  u64 prefix = hb >= 63 ? 0ull : (u64(st.mid_min) & ~((2ull << hb) - 1ull));
  if (hb < 0) prefix = u64(st.mid_min);
  while (hb >= 0) {
    const int shift = hb >= kRadixBits - 1 ? hb - (kRadixBits - 1) : 0;
    const u64 himask = hb >= 63 ? 0ull : ~((2ull << hb) - 1ull);
    for (int b = threadIdx.x; b < kRadixBins; b += kBlock) rh[b] = 0;
    __syncthreads();
    for (i64 e = threadIdx.x; e < zc; e += kBlock) {
      const u64 key = ckey(zlo + e);
      if ((key & himask) == prefix) atomicAdd(&rh[u32(key >> shift) & (kRadixBins - 1)], 1u);
    }
    __syncthreads();
    const int per = kRadixBins / kBlock;
    u32 sum = 0;
    for (int b = 0; b < per; ++b) sum += rh[threadIdx.x * per + b];
    u32 total;
    const u32 excl = block_excl_scan(sum, sh4, &total);
    if (t >= excl && t < u64(excl) + sum) {
      u32 c = excl;
      for (int b = 0; b < per; ++b) {
        const u32 v = rh[threadIdx.x * per + b];
        if (t < u64(c) + v) {
          info[0] = u32(threadIdx.x * per + b);
          info[1] = c;
          break;
        }
        c += v;
      }
    }
    __syncthreads();
    const u32 digit = info[0];
    t -= info[1];
    const int width = hb - shift + 1;
    prefix |= u64(digit & ((1u << width) - 1u)) << shift;
    hb = shift - 1;
    __syncthreads();
  }
  const u64 pivot = prefix;
  for (i64 e = threadIdx.x; e < zc; e += kBlock) {
    const i64 p = zlo + e;
    float row[NCOL];
#pragma unroll
    for (int c = 0; c < NCOL; ++c) row[c] = dst[i64(c) * nc + p];
    float key = row[0], nkey = row[0];
#pragma unroll
    for (int c = 1; c < D; ++c) {
      key = c == a.axis ? row[c] : key;
      nkey = c == a.next_axis ? row[c] : nkey;
    }
    const u64 k = composite_key(key, __float_as_uint(row[D]));
    if (k == pivot) pivot_found<NCOL>(a, h, lo, n, row, k);
    else if (a.next_bins > 0) add_next_hist(a, s, h, k < pivot ? 0 : 1, nkey);
  }
}

template <int CAP>
__global__ __launch_bounds__(kBlock) void k_refine(LevelArgs a) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  refine_body<CAP>(a, blockIdx.x);
}

// The wave-per-segment and workgroup-per-segment halves of a level's median step take
// disjoint segments (middle zone <= 64 rows or larger), so one launch runs both: blocks
// [0, gs) are the small path, the rest one workgroup per segment. Saves a dispatch (~5 us of
// launch and drain) per level, which adds up over the ~20 levels of a small build.
template <int NCOL, int CAP>
__global__ __launch_bounds__(kBlock) void k_refine_both(LevelArgs a, i64 segs, int gs) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  if (int(blockIdx.x) < gs) refine_small_body<NCOL>(a, segs, blockIdx.x);
  else refine_body<CAP>(a, i64(blockIdx.x) - gs);
}

template <int NCOL>
__global__ __launch_bounds__(kBlock) void k_pivot_both(LevelArgs a, i64 segs, int gs) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  if (int(blockIdx.x) < gs) pivot_small_body<NCOL>(a, segs, blockIdx.x);
  else pivot_body<NCOL>(a, i64(blockIdx.x) - gs);
}

// Second-stage histogram of level l+1 before a pair's scatter: rows are still grouped by
// level-l segment, so each row is routed to its child first (bucket, or pivot comparison for
// level l's median bucket); rows in the child's median bucket add to the child's sub-bucket
// histogram (hist2 of level l+1, [2 * segs][kBins2]).
__global__ __launch_bounds__(kBlock) void k_hist2p(LevelArgs a, PairArgs pa) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  __shared__ u32 sh[2 * kBins2];
  i64 s, bidx;
  int part;
  seg_part(a.bps, a.xcd, s, part, bidx);
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  for (int b = threadIdx.x; b < 2 * kBins2; b += kBlock) sh[b] = 0;
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  const SegState* st = a.state + h;
  const u32 bstar = st->bstar, stage2 = st->stage2, sbstar = st->sbstar;
  const u64 pivot = st->pivot;
  BucketParams p2;
  p2.lo = st->p2lo;
  p2.scale = st->p2scale;
  const BucketParams prm = a.params[h];
  const SegState* c0 = a.state + 2 * h + 1;
  const SegState* c1 = a.state + 2 * h + 2;
  const BucketParams cpr0 = a.params[2 * h + 1], cpr1 = a.params[2 * h + 2];
  const BucketParams q0{c0->p2lo, c0->p2scale}, q1{c1->p2lo, c1->p2scale};
  const u32 cb0 = c0->bstar, cb1 = c1->bstar;
  const i64 nc = a.ncol;
  const float* kc = a.src + i64(a.axis) * nc;
  const float* k1c = a.src + i64(a.next_axis) * nc;
  __shared__ u32 bc[4];
  if (threadIdx.x < 4) bc[threadIdx.x] = 0;
  u32 cnt[4] = {0, 0, 0, 0};  // certain rows: child 0 left / right, child 1 left / right
  __syncthreads();
  sweep_keys<2>(kc, k1c, lo, b0, b1, [&](float k0, float k1, i64 e) {
    const u32 z0 = zone_of(k0, prm, a.bins, bstar, stage2, p2, sbstar);
    u32 c = z0 == 0 ? 0u : 1u;
    if (z0 == 1) {
      const u64 ck = composite_key(k0, src_id(a, lo + e));
      if (ck == pivot) return;
      c = ck < pivot ? 0u : 1u;
    }
    const u32 bk = bucket_of(k1, c == 0 ? cpr0 : cpr1, pa.bins1), cb = c == 0 ? cb0 : cb1;
    if (bk == cb) {
      atomicAdd(&sh[c * kBins2 + bucket_of(k1, c == 0 ? q0 : q1, kBins2)], 1u);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) cnt[k] += u32(k) == 2 * c + (bk > cb ? 1u : 0u) ? 1u : 0u;
    }
  });
  if (pa.bcnt) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32 v = dev::wave_incl_scan(cnt[k]);  // lane 63 holds the wave's total
      if (dev::lane() == 63 && v) atomicAdd(&bc[k], v);
    }
  }
  __syncthreads();
  if (pa.bcnt && threadIdx.x < 4) pa.bcnt[bidx * 4 + threadIdx.x] = bc[threadIdx.x];
  u32* hs = a.hist2 + (2 * s) * kBins2;
  for (int b = threadIdx.x; b < 2 * kBins2; b += kBlock) {
    const u32 v = sh[b];
    if (v) atomicAdd(&hs[b], v);
  }
}

// Per-block write offsets of the certain rows (one workgroup per level-l segment): for each
// (child, left/right zone) an exclusive scan of the blocks' counts from the zone's start;
// the zone cursor then points past all certain rows, where the uncertain rows (the
// child's median bucket, placed by the second stage) are appended with atomics.
__global__ __launch_bounds__(kBlock) void k_block_bases(LevelArgs a, PairArgs pa) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  __shared__ u32 sh4[4];
  const i64 s = blockIdx.x;
  const i64 h = a.heap0 + s;
  if (a.seg_n[h] <= 0) return;
  const u32* cnt = pa.bcnt + s * a.bps * 4;
  u32* base = pa.bbase + s * a.bps * 4;
  // thread t owns blocks [t * per, t * per + per): all loads of a thread are issued together
  const int per = (a.bps + kBlock - 1) / kBlock;
  const int b0 = min(a.bps, int(threadIdx.x) * per), b1 = min(a.bps, b0 + per);
  u32 sum[4] = {0, 0, 0, 0};
  for (int b = b0; b < b1; ++b) {
    const uint4 v = reinterpret_cast<const uint4*>(cnt)[b];
    sum[0] += v.x;
    sum[1] += v.y;
    sum[2] += v.z;
    sum[3] += v.w;
  }
  u32 off[4], start[4], tot[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    start[k] = a.state[2 * h + 1 + k / 2].cur[(k & 1) ? 2 : 0];
    off[k] = start[k] + block_excl_scan(sum[k], sh4, &tot[k]);
    __syncthreads();  // sh4 is reused by the next scan
  }
  for (int b = b0; b < b1; ++b) {
    const uint4 v = reinterpret_cast<const uint4*>(cnt)[b];
    reinterpret_cast<uint4*>(base)[b] = make_uint4(off[0], off[1], off[2], off[3]);
    off[0] += v.x;
    off[1] += v.y;
    off[2] += v.z;
    off[3] += v.w;
  }
  if (threadIdx.x < 4) {
    const int k = int(threadIdx.x);
    a.state[2 * h + 1 + k / 2].cur[(k & 1) ? 2 : 0] = start[k] + tot[k];
  }
}

// Pass B of a pair: a = level l (src -> dst), children states/params are level l+1's.
// PFX: prefix placement (pa.bbase): rows of certain zones are written from per-block
// offsets; rows in a child's median bucket (their zone is decided by the second stage)
// form 6 more pseudo-zones placed with cursor atomics.
template <int NCOL, int KI, bool PFX = false, bool ATOM = false>
__global__ __launch_bounds__(kBlock) void k_partition2(LevelArgs a, PairArgs pa) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int kItems = KI;
  constexpr int kChunk = kBlock * KI;
  constexpr int NZ = PFX ? 12 : 6;
  constexpr int W = kBlock / 64;
  extern __shared__ __align__(16) u32 nh[];  // [4 * bins2]
  __shared__ u32 gcnt[NZ][64];
  // ATOM: zone ranks from one LDS atomic per row on its wave's zone counter (see k_partition3)
  __shared__ u32 wcnt[ATOM ? W : 1][16];
  __shared__ u32 wbase[ATOM ? W : 1][16];
  if (ATOM && threadIdx.x < W * 16) (&wcnt[0][0])[threadIdx.x] = 0;
  __shared__ u32 bcur[6];
  __shared__ unsigned long long bmin[2], bmax[2];  // children's middle-zone key ranges, flushed once
  if (threadIdx.x < 2) {
    bmin[threadIdx.x] = ~0ull;
    bmax[threadIdx.x] = 0ull;
  }
  constexpr int D = NCOL - 1;
  i64 s, bidx;
  int part;
  seg_part(a.bps, a.xcd, s, part, bidx);
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  const int nb2 = pa.bins2;
  const bool fuse = nb2 > 0;
  if (fuse)
    for (int b = threadIdx.x; b < 4 * nb2; b += kBlock) nh[b] = 0;
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  const SegState* st = a.state + h;
  const u32 bstar = st->bstar, stage2 = st->stage2, sbstar = st->sbstar;
  const u64 pivot = st->pivot;
  BucketParams p2;
  p2.lo = st->p2lo;
  p2.scale = st->p2scale;
  const BucketParams prm = a.params[h];
  // children (level l+1, never second-stage: a pair is only formed when l+1 has none);
  // grandchild bucketing in LDS to keep the scalar register file from spilling
  SegState* const cst0 = a.state + 2 * h + 1;
  SegState* const cst1 = a.state + 2 * h + 2;
  __shared__ BucketParams sgp[4];
  if (fuse && threadIdx.x < 4) sgp[threadIdx.x] = a.params[2 * (2 * h + 1 + threadIdx.x / 2) + 1 + (threadIdx.x & 1)];
  __shared__ BucketParams c2p[2];  // children's second-stage bucketing (pa.stage2_1)
  __shared__ u32 c2sb[2];
  if (pa.stage2_1 && threadIdx.x < 2) {
    const SegState* cs = threadIdx.x == 0 ? cst0 : cst1;
    c2p[threadIdx.x] = BucketParams{cs->p2lo, cs->p2scale};
    c2sb[threadIdx.x] = cs->sbstar;
  }
  const u32 cbs0 = cst0->bstar, cbs1 = cst1->bstar;
  const BucketParams cpr0 = a.params[2 * h + 1], cpr1 = a.params[2 * h + 2];
  const i64 clo0 = a.seg_lo[2 * h + 1], clo1 = a.seg_lo[2 * h + 2];
  __syncthreads();  // c2p / c2sb / sgp are read by every wave below
  const float* __restrict__ src = a.src;
  float* __restrict__ dst = a.dst;
  const i64 nc = a.ncol;
  const int axis = a.axis, ax1 = a.next_axis, ax2 = pa.axis2;
  const int w = threadIdx.x / 64;
  const int ln = dev::lane();
  // 3 * child + zone, or 7 (none); unc: the row lies in the child's median bucket
  auto classify = [&](float k0, float k1, u32 id, bool valid, bool& unc) -> u32 {
    unc = false;
    if (!valid) return 7u;
    const u32 z0 = zone_of(k0, prm, a.bins, bstar, stage2, p2, sbstar);
    u32 c = z0 == 0 ? 0u : 1u;
    if (z0 == 1) {
      const u64 ck = composite_key(k0, id);
      if (ck == pivot) return 7u;
      c = ck < pivot ? 0u : 1u;
    }
    const u32 b1 = c == 0 ? bucket_of(k1, cpr0, pa.bins1) : bucket_of(k1, cpr1, pa.bins1);
    const u32 cb = c == 0 ? cbs0 : cbs1;
    u32 z1 = b1 < cb ? 0u : (b1 == cb ? 1u : 2u);
    unc = z1 == 1;
    if (pa.stage2_1 && z1 == 1) {
      const u32 sb = bucket_of(k1, c2p[c], kBins2), sbs = c2sb[c];
      z1 = sb < sbs ? 0u : (sb == sbs ? 1u : 2u);
    }
    return 3 * c + z1;
  };
  if (PFX) {
    if (threadIdx.x < 6) {
      const int t = int(threadIdx.x);
      bcur[t] = (t == 1 || t == 4) ? 0u : pa.bbase[bidx * 4 + (t / 3) * 2 + (t % 3 == 2 ? 1 : 0)];
    }
  } else if (a.block_reserve) {
    u32 cnt[6] = {0, 0, 0, 0, 0, 0};
    const float* kc = src + i64(axis) * nc + lo;
    const float* k1c = src + i64(ax1) * nc + lo;
    constexpr int U = 8;
    for (i64 e0 = b0 + threadIdx.x; e0 < b1; e0 += kBlock * U) {
      float k0[U], k1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const i64 e = e0 + i64(u) * kBlock;
        k0[u] = e < b1 ? kc[e] : 0.0f;
        k1[u] = e < b1 ? k1c[e] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const i64 e = e0 + i64(u) * kBlock;
        if (e >= b1) continue;
        const u32 z0 = zone_of(k0[u], prm, a.bins, bstar, stage2, p2, sbstar);
        bool unc;
        const u32 q = classify(k0[u], k1[u], z0 == 1 ? src_id(a, lo + e) : 0u, true, unc);
#pragma unroll
        for (int z = 0; z < 6; ++z) cnt[z] += q == u32(z) ? 1u : 0u;
      }
    }
#pragma unroll
    for (int z = 0; z < 6; ++z) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cnt[z] += __shfl_xor(cnt[z], o, 64);
      if (ln == 0) gcnt[z][w] = cnt[z];
    }
    __syncthreads();
    if (threadIdx.x < 6) {
      u32 tz = 0;
      for (int k = 0; k < kBlock / 64; ++k) tz += gcnt[threadIdx.x][k];
      const int c = threadIdx.x / 3, z = threadIdx.x % 3;
      bcur[threadIdx.x] = tz ? atomicAdd(&(c == 0 ? cst0 : cst1)->cur[z], tz) : 0u;
    }
  }
  __syncthreads();

  // Each thread loads 4 consecutive rows of a column with one 16-B load (item i = 4 g + j is
  // row 4 (g * kBlock + tid) + j of a chunk that starts on a 16-B aligned absolute row; rows
  // outside [b0, b1) are loaded from the padded buffer and masked)
  static_assert(kItems % 4 == 0, "16-B row loads take 4 rows per item group");
  const i64 cstart = ((lo + b0) & ~i64(3)) - lo;
  for (i64 c0 = cstart; c0 < b1; c0 += kChunk) {
    float row[kItems][NCOL];
    bool vld[kItems];
#pragma unroll
    for (int g = 0; g < kItems / 4; ++g) {
      const i64 e4 = c0 + (i64(g) * kBlock + threadIdx.x) * 4;  // relative row of sub-item 0
      const bool any = e4 < b1;
      const i64 p4 = lo + (any ? e4 : (((lo + b0) & ~i64(3)) - lo));
#pragma unroll
      for (int c = 0; c < NCOL; ++c) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!(c == D && a.id_implicit)) v = *reinterpret_cast<const float4*>(src + i64(c) * nc + p4);
        row[4 * g + 0][c] = v.x;
        row[4 * g + 1][c] = v.y;
        row[4 * g + 2][c] = v.z;
        row[4 * g + 3][c] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const i64 e = e4 + j;
        vld[4 * g + j] = e >= b0 && e < b1;
        if (D >= 0 && a.id_implicit) row[4 * g + j][D] = __uint_as_float(a.id_base0 + u32(lo + e));
      }
    }
    u32 zone_pre[kItems];  // (zone index << 16) | rank-in-wave; index q, or 6 + q (PFX uncertain), 15 none
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      float k0 = row[i][0], k1 = row[i][0], k2 = row[i][0];
#pragma unroll
      for (int c = 1; c < D; ++c) {
        k0 = c == axis ? row[i][c] : k0;
        k1 = c == ax1 ? row[i][c] : k1;
        k2 = c == ax2 ? row[i][c] : k2;
      }
      bool unc;
      const u32 q = classify(k0, k1, __float_as_uint(row[i][D]), vld[i], unc);
      const u32 zi = q >= 6 ? 15u : (PFX && unc ? q + 6 : q);
      if constexpr (ATOM) {
        zone_pre[i] = (zi << 16) | atomicAdd(&wcnt[w][zi], 1u);
      } else {
        zone_pre[i] = (zi << 16) | dev::wave_zone_rank<NZ>(zi, &gcnt[0][i * 4 + w], 64);
      }
      if (fuse && q < 6 && q != 1 && q != 4) {
        const u32 g = (q / 3) * 2 + (q % 3 == 2 ? 1u : 0u);
        atomicAdd(&nh[g * nb2 + bucket_of(k2, sgp[g], nb2)], 1u);
      }
      if (__ballot(q == 1 || q == 4)) {  // level l+1 middle zones: track their composite key ranges
        const u64 ck = composite_key(k1, __float_as_uint(row[i][D]));
        wave_minmax_atomic(q == 1, ck, &bmin[0], &bmax[0]);
        wave_minmax_atomic(q == 4, ck, &bmin[1], &bmax[1]);
      }
    }
    __syncthreads();
    if constexpr (ATOM) {
      if (threadIdx.x < NZ) {  // thread z: zone z's waves, scanned and reserved at once
        const int z = int(threadIdx.x);
        u32 c[W], tot = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          c[k] = wcnt[k][z];
          tot += c[k];
        }
        u32 base = 0;
        if (PFX && z >= 6) {
          base = tot ? atomicAdd(&(z < 9 ? cst0 : cst1)->cur[(z - 6) % 3], tot) : 0u;
        } else if (PFX || a.block_reserve) {
          base = bcur[z];
          bcur[z] = base + tot;
        } else {
          base = tot ? atomicAdd(&(z < 3 ? cst0 : cst1)->cur[z % 3], tot) : 0u;
        }
#pragma unroll
        for (int k = 0; k < W; ++k) {
          wbase[k][z] = base;
          base += c[k];
          wcnt[k][z] = 0;
        }
      }
      if (threadIdx.x >= NZ && threadIdx.x < NZ + W) wcnt[threadIdx.x - NZ][15] = 0;
    } else
    for (int z = w; z < NZ; z += kBlock / 64) {  // wave w scans zones w, w+4 (, w+8)
      const u32 v = ln < kItems * 4 ? gcnt[z][ln] : 0u;
      const u32 incl = dev::wave_incl_scan(v);
      const u32 tot = __shfl(incl, 63, 64);
      u32 base = 0;
      if (PFX && z >= 6) {
        if (ln == 0 && tot) base = atomicAdd(&(z < 9 ? cst0 : cst1)->cur[(z - 6) % 3], tot);
        base = __shfl(base, 0, 64);
      } else if (PFX || a.block_reserve) {
        base = bcur[z];
        if (ln == 0) bcur[z] = base + tot;
      } else {
        if (ln == 0 && tot) base = atomicAdd(&(z < 3 ? cst0 : cst1)->cur[z % 3], tot);
        base = __shfl(base, 0, 64);
      }
      gcnt[z][ln] = base + incl - v;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      const u32 zi = zone_pre[i] >> 16;
      i64 dest = -1;
      if (zi < u32(NZ)) {
        const u32 c = (zi % 6) / 3;
        const u32 off = (ATOM ? wbase[w][zi] : gcnt[zi][i * 4 + w]) + (zone_pre[i] & 0xffffu);
        const i64 cn = c == 0 ? n / 2 : n - n / 2 - 1;
        if (i64(off) >= cn) {
          atomicOr(a.err, 1u);
        } else {
          dest = (c == 0 ? clo0 : clo1) + off;
        }
      }
#pragma unroll
      for (int c = 0; c < NCOL; ++c)
        if (dest >= 0) dst[i64(c) * nc + dest] = row[i][c];
    }
    __syncthreads();
  }
  if (threadIdx.x < 2 && bmin[threadIdx.x] != ~0ull) {
    SegState* cs = threadIdx.x == 0 ? cst0 : cst1;
    atomicMin(&cs->mid_min, bmin[threadIdx.x]);
    atomicMax(&cs->mid_max, bmax[threadIdx.x]);
  }
  if (fuse) {
    u32* hn = pa.hist2n + (4 * s) * nb2;
    for (int b = threadIdx.x; b < 4 * nb2; b += kBlock) {
      const u32 v = nh[b];
      if (v) atomicAdd(&hn[b], v);
    }
  }
}

// =====================================================================================
// Triple global levels: levels l, l+1 and l+2 are moved by ONE scatter pass.
//   k_scan       as for a pair: level l's median bucket staged, level l+1's histograms;
//   k_pivot*     level l's exact pivot;  k_select  level l+1;
//   k_scan2      keys of l, l+1, l+2 (12 B / row): every row is routed to its child by level
//                l's exact pivot; rows of the child's median bucket of level l+1 are staged in
//                the child's middle-zone area of dst (scratch), every other row adds its
//                level-(l+2) key to its grandchild's histogram (fused, LDS);
//   k_pivot*     level l+1's exact pivots (the staged rows; their level-(l+2) keys complete the
//                grandchildren's histograms);  k_select  level l+2;
//   k_partition3 one read + one write of every row: grandchild (exact pivots of l and l+1) and
//                zone inside it (level l+2's median bucket) give 12 destination zones; the
//                level-(l+3) histograms of the 8 great-grandchildren are fused in;
//   k_refine*    level l+2's middle zones.
// Traffic per three levels: 8 + 12 + 32 B / row instead of 1.5 pairs' 60 B.
struct TripleArgs {
  int bins1;    // level l+1 bins
  int axis2;    // level l+2 axis
  int bins2;    // level l+2 bins
  u32* hist2;   // level l+2 histograms [4 * segs][bins2] (k_scan2)
  int axis3;    // level l+3 axis
  int bins3;    // level l+3 bins (0: l+3 is the subtree level)
  u32* hist3;   // level l+3 histograms [8 * segs][bins3] (k_partition3)
};

template <int NCOL>
__global__ __launch_bounds__(kBlock) void k_scan2(LevelArgs a, TripleArgs ta) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  extern __shared__ __align__(16) u32 nh[];  // [4 * bins2] + 64 per-lane dummy words
  constexpr int D = NCOL - 1;
  const i64 s = blockIdx.x / a.bps;
  const int part = blockIdx.x % a.bps;
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  const int nb = ta.bins2;
  for (int b = threadIdx.x; b < 4 * nb + 64; b += kBlock) nh[b] = 0;
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  const SegState* st = a.state + h;
  const u32 bstar = st->bstar, stage2 = st->stage2, sbstar = st->sbstar;
  const u64 pivot = st->pivot;
  BucketParams p2;
  p2.lo = st->p2lo;
  p2.scale = st->p2scale;
  const BucketParams prm = a.params[h];
  SegState* const cst0 = a.state + 2 * h + 1;
  SegState* const cst1 = a.state + 2 * h + 2;
  const BucketParams cp0 = a.params[2 * h + 1], cp1 = a.params[2 * h + 2];
  const u32 cb0 = cst0->bstar, cb1 = cst1->bstar;
  const i64 clo0 = a.seg_lo[2 * h + 1], clo1 = a.seg_lo[2 * h + 2];
  const i64 cn0 = a.seg_n[2 * h + 1], cn1 = a.seg_n[2 * h + 2];
  __shared__ BucketParams gp[4];  // grandchildren's level-(l+2) bucketing
  constexpr int kStage = 512;
  __shared__ u32 sidx[2][kStage];
  __shared__ u32 mcnt[2], mbase[2];
  __shared__ unsigned long long bmin[2], bmax[2];
  if (threadIdx.x < 4) gp[threadIdx.x] = a.params[2 * (2 * h + 1 + threadIdx.x / 2) + 1 + (threadIdx.x & 1)];
  if (threadIdx.x < 2) {
    mcnt[threadIdx.x] = 0;
    bmin[threadIdx.x] = ~0ull;
    bmax[threadIdx.x] = 0ull;
  }
  __syncthreads();
  const float* __restrict__ src = a.src;
  float* __restrict__ dst = a.dst;
  const i64 nc = a.ncol;
  const int ln = dev::lane();
  const u32 hdummy = u32(4 * nb) + u32(ln);
  // One row (all lanes of a wave together: ballots): child by level l's exact pivot; the
  // child's median bucket of level l+1 -> staged, else the grandchild's level-(l+2) histogram.
  auto visit = [&](float k0, float k1, float k2, i64 e, bool valid) {
    const u32 z = valid ? zone_of(k0, prm, a.bins, bstar, stage2, p2, sbstar) : 3u;
    bool live = valid;
    u32 c = z == 0 ? 0u : 1u;
    if (z == 1) {
      const u64 ck = composite_key(k0, src_id(a, lo + e));
      live = ck != pivot;  // level l's median: already written out
      c = ck < pivot ? 0u : 1u;
    }
    const u32 b1 = bucket_of(k1, c == 0 ? cp0 : cp1, ta.bins1), cb = c == 0 ? cb0 : cb1;
    const bool mid = live && b1 == cb;
    const u32 g = 2 * c + (b1 > cb ? 1u : 0u);
    atomicAdd(&nh[(live && !mid) ? g * u32(nb) + bucket_of(k2, gp[g], nb) : hdummy], 1u);
    if (__ballot(mid)) {  // rare: note the child's median-bucket rows (per child list)
#pragma unroll
      for (u32 cc = 0; cc < 2; ++cc) {
        const bool me = mid && c == cc;
        const u64 m = __ballot(me);
        if (!m) continue;
        const int leader = __ffsll((long long)m) - 1;
        u32 base = 0;
        if (ln == leader) base = atomicAdd(&mcnt[cc], u32(__popcll(m)));
        base = __shfl(base, leader, 64);
        const u32 slot = base + mbcnt(m);
        const bool direct = me && slot >= u32(kStage);
        if (me && !direct) sidx[cc][slot] = u32(e - b0);
        if (__ballot(direct)) {  // staging list full: reserve and copy directly
          u64 ck = 0;
          if (direct) {
            const u32 q = atomicAdd(&(cc == 0 ? cst0 : cst1)->cur[1], 1u);
            if (i64(q) >= (cc == 0 ? cn0 : cn1)) {
              atomicOr(a.err, 1u);
            } else {
#pragma unroll
              for (int col = 0; col < NCOL; ++col) dst[i64(col) * nc + (cc == 0 ? clo0 : clo1) + q] = src_col(a, col, lo + e);
            }
            ck = composite_key(k1, src_id(a, lo + e));
          }
          wave_minmax_atomic(direct, ck, &bmin[cc], &bmax[cc]);
        }
      }
    }
  };
  const i64 abs0 = lo + b0, abs1 = lo + b1;
  const i64 A = min(abs1, (abs0 + 3) & ~i64(3));
  const i64 nv = (abs1 - A) >> 2;
  const i64 Bend = A + 4 * nv;
  const float* kc = src + i64(a.axis) * nc;
  const float* k1c = src + i64(a.next_axis) * nc;
  const float* k2c = src + i64(ta.axis2) * nc;
  {
    const int t = int(threadIdx.x);
    const bool head = t < 3 && abs0 + t < A, tail = t >= 3 && t < 6 && Bend + (t - 3) < abs1;
    const i64 p = head ? abs0 + t : (tail ? Bend + (t - 3) : lo);
    const bool v = head | tail;
    visit(v ? kc[p] : 0.0f, v ? k1c[p] : 0.0f, v ? k2c[p] : 0.0f, p - lo, v);
  }
  const float4* k04 = reinterpret_cast<const float4*>(kc + A);
  const float4* k14 = reinterpret_cast<const float4*>(k1c + A);
  const float4* k24 = reinterpret_cast<const float4*>(k2c + A);
  constexpr int U4 = 2;
  for (i64 v0 = 0; v0 < nv; v0 += kBlock * U4) {
    float4 x0[U4], x1[U4], x2[U4];
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      const i64 v = v0 + i64(u) * kBlock + threadIdx.x;
      const i64 vi = v < nv ? v : 0;
      x0[u] = k04[vi];
      x1[u] = k14[vi];
      x2[u] = k24[vi];
    }
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      const i64 v = v0 + i64(u) * kBlock + threadIdx.x;
      const bool in = v < nv;
      const i64 e = A - lo + 4 * v;
      visit(x0[u].x, x1[u].x, x2[u].x, e, in);
      visit(x0[u].y, x1[u].y, x2[u].y, e + 1, in);
      visit(x0[u].z, x1[u].z, x2[u].z, e + 2, in);
      visit(x0[u].w, x1[u].w, x2[u].w, e + 3, in);
    }
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const u32 staged = min(mcnt[threadIdx.x], u32(kStage));
    mbase[threadIdx.x] = staged ? atomicAdd(&(threadIdx.x == 0 ? cst0 : cst1)->cur[1], staged) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (u32 cc = 0; cc < 2; ++cc) {
    const u32 staged = min(mcnt[cc], u32(kStage));
    const i64 clo = cc == 0 ? clo0 : clo1, cn = cc == 0 ? cn0 : cn1;
    for (u32 r0 = 0; r0 < staged; r0 += kBlock) {  // uniform trip count: every lane reaches the wave ops
      const u32 k2 = r0 + threadIdx.x;
      const bool act = k2 < staged;
      const i64 q = i64(mbase[cc]) + k2;
      u64 ck = 0;
      if (act) {
        const i64 e = b0 + sidx[cc][k2];
        float row[NCOL];
#pragma unroll
        for (int col = 0; col < NCOL; ++col) row[col] = src_col(a, col, lo + e);
        if (q >= cn) {
          atomicOr(a.err, 1u);
        } else {
#pragma unroll
          for (int col = 0; col < NCOL; ++col) dst[i64(col) * nc + clo + q] = row[col];
        }
        float key = row[0];
#pragma unroll
        for (int col = 1; col < D; ++col) key = col == a.next_axis ? row[col] : key;
        ck = composite_key(key, __float_as_uint(row[D]));
      }
      wave_minmax_atomic(act, ck, &bmin[cc], &bmax[cc]);
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 && bmin[threadIdx.x] != ~0ull) {
    SegState* cs = threadIdx.x == 0 ? cst0 : cst1;
    atomicMin(&cs->mid_min, bmin[threadIdx.x]);
    atomicMax(&cs->mid_max, bmax[threadIdx.x]);
  }
  u32* hn = ta.hist2 + (4 * s) * nb;
  for (int b = threadIdx.x; b < 4 * nb; b += kBlock) {
    const u32 v = nh[b];
    if (v) atomicAdd(&hn[b], v);
  }
}

// Pass of a triple: a = level l (src -> dst); grandchildren (heap 4h + 3 + g) receive the rows.
template <int NCOL, int KI, bool ATOM = true, int NH = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(NH > 0 ? 4 : 1))) void k_partition3(LevelArgs a, TripleArgs ta) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int kItems = KI;
  constexpr int kChunk = kBlock * KI;
  constexpr int NZ = 12;  // 4 grandchildren x (left of / inside / right of the level-(l+2) median bucket)
  constexpr int D = NCOL - 1;
  static_assert(kItems % 4 == 0, "16-B row loads take 4 rows per item group");
  constexpr int W = kBlock / 64;
  constexpr bool STG = !ATOM && NH > 0;  // stores through an LDS tile in zone order (as k_g3_part)
  constexpr int NP = STG ? NH : 1;
  constexpr int HI = KI / NP;
  constexpr int HROWS = kBlock * HI;
  static_assert(KI % NP == 0, "whole items per part");
  constexpr int PK = STG ? 2 : 1;  // counts per histogram word (STG: 16-bit, blocks of < 64 Ki rows)
  extern __shared__ __align__(16) u32 nh[];  // [8 * bins3], then (STG) the tile
  __shared__ u32 zb_s[16], ztot_s[16], zpst[NP][16], zls[16];
  // Zone ranks: every row takes its rank inside (wave, zone) from one LDS atomic on the wave's
  // counter of its zone (16 counters per wave, the last one for rows that stay behind); after
  // a barrier the waves' counts are scanned per zone and reserved in the grandchild's zone.
  // One atomic per row instead of 12 ballots and 12 count stores per row.
  __shared__ u32 wcnt[W][16];
  __shared__ u32 wbase[W][16];
  __shared__ u32 gcnt[ATOM ? 1 : NZ][64];
  __shared__ unsigned long long bmin[4], bmax[4];  // grandchildren's middle-zone key ranges, flushed once
  __shared__ BucketParams gpar[4], ggp[8];
  __shared__ u32 gbs[4];
  __shared__ i64 glo[4], gn[4];
  i64 s, bidx;
  int part;
  seg_part(a.bps, a.xcd, s, part, bidx);
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  const int nb3 = ta.bins3;
  const bool fuse = nb3 > 0;
  if (fuse)
    for (int b = threadIdx.x; b < (8 * nb3 + PK - 1) / PK; b += kBlock) nh[b] = 0;
  const i64 g0 = 4 * h + 3;  // heap index of the first grandchild
  if (threadIdx.x < W * 16) (&wcnt[0][0])[threadIdx.x] = 0;
  if (threadIdx.x < 4) {
    const int t = int(threadIdx.x);
    bmin[t] = ~0ull;
    bmax[t] = 0ull;
    gpar[t] = a.params[g0 + t];
    gbs[t] = a.state[g0 + t].bstar;
    glo[t] = a.seg_lo[g0 + t];
    gn[t] = a.seg_n[g0 + t];
  }
  if (fuse && threadIdx.x < 8) ggp[threadIdx.x] = a.params[2 * g0 + 1 + threadIdx.x];
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  const SegState* st = a.state + h;
  const u32 bstar = st->bstar, stage2 = st->stage2, sbstar = st->sbstar;
  const u64 pivot = st->pivot;
  BucketParams p2;
  p2.lo = st->p2lo;
  p2.scale = st->p2scale;
  const BucketParams prm = a.params[h];
  const SegState* const cst0 = a.state + 2 * h + 1;
  const SegState* const cst1 = a.state + 2 * h + 2;
  const u32 cbs0 = cst0->bstar, cbs1 = cst1->bstar;
  const u64 cpv0 = cst0->pivot, cpv1 = cst1->pivot;
  const BucketParams cpr0 = a.params[2 * h + 1], cpr1 = a.params[2 * h + 2];
  __syncthreads();
  const float* __restrict__ src = a.src;
  float* __restrict__ dst = a.dst;
  const i64 nc = a.ncol;
  const int axis = a.axis, ax1 = a.next_axis, ax2 = ta.axis2, ax3 = ta.axis3;
  const int w = threadIdx.x / 64;
  const int ln = dev::lane();
  // 3 * grandchild + zone, or 15 (absent row, or the median of level l or l+1)
  auto classify = [&](float k0, float k1, float k2, u32 id, bool valid) -> u32 {
    if (!valid) return 15u;
    const u32 z0 = zone_of(k0, prm, a.bins, bstar, stage2, p2, sbstar);
    u32 c = z0 == 0 ? 0u : 1u;
    if (z0 == 1) {
      const u64 ck = composite_key(k0, id);
      if (ck == pivot) return 15u;
      c = ck < pivot ? 0u : 1u;
    }
    const u32 b1 = bucket_of(k1, c == 0 ? cpr0 : cpr1, ta.bins1);
    const u32 cb = c == 0 ? cbs0 : cbs1;
    u32 g = b1 < cb ? 0u : 1u;
    if (b1 == cb) {
      const u64 ck = composite_key(k1, id);
      const u64 cp = c == 0 ? cpv0 : cpv1;
      if (ck == cp) return 15u;
      g = ck < cp ? 0u : 1u;
    }
    const u32 gi = 2 * c + g;
    const u32 b2 = bucket_of(k2, gpar[gi], ta.bins2), gb = gbs[gi];
    return 3 * gi + (b2 < gb ? 0u : (b2 == gb ? 1u : 2u));
  };
  const i64 cstart = ((lo + b0) & ~i64(3)) - lo;
  for (i64 c0 = cstart; c0 < b1; c0 += kChunk) {
    float row[kItems][NCOL];
    bool vld[kItems];
#pragma unroll
    for (int g = 0; g < kItems / 4; ++g) {
      const i64 e4 = c0 + (i64(g) * kBlock + threadIdx.x) * 4;  // relative row of sub-item 0
      const bool any = e4 < b1;
      const i64 p4 = lo + (any ? e4 : cstart);
#pragma unroll
      for (int c = 0; c < NCOL; ++c) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!(c == D && a.id_implicit)) v = *reinterpret_cast<const float4*>(src + i64(c) * nc + p4);
        row[4 * g + 0][c] = v.x;
        row[4 * g + 1][c] = v.y;
        row[4 * g + 2][c] = v.z;
        row[4 * g + 3][c] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const i64 e = e4 + j;
        vld[4 * g + j] = e >= b0 && e < b1;
        if (a.id_implicit) row[4 * g + j][D] = __uint_as_float(a.id_base0 + u32(lo + e));
      }
    }
    u32 zone_pre[kItems];  // (zone << 16) | rank among the wave's rows of that zone in this chunk
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      float k0 = row[i][0], k1 = row[i][0], k2 = row[i][0], k3 = row[i][0];
#pragma unroll
      for (int c = 1; c < D; ++c) {
        k0 = c == axis ? row[i][c] : k0;
        k1 = c == ax1 ? row[i][c] : k1;
        k2 = c == ax2 ? row[i][c] : k2;
        k3 = c == ax3 ? row[i][c] : k3;
      }
      const u32 id = __float_as_uint(row[i][D]);
      const u32 q = classify(k0, k1, k2, id, vld[i]);
      if constexpr (ATOM) {
        zone_pre[i] = (q << 16) | atomicAdd(&wcnt[w][q], 1u);
      } else {
        zone_pre[i] = (q << 16) | dev::wave_zone_rank<NZ>(q, &gcnt[0][i * 4 + w], 64);
      }
      const u32 zz = q % 3;
      if (fuse && q < u32(NZ) && zz != 1) {
        const u32 gg = 2 * (q / 3) + (zz == 2 ? 1u : 0u);
        const u32 hb = gg * u32(nb3) + bucket_of(k3, ggp[gg], nb3);
        atomicAdd(&nh[hb / PK], STG ? 1u << ((hb & 1u) * 16) : 1u);
      }
      if (__ballot(q < u32(NZ) && zz == 1)) {  // level l+2 middle zones: track their composite key ranges
        const u64 ck = composite_key(k2, id);
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) wave_minmax_atomic(q == u32(3 * gi + 1), ck, &bmin[gi], &bmax[gi]);
      }
    }
    __syncthreads();
    if constexpr (!ATOM) {
      // wave w scans zones w, w+4, w+8; lane k reserves the wave's k-th zone (all in flight at once)
      constexpr int ZW = (NZ + W - 1) / W;
      u32 v[ZW], incl[ZW], tot[ZW];
#pragma unroll
      for (int k = 0; k < ZW; ++k) {
        const int z = w + k * W;
        v[k] = (z < NZ && ln < kItems * 4) ? gcnt[z < NZ ? z : 0][ln] : 0u;
        incl[k] = dev::wave_incl_scan(v[k]);
        tot[k] = __shfl(incl[k], 63, 64);
      }
      u32 mine = 0;
#pragma unroll
      for (int k = 0; k < ZW; ++k) mine = ln == k ? tot[k] : mine;
      const int zl = w + ln * W;
      u32 base = 0;
      if (ln < ZW && zl < NZ && mine) base = atomicAdd(&a.state[g0 + zl / 3].cur[zl % 3], mine);
#pragma unroll
      for (int k = 0; k < ZW; ++k) {
        const int z = w + k * W;
        const u32 b = __shfl(base, k, 64);
        if (z < NZ) gcnt[z][ln] = (STG ? 0u : b) + incl[k] - v[k];  // STG: offset inside the chunk's zone run
        if constexpr (STG) {
          u32 ps[NP];
#pragma unroll
          for (int hp = 0; hp < NP; ++hp) ps[hp] = hp == 0 ? 0u : u32(__shfl(int(incl[k]), hp * HI * W - 1, 64));
          if (z < NZ && ln == 0) {
            zb_s[z] = b;
            ztot_s[z] = tot[k];
#pragma unroll
            for (int hp = 0; hp < NP; ++hp) zpst[hp][z] = ps[hp];
          }
        }
      }
    } else if (threadIdx.x < NZ) {  // thread z: zone z's waves, scanned, reserved in the grandchild at once
      const int z = int(threadIdx.x);
      u32 c[W], tot = 0;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        c[k] = wcnt[k][z];
        tot += c[k];
      }
      u32 base = tot ? atomicAdd(&a.state[g0 + z / 3].cur[z % 3], tot) : 0u;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        wbase[k][z] = base;
        base += c[k];
        wcnt[k][z] = 0;  // the next chunk's counters (read by no one else before the barrier)
      }
    }
    if (ATOM && threadIdx.x >= NZ && threadIdx.x < NZ + W) wcnt[threadIdx.x - NZ][15] = 0;
    __syncthreads();
    if constexpr (STG) {
      float* tile = reinterpret_cast<float*>(nh + ((max(1, (8 * nb3 + 1) / 2) + 3) & ~3));
      unsigned char* tz = reinterpret_cast<unsigned char*>(tile + NCOL * HROWS);
#pragma unroll
      for (int hp = 0; hp < NP; ++hp) {
        const u32 ch = ln < NZ ? (hp + 1 < NP ? zpst[hp + 1 < NP ? hp + 1 : 0][ln] : ztot_s[ln]) - zpst[hp][ln] : 0u;
        const u32 inc = dev::wave_incl_scan(ch);
        const u32 ex = inc - ch;
        if (w == 0 && ln < NZ) zls[ln] = ex;
        if (w == 0 && ln == NZ - 1) zls[NZ] = inc;
#pragma unroll
        for (int ii = 0; ii < HI; ++ii) {
          const int i = hp * HI + ii;
          const u32 zi = zone_pre[i] >> 16;
          const u32 zs = zi < u32(NZ) ? zi : 0u;
          const u32 exz = u32(__shfl(int(ex), int(zs), 64));
          if (zi >= u32(NZ)) continue;
          const u32 p = exz + gcnt[zs][i * 4 + w] - zpst[hp][zs] + (zone_pre[i] & 0xffffu);
#pragma unroll
          for (int c = 0; c < NCOL; ++c) tile[c * HROWS + p] = row[i][c];
          tz[p] = (unsigned char)zi;
        }
        __syncthreads();
        const u32 T = zls[NZ];
        for (u32 j = threadIdx.x; j < T; j += kBlock) {
          const u32 zi = tz[j], gi = zi / 3;
          const u32 off = zb_s[zi] + zpst[hp][zi] + (j - zls[zi]);
          if (i64(off) >= gn[gi]) {
            atomicOr(a.err, 1u);
            continue;
          }
          const i64 dest = glo[gi] + off;
#pragma unroll
          for (int c = 0; c < NCOL; ++c) dst[i64(c) * nc + dest] = tile[c * HROWS + j];
        }
        __syncthreads();  // the tile, zls and (last part) gcnt are rewritten next
      }
    } else {
#pragma unroll
      for (int i = 0; i < kItems; ++i) {
        const u32 zi = zone_pre[i] >> 16;
        i64 dest = -1;
        if (zi < u32(NZ)) {
          const u32 gi = zi / 3;
          const u32 off = (ATOM ? wbase[w][zi] : gcnt[ATOM ? 0 : zi][i * 4 + w]) + (zone_pre[i] & 0xffffu);
          if (i64(off) >= gn[gi]) {
            atomicOr(a.err, 1u);
          } else {
            dest = glo[gi] + off;
          }
        }
#pragma unroll
        for (int c = 0; c < NCOL; ++c)
          if (dest >= 0) dst[i64(c) * nc + dest] = row[i][c];
      }
      // ATOM: the next chunk's atomics only touch the zeroed counters and its reads of wbase
      // follow two more barriers; ballots: the next chunk rewrites gcnt
      if (!ATOM) __syncthreads();
    }
  }
  __syncthreads();
  if (threadIdx.x < 4 && bmin[threadIdx.x] != ~0ull) {
    SegState* gs = a.state + g0 + threadIdx.x;
    atomicMin(&gs->mid_min, bmin[threadIdx.x]);
    atomicMax(&gs->mid_max, bmax[threadIdx.x]);
  }
  if (fuse) {
    u32* hn = ta.hist3 + (8 * s) * nb3;
    for (int b = threadIdx.x; b < 8 * nb3; b += kBlock) {
      const u32 v = STG ? (nh[b >> 1] >> ((b & 1) * 16)) & 0xffffu : nh[b];
      if (v) atomicAdd(&hn[b], v);
    }
  }
}

// =====================================================================================
// Sampled triples (G3). A triple (levels l, l+1, l+2 in one row-moving pass) otherwise needs the
// exact pivots of l and l+1 BEFORE its scatter: two key sweeps over every row (k_scan 8 B,
// k_scan2 12 B) and six small launches. Here those pivots are estimated from a sample first and
// made exact afterwards over the few rows the estimate could not place (SURVEY.md §5.8's
// "sample -> splitters -> exact fix-up", as the sampled top levels do for levels 0..3):
//   k_g3_sample<1>  (segments x blocks) stratified sample of each segment (one 64-row run per
//                   window): histograms of the children's keys on axis l+1 (the child from level
//                   l's exact median bucket b*; inside b*, against the bucket's middle);
//   k_g3_band<1>    per segment: each child's band [a, b] on axis l+1 holding its median with z
//                   standard deviations of the sample rank to spare, and its estimated pivot;
//   k_g3_sample<2>  the grandchildren's keys on axis l+2 (grandchild by the estimated pivot);
//   k_g3_band<2>    their bands; the segment's staging regions (one per tag, sized from the
//                   sample's band counts), the great-grandchildren's histogram bucketing;
//   k_g3_part       every row ONCE: certain at all three levels (outside b*, outside its child's
//                   band, outside its grandchild's band) -> straight into its great-grandchild
//                   (8 zones, fused level-(l+3) histogram); otherwise into the staging region of
//                   the level that could not place it (tag 0: b*, 1 + c: child band, 3 + g:
//                   grandchild band);
//   k_g3_res<0>     per segment: level l's median among the b* rows (b* holds rank n/2), written
//                   out; the b* rows routed on (appended to a child / grandchild band region, or
//                   inserted after their great-grandchild's certain rows);
//   k_g3_res<1>     per child: its median's rank inside its band (exact counts of the rows left
//                   of the band), found by a band histogram and a select over the median's bin,
//                   written out; the band rows routed on;
//   k_g3_res<2>     per grandchild: the same; every row is now in its great-grandchild.
// Traffic per three levels: 16 + 16 B per row plus the sample and the staged rows, instead of
// 8 + 12 + 16 + 16 B. A band that misses its median, or a region that overflows, marks the
// segment bad and sets the sampled-levels error bit (top4_band_miss_bit()): the caller rebuilds
// unsampled. A bad segment still leaves level l+3 consistent (its histograms are recounted from
// the slots), so the remaining levels run to completion without faults. Replaces
// build_tree_rec's std::sort of three levels (kdtree_sequential.cpp:30-66).
constexpr int kG3Bins = 1024;      // sample histogram bins per node
constexpr int kG3ResBins = 2048;   // band-row histogram bins of a resolve workgroup
constexpr int kG3Cand = 2048;      // candidates of a median's bin selected in LDS
constexpr int kG3Run = 64;         // sample rows per window (one wave's coalesced run)
constexpr int kG3SampU = 4;        // windows per wave per sample iteration (loads in flight)
constexpr int kG3Threads = 512;    // resolve workgroups
constexpr int kG3Gg = 8;           // great-grandchildren of a segment

struct G3Seg {
  u32 a1[2], b1[2];  // children's bands on axis l+1 (orderable keys, inclusive)
  u32 a2[4], b2[4];  // grandchildren's bands on axis l+2
  u32 p1[2];         // children's estimated pivots (orderable; the second sample pass routes by them)
  u32 tot[2];        // samples per child
  u32 bsamp[6];      // samples inside each band (children, grandchildren)
  u32 off[8];        // staging region of tag t: stage rows [lo + off[t], lo + off[t] + cap[t])
  u32 cap[8];
  u32 ins[8];        // staged rows inserted per great-grandchild (after its certain rows)
  u32 bad;           // a band missed or a region overflowed: the segment's subtree is invalid
  u32 pad[7];
  // the pass's zone cursors, one 64-B line each (every block of the segment reserves on them once
  // per chunk): zc[gg][0] certain rows placed per great-grandchild (its first slots), zc[8 + t][0]
  // rows staged per tag t (may exceed cap: overflow)
  u32 zc[16][16];
};

struct G3Args {
  G3Seg* g3;       // per level-l segment (level-relative index)
  u32* shist;      // sample histograms [segment][6][kG3Bins] (level-relative)
  float* stage;    // staging columns (NCOL, stride ncol); a segment's regions lie in its [lo, lo + n)
  i64 seg0;        // level-relative index of the launch's first segment
  int axis2, axis3;
  int bins3;       // level l+3 bins (0: l+3 is not a histogrammed global level)
  u32* hist3;      // level l+3 histograms [8 * segs][bins3] (launch-relative)
  int sample_div;  // one run of kG3Run rows per window of kG3Run * sample_div rows
  int sblocks;     // sample blocks per segment
  float z;         // band half-width in standard deviations of the sample rank
  u32 salt;        // per build: the sample positions (so a miss) are never fixed by the input
  // multi-block resolve (k_g3_m*): per-node state, band histograms, median-bin candidates
  struct G3Node* nodes;     // [segment][6]
  u32* mhist;               // [segment][6][kG3ResBins]
  u64* cand;                // [segment][6][kG3MCand]
};

__device__ __forceinline__ u32 g3_mix(u32 x) {  // murmur3 finaliser
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ void g3_bad(u32* err, G3Seg* gs) {
  atomicOr(&gs->bad, 1u);
  atomicOr(err, top4::kErrBit);
}

// Edges of level l's median bucket b* on its axis (the cell's range when the bucketing is flat).
__device__ __forceinline__ void g3_bstar_edges(const LevelArgs& a, i64 h, float* e_lo, float* e_hi) {
  const BucketParams prm = a.params[h];
  const u32 bstar = a.state[h].bstar;
  const float* cell = a.cells + h * 2 * a.dim;
  *e_lo = cell[2 * a.axis];
  *e_hi = cell[2 * a.axis + 1];
  if (prm.scale > 0.0f) {
    *e_lo = prm.lo + float(bstar) / prm.scale;
    *e_hi = prm.lo + float(bstar + 1) / prm.scale;
  }
}

__device__ __forceinline__ float g3_lo_of(u32 A) { return A ? from_orderable(A) : -INFINITY; }
__device__ __forceinline__ float g3_hi_of(u32 B) { return B != 0xffffffffu ? from_orderable(B) : INFINITY; }

// Range on axis `ax` of descendant (depth, idx) of a segment (depth 1: child idx; 2: grandchild;
// 3: great-grandchild), from the segment's cell narrowed by b*'s edges and the bands that are
// known (pass the band arrays, or nullptr for the ones not known yet). Any monotone bucketing is
// correct: this only sets a histogram's resolution.
__device__ __forceinline__ void g3_range(const float* cell, int ax, int axis, int ax1, int ax2, float e_lo,
                                         float e_hi, int depth, int idx, const u32* a1, const u32* b1,
                                         const u32* a2, const u32* b2, float* lo_out, float* hi_out) {
  float lo = cell[2 * ax], hi = cell[2 * ax + 1];
  const int s0 = idx >> (depth - 1);
  if (ax == axis) {
    if (s0 == 0) hi = fminf(hi, e_hi);
    else lo = fmaxf(lo, e_lo);
  }
  if (depth >= 2 && ax == ax1 && a1 != nullptr) {
    const int s1 = (idx >> (depth - 2)) & 1;
    if (s1 == 0) hi = fminf(hi, g3_hi_of(b1[s0]));
    else lo = fmaxf(lo, g3_lo_of(a1[s0]));
  }
  if (depth == 3 && ax == ax2 && a2 != nullptr) {
    const int gi = idx >> 1;
    if ((idx & 1) == 0) hi = fminf(hi, g3_hi_of(b2[gi]));
    else lo = fmaxf(lo, g3_lo_of(a2[gi]));
  }
  if (!(hi >= lo)) hi = lo;
  *lo_out = lo;
  *hi_out = hi;
}

// Sample-histogram bucketing of node k of a segment (0, 1: children on axis l+1; 2 + g:
// grandchildren on axis l+2). Sampler and band kernel compute the same one.
__device__ __forceinline__ BucketParams g3_node_params(const LevelArgs& a, const G3Args& g, const G3Seg* gs, i64 h,
                                                       int k) {
  float e_lo, e_hi, lo, hi;
  g3_bstar_edges(a, h, &e_lo, &e_hi);
  const float* cell = a.cells + h * 2 * a.dim;
  if (k < 2)
    g3_range(cell, a.next_axis, a.axis, a.next_axis, g.axis2, e_lo, e_hi, 1, k, nullptr, nullptr, nullptr, nullptr,
             &lo, &hi);
  else
    g3_range(cell, g.axis2, a.axis, a.next_axis, g.axis2, e_lo, e_hi, 2, k - 2, gs->a1, gs->b1, nullptr, nullptr,
             &lo, &hi);
  return make_params(lo, hi, kG3Bins);
}

// Sample pass PASS (1: children, 2: grandchildren), grid segs x sblocks.
template <int PASS>
__global__ __launch_bounds__(kBlock) void k_g3_sample(LevelArgs a, G3Args g) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int NN = PASS == 1 ? 2 : 4;
  __shared__ u32 hs[NN * kG3Bins];
  __shared__ BucketParams pn[NN];
  __shared__ u32 p1[2];
  const i64 s = blockIdx.x / g.sblocks;
  const int part = blockIdx.x % g.sblocks;
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  const G3Seg* gs = g.g3 + g.seg0 + s;
  for (int i = threadIdx.x; i < NN * kG3Bins; i += kBlock) hs[i] = 0u;
  if (threadIdx.x < NN) pn[threadIdx.x] = g3_node_params(a, g, gs, h, PASS == 1 ? int(threadIdx.x) : 2 + int(threadIdx.x));
  if (PASS == 2 && threadIdx.x < 2) p1[threadIdx.x] = gs->p1[threadIdx.x];
  __syncthreads();
  if (n > 0) {
    const BucketParams prm = a.params[h];
    const u32 bstar = a.state[h].bstar;
    float e_lo, e_hi;
    g3_bstar_edges(a, h, &e_lo, &e_hi);
    const float emid = 0.5f * (e_lo + e_hi);
    const i64 nc = a.ncol;
    const float* c0 = a.src + i64(a.axis) * nc + lo;
    const float* c1 = a.src + i64(a.next_axis) * nc + lo;
    const float* c2 = a.src + i64(g.axis2) * nc + lo;
    const i64 W = i64(kG3Run) * g.sample_div;
    const i64 nwin = (n + W - 1) / W;
    const i64 w0 = nwin * part / g.sblocks, w1 = nwin * (part + 1) / g.sblocks;
    const int w = threadIdx.x / 64, ln = dev::lane();
    const u32 sseed = g3_mix(g.salt * 0x9e3779b9u + u32(g.seg0 + s));
    for (i64 r0 = w0 + i64(w) * kG3SampU; r0 < w1; r0 += i64(kBlock / 64) * kG3SampU) {
      float k0[kG3SampU], k1[kG3SampU], k2[kG3SampU];
      bool v[kG3SampU];
#pragma unroll
      for (int u = 0; u < kG3SampU; ++u) {  // the windows' runs (all loads in flight together)
        const i64 r = r0 + u;
        const i64 wb = r * W, wl = min(W, n - wb);
        const i64 span = wl > kG3Run ? wl - kG3Run + 1 : 1;
        const i64 e = wb + i64(g3_mix(u32(r) ^ sseed) % u32(span)) + ln;
        v[u] = r < w1 && e < wb + wl;
        const i64 ei = v[u] ? e : 0;
        k0[u] = c0[ei];
        k1[u] = c1[ei];
        k2[u] = PASS == 2 ? c2[ei] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kG3SampU; ++u) {
        if (!v[u]) continue;
        const u32 b = bucket_of(k0[u], prm, a.bins);
        const u32 c = b != bstar ? (b < bstar ? 0u : 1u) : (k0[u] < emid ? 0u : 1u);
        if (PASS == 1) {
          atomicAdd(&hs[c * kG3Bins + bucket_of(k1[u], pn[c], kG3Bins)], 1u);
        } else {
          const u32 gi = 2 * c + (orderable(k1[u]) < p1[c] ? 0u : 1u);
          atomicAdd(&hs[gi * kG3Bins + bucket_of(k2[u], pn[gi], kG3Bins)], 1u);
        }
      }
    }
  }
  __syncthreads();
  u32* out = g.shist + (g.seg0 + s) * 6 * kG3Bins + (PASS == 1 ? 0 : 2 * kG3Bins);
  for (int i = threadIdx.x; i < NN * kG3Bins; i += kBlock) {
    const u32 x = hs[i];
    if (x) atomicAdd(&out[i], x);
  }
}

// One wave: the bin of a kG3Bins histogram holding the rank-th element (kG3Bins when
// rank >= total); *below = elements before that bin, *total = all.
__device__ __forceinline__ u32 g3_wave_find(const u32* h, u32 rank, u32* below, u32* total) {
  constexpr int per = kG3Bins / 64;
  const int ln = dev::lane();
  u32 v[per], sum = 0;
#pragma unroll
  for (int i = 0; i < per; ++i) {
    v[i] = h[ln * per + i];
    sum += v[i];
  }
  const u32 incl = dev::wave_incl_scan(sum), excl = incl - sum;
  *total = u32(__shfl(int(incl), 63, 64));
  const u64 m = __ballot(rank >= excl && rank < incl);
  if (!m) {
    *below = *total;
    return u32(kG3Bins);
  }
  const int src = __ffsll((long long)m) - 1;
  u32 bin = 0, bel = excl;
  if (ln == src) {
    int i = 0;
    while (i + 1 < per && rank >= bel + v[i]) bel += v[i++];
    bin = u32(ln * per + i);
  }
  *below = u32(__shfl(int(bel), src, 64));
  return u32(__shfl(int(bin), src, 64));
}

// Keys just below / above every value of bin b of a value-linear bucketing (a margin for the
// bucketing's rounding), as in top4.
__device__ __forceinline__ u32 g3_key_below(BucketParams p, u32 b) {
  const float e = p.lo + float(b) / p.scale;
  return orderable(e - (fabsf(e) * 1e-5f + float(kG3Bins) / p.scale * 1e-6f));
}
__device__ __forceinline__ u32 g3_key_above(BucketParams p, u32 b) {
  const float e = p.lo + float(b + 1) / p.scale;
  return orderable(e + (fabsf(e) * 1e-5f + float(kG3Bins) / p.scale * 1e-6f));
}

// One wave: the band of a node from its sample histogram: inclusive [*A, *B] of orderable keys,
// the estimated pivot, the samples of the band's bins and all samples.
__device__ __forceinline__ void g3_band(const u32* hb, BucketParams p, float z, u32* A, u32* B, u32* P, u32* bs,
                                        u32* tot) {
  u32 below = 0, c = 0;
  (void)g3_wave_find(hb, 0, &below, &c);
  *tot = c;
  *A = 0u;
  *B = 0xffffffffu;
  *P = orderable(p.lo);
  *bs = c;
  if (c == 0 || !(p.scale > 0.0f)) return;  // no resolution: the whole range is the band
  const u32 half = u32(ceilf(z * sqrtf(float(c)) * 0.5f)) + 2u;
  const u32 rm = c / 2, rlo = rm > half ? rm - half : 0u, rhi = min(c - 1, rm + half);
  u32 t = 0, bel_lo = 0, bel_hi = 0;
  const u32 bl = g3_wave_find(hb, rlo, &bel_lo, &t);
  const u32 bm = g3_wave_find(hb, rm, &below, &t);
  const u32 bh = g3_wave_find(hb, rhi, &bel_hi, &t);
  const bool open_lo = rlo == 0 || bl == 0, open_hi = rhi >= c - 1 || bh >= u32(kG3Bins - 1);
  *A = open_lo ? 0u : g3_key_below(p, bl);
  *B = open_hi ? 0xffffffffu : g3_key_above(p, bh);
  *P = orderable(p.lo + (float(bm) + 0.5f) / p.scale);
  *bs = (open_hi ? c : bel_hi + hb[bh]) - (open_lo ? 0u : bel_lo);
}

// Bands from the sample histograms (one workgroup per segment). PASS 1: children; PASS 2:
// grandchildren, then the staging layout, the counters, provisional cells of the 14 nodes below
// (exact ones replace them as the medians are found; a bad segment keeps them), the
// great-grandchildren's bucketing and their zeroed level-(l+3) histograms.
template <int PASS>
__global__ __launch_bounds__(kBlock) void k_g3_band(LevelArgs a, G3Args g) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  __shared__ BucketParams pn[4];
  __shared__ u32 sa1[2], sb1[2], sa2[4], sb2[4], sbs[6], stot[2];
  const i64 s = blockIdx.x, h = a.heap0 + s;
  const i64 n = a.seg_n[h];
  G3Seg* gs = g.g3 + g.seg0 + s;
  const u32* hsamp = g.shist + (g.seg0 + s) * 6 * kG3Bins;
  const int w = threadIdx.x / 64, ln = dev::lane(), tid = threadIdx.x;
  const int D = a.dim;
  if (PASS == 1) {
    if (tid < 2) pn[tid] = g3_node_params(a, g, gs, h, tid);
    __syncthreads();
    if (w < 2) {
      u32 A, B, P, bs, tot;
      g3_band(hsamp + w * kG3Bins, pn[w], g.z, &A, &B, &P, &bs, &tot);
      if (ln == 0) {
        gs->a1[w] = A;
        gs->b1[w] = B;
        gs->p1[w] = P;
        gs->bsamp[w] = bs;
        gs->tot[w] = tot;
      }
    }
    return;
  }
  if (tid < 4) pn[tid] = g3_node_params(a, g, gs, h, 2 + tid);
  if (tid < 2) {
    sa1[tid] = gs->a1[tid];
    sb1[tid] = gs->b1[tid];
    sbs[tid] = gs->bsamp[tid];
    stot[tid] = gs->tot[tid];
  }
  __syncthreads();
  {
    u32 A, B, P, bs, tot;
    g3_band(hsamp + (2 + w) * kG3Bins, pn[w], g.z, &A, &B, &P, &bs, &tot);
    if (ln == 0) {
      gs->a2[w] = A;
      gs->b2[w] = B;
      gs->bsamp[2 + w] = bs;
      sa2[w] = A;
      sb2[w] = B;
      sbs[2 + w] = bs;
    }
  }
  __syncthreads();
  if (tid == 0) {  // staging layout: the band regions first, tag 0 (b*'s rows, counted exactly) last
    const u32 mid = a.state[h].cnt_mid;
    const u32 ctot = stot[0] + stot[1];
    const float scale = float(n) / float(max(1u, ctot));
    u32 cap[7];
    for (int t = 1; t <= 2; ++t) cap[t] = u32(fminf(float(sbs[t - 1]) * scale * 1.5f + 2048.0f, float(n)));
    for (int t = 3; t <= 6; ++t)  // + the rows the resolves append: b*'s and some of the child band's
      cap[t] = u32(fminf(float(sbs[t - 1]) * scale * 1.5f + 2048.0f + float(mid) + 0.5f * float(cap[1 + (t - 3) / 2]),
                         float(n)));
    u64 off = 0;
    for (int t = 1; t <= 6; ++t) {
      gs->off[t] = u32(off);
      off += cap[t];
    }
    const bool fits = off + mid <= u64(n);
    for (int t = 1; t <= 6; ++t) gs->cap[t] = fits ? cap[t] : 0u;
    gs->off[0] = u32(n) - mid;
    gs->cap[0] = fits ? mid : 0u;
    gs->off[7] = 0u;
    gs->cap[7] = 0u;
    gs->bad = fits ? 0u : 1u;
    if (!fits) atomicOr(a.err, top4::kErrBit);
  }
  if (tid < 8) {
    gs->zc[8 + (tid)][0] = 0u;
    gs->zc[tid][0] = 0u;
    gs->ins[tid] = 0u;
  }
  if (g.bins3 > 0)
    for (int i = tid; i < kG3Gg * g.bins3; i += kBlock) g.hist3[(kG3Gg * s) * g.bins3 + i] = 0u;
  if (g.mhist != nullptr)  // the multi-block resolve's band histograms
    for (int i = tid; i < 6 * kG3ResBins; i += kBlock) g.mhist[(g.seg0 + s) * 6 * kG3ResBins + i] = 0u;
  float e_lo, e_hi;
  g3_bstar_edges(a, h, &e_lo, &e_hi);
  const float* cell = a.cells + h * 2 * D;
  for (int e = tid; e < 14 * D; e += kBlock) {  // (node, axis) per thread
    const int k = 1 + e / D, c = e % D;
    const int depth = k < 3 ? 1 : (k < 7 ? 2 : 3);
    const int idx = k - ((1 << depth) - 1);
    float lo, hi;
    g3_range(cell, c, a.axis, a.next_axis, g.axis2, e_lo, e_hi, depth, idx, sa1, sb1, sa2, sb2, &lo, &hi);
    const i64 hk = k < 3 ? 2 * h + k : (k < 7 ? 4 * h + k : 8 * h + k);
    a.cells[hk * 2 * D + 2 * c] = lo;
    a.cells[hk * 2 * D + 2 * c + 1] = hi;
    if (depth == 3 && c == g.axis3 && g.bins3 > 0) a.params[hk] = make_params(lo, hi, g.bins3);
  }
}

// The pass: every row once; 8 great-grandchild zones + the 7 staging regions. Zone ranks as in
// k_partition3: LDS atomics (ATOM) or wave ballots.
// NH > 0 (ballot ranks only): the chunk's rows leave through LDS, in NH parts of KI / NH items:
// each part's rows are written to an LDS tile in zone order, then stored by consecutive threads
// at consecutive destinations, so every store instruction writes whole runs of one zone instead
// of ~8 scattered 32-B pieces (one per zone a wave's 64 rows fall into).
template <int NCOL, int KI, bool ATOM, int NH = 0>
__global__ __launch_bounds__(kBlock) void k_g3_part(LevelArgs a, G3Args g) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int kItems = KI;
  constexpr int kCh = kBlock * KI;
  constexpr int NZ = 15;  // 0..7 great-grandchild, 8 + t staging tag t
  constexpr int D = NCOL - 1;
  constexpr int W = kBlock / 64;
  constexpr bool STG = !ATOM && NH > 0;
  constexpr int NP = STG ? NH : 1;          // parts of a chunk
  constexpr int HI = KI / NP;               // items per part
  constexpr int HROWS = kBlock * HI;        // rows per part (LDS tile)
  static_assert(kItems % 4 == 0, "16-B row loads take 4 rows per item group");
  static_assert(KI % NP == 0, "whole items per part");
  // [8 * bins3] counts (STG: two 16-bit counts per word -- the host stages only blocks of < 64 Ki
  // rows -- so the tile fits beside it at four workgroups per CU), then (STG) the tile: NCOL x HROWS
  // floats + a zone byte per row
  extern __shared__ __align__(16) u32 nh[];
  constexpr int PK = STG ? 2 : 1;  // counts per histogram word
  __shared__ u32 zb_s[16], ztot_s[16], zpst[NP][16], zls[16];
  __shared__ u32 wcnt[W][16];
  __shared__ u32 wbase[W][16];
  __shared__ u32 gcnt[ATOM ? 1 : NZ][64];
  __shared__ BucketParams ggp[8];
  __shared__ i64 glo[8], gn[8];
  __shared__ u32 roff[8], rcap[8];
  __shared__ u32 ba1[2], bb1[2], ba2[4], bb2[4];
  __shared__ u32 sbad;
  i64 s, bidx;
  int part;
  seg_part(a.bps, a.xcd, s, part, bidx);
  const i64 h = a.heap0 + s;
  const i64 lo = a.seg_lo[h], n = a.seg_n[h];
  const int nb3 = g.bins3;
  const bool fuse = nb3 > 0;
  G3Seg* gs = g.g3 + g.seg0 + s;
  if (fuse)
    for (int b = threadIdx.x; b < (kG3Gg * nb3 + PK - 1) / PK; b += kBlock) nh[b] = 0;
  const i64 gg0 = 8 * h + 7;
  if (threadIdx.x < W * 16) (&wcnt[0][0])[threadIdx.x] = 0;
  if (threadIdx.x < 8) {
    const int t = int(threadIdx.x);
    if (fuse) ggp[t] = a.params[gg0 + t];
    glo[t] = a.seg_lo[gg0 + t];
    gn[t] = a.seg_n[gg0 + t];
    roff[t] = gs->off[t];
    rcap[t] = gs->cap[t];
  }
  if (threadIdx.x < 2) {
    ba1[threadIdx.x] = gs->a1[threadIdx.x];
    bb1[threadIdx.x] = gs->b1[threadIdx.x];
  }
  if (threadIdx.x < 4) {
    ba2[threadIdx.x] = gs->a2[threadIdx.x];
    bb2[threadIdx.x] = gs->b2[threadIdx.x];
  }
  if (threadIdx.x == 0) sbad = 0u;
  const i64 per = (n + a.bps - 1) / a.bps;
  const i64 b0 = min(n, i64(part) * per), b1 = min(n, b0 + per);
  const u32 bstar = a.state[h].bstar;
  const BucketParams prm = a.params[h];
  __syncthreads();
  const float* __restrict__ src = a.src;
  float* __restrict__ dst = a.dst;
  float* __restrict__ stg = g.stage;
  const i64 nc = a.ncol;
  const int axis = a.axis, ax1 = a.next_axis, ax2 = g.axis2, ax3 = g.axis3;
  const int w = threadIdx.x / 64;
  auto classify = [&](float k0, float k1, float k2, bool valid) -> u32 {
    if (!valid) return 15u;
    const u32 b = bucket_of(k0, prm, a.bins);
    if (b == bstar) return 8u;  // tag 0
    const u32 c = b < bstar ? 0u : 1u;
    const u32 o1 = orderable(k1);
    if (o1 >= ba1[c] && o1 <= bb1[c]) return 9u + c;  // tag 1 + c
    const u32 gi = 2 * c + (o1 > bb1[c] ? 1u : 0u);
    const u32 o2 = orderable(k2);
    if (o2 >= ba2[gi] && o2 <= bb2[gi]) return 11u + gi;  // tag 3 + gi
    return 2 * gi + (o2 > bb2[gi] ? 1u : 0u);
  };
  const i64 cstart = ((lo + b0) & ~i64(3)) - lo;
  for (i64 c0 = cstart; c0 < b1; c0 += kCh) {
    float row[kItems][NCOL];
    bool vld[kItems];
#pragma unroll
    for (int gq = 0; gq < kItems / 4; ++gq) {
      const i64 e4 = c0 + (i64(gq) * kBlock + threadIdx.x) * 4;
      const i64 p4 = lo + (e4 < b1 ? e4 : cstart);
#pragma unroll
      for (int c = 0; c < NCOL; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(src + i64(c) * nc + p4);
        row[4 * gq + 0][c] = v.x;
        row[4 * gq + 1][c] = v.y;
        row[4 * gq + 2][c] = v.z;
        row[4 * gq + 3][c] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) vld[4 * gq + j] = e4 + j >= b0 && e4 + j < b1;
    }
    u32 zone_pre[kItems];
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      float k0 = row[i][0], k1 = row[i][0], k2 = row[i][0], k3 = row[i][0];
#pragma unroll
      for (int c = 1; c < D; ++c) {
        k0 = c == axis ? row[i][c] : k0;
        k1 = c == ax1 ? row[i][c] : k1;
        k2 = c == ax2 ? row[i][c] : k2;
        k3 = c == ax3 ? row[i][c] : k3;
      }
      const u32 q = classify(k0, k1, k2, vld[i]);
      if constexpr (ATOM) {
        zone_pre[i] = (q << 16) | atomicAdd(&wcnt[w][q], 1u);
      } else {
        zone_pre[i] = (q << 16) | dev::wave_zone_rank<NZ>(q, &gcnt[0][i * 4 + w], 64);
      }
      if (fuse && q < 8u) {
        const u32 hb = q * u32(nb3) + bucket_of(k3, ggp[q], nb3);
        atomicAdd(&nh[hb / PK], STG ? 1u << ((hb & 1u) * 16) : 1u);
      }
    }
    __syncthreads();
    if constexpr (!ATOM) {
      // wave w scans zones w, w + 4, ...; lane k then reserves the wave's k-th zone, so all of the
      // wave's reservations are in flight together (one atomic round trip per chunk, not one per
      // zone: the sequential form put ~4 global-atomic latencies on every chunk's critical path)
      constexpr int ZW = (NZ + W - 1) / W;
      const int ln = dev::lane();
      u32 v[ZW], incl[ZW], tot[ZW];
#pragma unroll
      for (int k = 0; k < ZW; ++k) {
        const int z = w + k * W;
        v[k] = (z < NZ && ln < kItems * 4) ? gcnt[z < NZ ? z : 0][ln] : 0u;
        incl[k] = dev::wave_incl_scan(v[k]);
        tot[k] = __shfl(incl[k], 63, 64);
      }
      u32 mine = 0;
#pragma unroll
      for (int k = 0; k < ZW; ++k) mine = ln == k ? tot[k] : mine;
      const int zl = w + ln * W;
      u32 base = 0;
      if (ln < ZW && zl < NZ && mine) base = atomicAdd(&gs->zc[zl][0], mine);
#pragma unroll
      for (int k = 0; k < ZW; ++k) {
        const int z = w + k * W;
        const u32 b = __shfl(base, k, 64);
        if (z < NZ) gcnt[z][ln] = (STG ? 0u : b) + incl[k] - v[k];  // STG: offset inside the chunk's zone run
        if constexpr (STG) {
          u32 ps[NP];  // part h's first row inside the zone run (groups are item-major: i * W + w)
#pragma unroll
          for (int hp = 0; hp < NP; ++hp) ps[hp] = hp == 0 ? 0u : u32(__shfl(int(incl[k]), hp * HI * W - 1, 64));
          if (z < NZ && ln == 0) {
            zb_s[z] = b;
            ztot_s[z] = tot[k];
#pragma unroll
            for (int hp = 0; hp < NP; ++hp) zpst[hp][z] = ps[hp];
          }
        }
      }
    } else if (threadIdx.x < NZ) {  // zone z's waves, scanned, reserved once per chunk
      const int z = int(threadIdx.x);
      u32 c[W], tot = 0;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        c[k] = wcnt[k][z];
        tot += c[k];
      }
      u32 base = tot ? atomicAdd(&gs->zc[z][0], tot) : 0u;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        wbase[k][z] = base;
        base += c[k];
        wcnt[k][z] = 0;
      }
    }
    if (ATOM && threadIdx.x >= NZ && threadIdx.x < NZ + W) wcnt[threadIdx.x - NZ][15] = 0;
    __syncthreads();
    // destination of the row at offset `off` of zone zi's reservation (false: past its capacity)
    auto dest = [&](u32 zi, u32 off, i64& d, float*& out) -> bool {
      d = -1;
      out = dst;
      if (zi < 8u) {
        if (i64(off) < gn[zi]) d = glo[zi] + off;
      } else if (off < rcap[zi - 8]) {
        d = lo + roff[zi - 8] + off;
        out = stg;
      }
      return d >= 0;
    };
    if constexpr (STG) {
      float* tile = reinterpret_cast<float*>(nh + ((max(1, (kG3Gg * nb3 + 1) / 2) + 3) & ~3));
      unsigned char* tz = reinterpret_cast<unsigned char*>(tile + NCOL * HROWS);
      const int ln = dev::lane();
#pragma unroll
      for (int hp = 0; hp < NP; ++hp) {
        // part hp's tile: zones in order, each zone's rows in (item, wave, lane) order
        const u32 ch = ln < NZ ? (hp + 1 < NP ? zpst[hp + 1 < NP ? hp + 1 : 0][ln] : ztot_s[ln]) - zpst[hp][ln] : 0u;
        const u32 inc = dev::wave_incl_scan(ch);
        const u32 ex = inc - ch;
        if (w == 0 && ln < NZ) zls[ln] = ex;
        if (w == 0 && ln == NZ - 1) zls[NZ] = inc;
#pragma unroll
        for (int ii = 0; ii < HI; ++ii) {
          const int i = hp * HI + ii;
          const u32 zi = zone_pre[i] >> 16;
          const u32 zs = zi < u32(NZ) ? zi : 0u;
          const u32 exz = u32(__shfl(int(ex), int(zs), 64));
          if (zi >= u32(NZ)) continue;
          const u32 p = exz + gcnt[zs][i * 4 + w] - zpst[hp][zs] + (zone_pre[i] & 0xffffu);
#pragma unroll
          for (int c = 0; c < NCOL; ++c) tile[c * HROWS + p] = row[i][c];
          tz[p] = (unsigned char)zi;
        }
        __syncthreads();
        const u32 T = zls[NZ];
        for (u32 j = threadIdx.x; j < T; j += kBlock) {
          const u32 zi = tz[j];
          const u32 off = zb_s[zi] + zpst[hp][zi] + (j - zls[zi]);
          i64 d;
          float* out;
          if (!dest(zi, off, d, out)) {
            sbad = 1u;
            continue;
          }
#pragma unroll
          for (int c = 0; c < NCOL; ++c) out[i64(c) * nc + d] = tile[c * HROWS + j];
        }
        __syncthreads();  // the tile, zls and (last part) gcnt are rewritten next
      }
    } else {
#pragma unroll
      for (int i = 0; i < kItems; ++i) {
        const u32 zi = zone_pre[i] >> 16;
        if (zi >= u32(NZ)) continue;
        const u32 off = (ATOM ? wbase[w][zi] : gcnt[ATOM ? 0 : zi][i * 4 + w]) + (zone_pre[i] & 0xffffu);
        i64 d;
        float* out;
        if (!dest(zi, off, d, out)) {
          sbad = 1u;
          continue;
        }
#pragma unroll
        for (int c = 0; c < NCOL; ++c) out[i64(c) * nc + d] = row[i][c];
      }
      if (!ATOM) __syncthreads();  // the next chunk rewrites gcnt
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && sbad) g3_bad(a.err, gs);
  if (fuse) {
    u32* hn = g.hist3 + (kG3Gg * s) * nb3;
    for (int b = threadIdx.x; b < kG3Gg * nb3; b += kBlock) {
      const u32 v = STG ? (nh[b >> 1] >> ((b & 1) * 16)) & 0xffffu : nh[b];
      if (v) atomicAdd(&hn[b], v);
    }
  }
}

// rank-th smallest (0-based) of the composites that each(f) visits (every thread of the NT calls
// it and visits its share): MSD radix select on 8-bit digits below the highest bit in which the
// candidates differ.
template <int NT, class Each>
__device__ u64 g3_block_select(Each each, u32 rank) {
  __shared__ __align__(16) u32 hist[256];
  __shared__ u64 rmn[NT / 64], rmx[NT / 64];
  __shared__ u32 info[2];
  u64 mn = ~0ull, mx = 0ull;
  each([&](u64 v) {
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  });
  mn = dev::wave_min_u64(mn);
  mx = dev::wave_max_u64(mx);
  __syncthreads();
  if (dev::lane() == 0) {
    rmn[threadIdx.x / 64] = mn;
    rmx[threadIdx.x / 64] = mx;
  }
  __syncthreads();
  mn = rmn[0];
  mx = rmx[0];
  for (int k = 1; k < NT / 64; ++k) {
    mn = rmn[k] < mn ? rmn[k] : mn;
    mx = rmx[k] > mx ? rmx[k] : mx;
  }
  const u64 diff = mn ^ mx;
  if (!diff) return mn;
  int hb = 63 - __builtin_clzll(diff);
  u64 prefix = hb >= 63 ? 0ull : (mn & ~((2ull << hb) - 1ull));
  while (hb >= 0) {
    const int sh = hb >= 7 ? hb - 7 : 0;
    const u32 dmask = (2u << (hb - sh)) - 1u;
    const u64 himask = hb >= 63 ? 0ull : ~((2ull << hb) - 1ull);
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0u;
    __syncthreads();
    each([&](u64 v) {
      if ((v & himask) == prefix) atomicAdd(&hist[u32(v >> sh) & dmask], 1u);
    });
    __syncthreads();
    if (threadIdx.x < 64) {
      const int l = threadIdx.x;
      u32 v4[4], s4 = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v4[q] = hist[4 * l + q];
        s4 += v4[q];
      }
      const u32 incl = dev::wave_incl_scan(s4);
      u32 c = incl - s4;
      if (rank >= c && rank < incl) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (rank >= c && rank < c + v4[q]) {
            info[0] = u32(4 * l + q);
            info[1] = c;
          }
          c += v4[q];
        }
      }
    }
    __syncthreads();
    prefix |= u64(info[0] & dmask) << sh;
    rank -= info[1];
    hb = sh - 1;
  }
  return prefix;
}

// Resolve of one node: LEVEL 0 the segment (over b*'s rows), 1 a child, 2 a grandchild (over
// its band rows). Grid: segments x nodes per segment.
template <int NCOL, int LEVEL>
__global__ __launch_bounds__(kG3Threads) void k_g3_res(LevelArgs a, G3Args g) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int NT = kG3Threads;
  constexpr int D = NCOL - 1;
  constexpr int NODES = LEVEL == 0 ? 1 : (LEVEL == 1 ? 2 : 4);  // nodes of this level per segment
  constexpr int NG = 8 / NODES;                                  // great-grandchildren below a node
  constexpr int R = 4;                                           // rows per thread per move chunk
  __shared__ u32 hres[kG3ResBins];
  __shared__ u64 cand[kG3Cand];
  __shared__ u32 h3[NG * kTripleBins];
  __shared__ u32 lc[16], lbase[16], ssum[NT / 64];
  __shared__ u32 ccnt, sbin, srank, scnt, sbad, sok, sm, st_, incomplete;
  __shared__ BucketParams bp;
  const i64 s = blockIdx.x / NODES;
  const int x = int(blockIdx.x % NODES);
  const i64 h = a.heap0 + s;
  G3Seg* gs = g.g3 + g.seg0 + s;
  const i64 n = a.seg_n[h];
  const int tid = threadIdx.x;
  const int nb3 = g.bins3;
  const i64 nc = a.ncol;
  const int ax = LEVEL == 0 ? a.axis : (LEVEL == 1 ? a.next_axis : g.axis2);
  const i64 hn = LEVEL == 0 ? h : (LEVEL == 1 ? 2 * h + 1 + x : 4 * h + 3 + x);  // the node
  const int tag = LEVEL == 0 ? 0 : (LEVEL == 1 ? 1 + x : 3 + x);
  const int fg = NG * x;               // its first great-grandchild (among the segment's eight)
  const i64 gg0 = 8 * h + 7 + fg;
  float* __restrict__ stg = g.stage;
  const i64 lo = a.seg_lo[h];
  const i64 nn = a.seg_n[hn], nlo = a.seg_lo[hn];
  for (int i = tid; i < NG * nb3; i += NT) h3[i] = 0u;
  if (tid < 16) lc[tid] = 0u;
  if (tid == 0) {  // the node's median: its rank among the staged rows, from exact counts of the rows left of them
    ccnt = 0u;
    sbad = 0u;
    u32 ok = n > 0 && gs->bad == 0u;
    const u32 m = gs->zc[8 + (tag)][0];
    i64 left = 0;
    if (LEVEL == 0) {
      const SegState st = a.state[h];
      left = st.cnt_less;
      ok = ok && m == st.cnt_mid;
    } else if (LEVEL == 1) {  // certain and resolved rows of the child's left grandchild
      left = i64(gs->zc[4 * x][0]) + gs->zc[4 * x + 1][0] + gs->ins[4 * x] + gs->ins[4 * x + 1] + gs->zc[8 + (3 + 2 * x)][0];
    } else {
      left = i64(gs->zc[2 * x][0]) + gs->ins[2 * x];
    }
    const i64 tt = nn / 2 - left;
    const bool hit = m <= gs->cap[tag] && tt >= 0 && tt < i64(m);
    if (ok && !hit) sbad = 1u;  // a band missed its median
    sok = ok && hit;
    sm = m;
    st_ = u32(tt);
  }
  __syncthreads();  // (every counter read before this workgroup moves rows)
  const bool ok = sok != 0u;
  const u32 m = sm, t = st_;
  const i64 r0 = lo + gs->off[tag];  // the node's staged rows: stage rows [r0, r0 + m)
  auto key_at = [&](u32 e) { return stg[i64(ax) * nc + r0 + e]; };
  auto id_at = [&](u32 e) { return reinterpret_cast<const u32*>(stg)[i64(D) * nc + r0 + e]; };
  u64 piv = 0;
  if (ok) {
    // the median's bin (LEVEL 0: all of b* is the candidate set)
    u32 bin = 0, cnt_bin = m, rank = t;
    if (LEVEL > 0) {
      if (tid == 0) {
        const float* cl = a.cells + hn * 2 * D;
        const u32 A = LEVEL == 1 ? gs->a1[x] : gs->a2[x], B = LEVEL == 1 ? gs->b1[x] : gs->b2[x];
        const float flo = fmaxf(g3_lo_of(A), cl[2 * ax]);
        const float fhi = fminf(g3_hi_of(B), cl[2 * ax + 1]);
        bp = make_params(flo, fhi > flo ? fhi : flo, kG3ResBins);
      }
      for (int i = tid; i < kG3ResBins; i += NT) hres[i] = 0u;
      __syncthreads();
      const BucketParams p = bp;
      for (u32 e0 = 0; e0 < m; e0 += NT * 8) {
        float k[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const u32 e = e0 + u * NT + tid;
          k[u] = key_at(e < m ? e : 0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (e0 + u * NT + tid < m) atomicAdd(&hres[bucket_of(k[u], p, kG3ResBins)], 1u);
      }
      __syncthreads();
      constexpr int per = kG3ResBins / NT;  // bins per thread, one block scan
      u32 v[per], sum = 0;
#pragma unroll
      for (int i = 0; i < per; ++i) {
        v[i] = hres[tid * per + i];
        sum += v[i];
      }
      const u32 incl = dev::wave_incl_scan(sum);
      if (dev::lane() == 63) ssum[tid / 64] = incl;
      __syncthreads();
      u32 ex = incl - sum;
      for (int k2 = 0; k2 < tid / 64; ++k2) ex += ssum[k2];
      if (t >= ex && t < ex + sum) {
        u32 c = ex;
        int i = 0;
        while (i + 1 < per && t >= c + v[i]) c += v[i++];
        sbin = u32(tid * per + i);
        srank = t - c;
        scnt = v[i];
      }
      __syncthreads();
      bin = sbin;
      rank = srank;
      cnt_bin = scnt;
    }
    // the bin's composites into LDS (streamed from the stage when they do not fit)
    const bool fits = cnt_bin <= u32(kG3Cand);
    const BucketParams p = bp;
    if (fits) {
      for (u32 e0 = 0; e0 < m; e0 += NT) {
        const u32 e = e0 + tid;
        bool mine = false;
        u64 ck = 0;
        if (e < m) {
          const float kf = key_at(e);
          mine = LEVEL == 0 || bucket_of(kf, p, kG3ResBins) == bin;
          if (mine) ck = composite_key(kf, id_at(e));
        }
        const u64 bm = __ballot(mine);
        if (!bm) continue;
        const int leader = __ffsll((long long)bm) - 1;
        u32 base = 0;
        if (dev::lane() == leader) base = atomicAdd(&ccnt, u32(__popcll(bm)));
        base = u32(__shfl(int(base), leader, 64));
        if (mine) cand[base + mbcnt(bm)] = ck;
      }
      __syncthreads();
    }
    piv = g3_block_select<NT>(
        [&](auto f) {
          if (fits) {
            for (u32 e = tid; e < cnt_bin; e += NT) f(cand[e]);
          } else {
            for (u32 e = tid; e < m; e += NT) {
              const float kf = key_at(e);
              if (LEVEL == 0 || bucket_of(kf, p, kG3ResBins) == bin) f(composite_key(kf, id_at(e)));
            }
          }
        },
        rank);
    // the node's children's cells: its cell split at the pivot
    const float pk = from_orderable(u32(piv >> 32));
    const float* cl = a.cells + hn * 2 * D;
    for (int q = tid; q < 2 * D; q += NT) {
      const float v0 = cl[q];
      a.cells[(2 * hn + 1) * 2 * D + q] = q == 2 * ax + 1 ? pk : v0;
      a.cells[(2 * hn + 2) * 2 * D + q] = q == 2 * ax ? pk : v0;
    }
  }
  // the staged rows move on: the median to its output slot; code 0..NG-1 a great-grandchild
  // (inserted after its certain rows), 8 + t the staging region of tag t (appended), 15 nothing
  const int axis = a.axis, ax1 = a.next_axis, ax2 = g.axis2, ax3 = g.axis3;
  u32 A1[2], B1[2], A2[4], B2[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    A1[i] = gs->a1[i];
    B1[i] = gs->b1[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    A2[i] = gs->a2[i];
    B2[i] = gs->b2[i];
  }
  auto dest = [&](const float* row) -> u32 {
    float k0 = row[0], k1 = row[0], k2 = row[0];
#pragma unroll
    for (int c = 1; c < D; ++c) {
      k0 = c == axis ? row[c] : k0;
      k1 = c == ax1 ? row[c] : k1;
      k2 = c == ax2 ? row[c] : k2;
    }
    const u32 id = __float_as_uint(row[D]);
    const u64 ck = composite_key(LEVEL == 0 ? k0 : (LEVEL == 1 ? k1 : k2), id);
    if (ck == piv) {
      const i64 mpos = nlo + nn / 2;
#pragma unroll
      for (int c = 0; c < D; ++c) a.out_pts[mpos * D + c] = row[c];
      a.out_ids[mpos] = id;
      return 15u;
    }
    const u32 side = ck < piv ? 0u : 1u;
    if (LEVEL == 2) return side;
    u32 gi;
    if (LEVEL == 0) {
      const u32 o1 = orderable(k1);
      if (o1 >= A1[side] && o1 <= B1[side]) return 9u + side;
      gi = 2 * side + (o1 > B1[side] ? 1u : 0u);
    } else {
      gi = 2 * u32(x) + side;
    }
    const u32 o2 = orderable(k2);
    if (o2 >= A2[gi] && o2 <= B2[gi]) return 11u + gi;
    return 2 * gi + (o2 > B2[gi] ? 1u : 0u) - u32(fg);
  };
  if (ok) {
    for (u32 e0 = 0; e0 < m; e0 += NT * R) {
      float row[R][NCOL];
      u32 code[R], rk[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const u32 e = e0 + u * NT + tid;
        const u32 ei = e < m ? e : 0;
#pragma unroll
        for (int c = 0; c < NCOL; ++c) row[u][c] = stg[i64(c) * nc + r0 + ei];
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        code[u] = e0 + u * NT + tid < m ? dest(row[u]) : 15u;
        rk[u] = code[u] < 15u ? atomicAdd(&lc[code[u]], 1u) : 0u;
      }
      __syncthreads();
      if (tid < 15) {  // one reservation per destination per chunk
        const u32 c = lc[tid];
        if (c) lbase[tid] = atomicAdd(tid < 8 ? &gs->ins[fg + tid] : &gs->zc[8 + (tid - 8)][0], c);
        lc[tid] = 0u;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const u32 cd = code[u];
        if (cd >= 15u) continue;
        const u32 q = lbase[cd] + rk[u];
        float* out = a.dst;
        i64 d = -1;
        if (cd < 8u) {
          const i64 gq = gg0 + cd;
          const i64 pos = i64(gs->zc[fg + cd][0]) + q;
          if (pos < a.seg_n[gq]) {
            d = a.seg_lo[gq] + pos;
            if (nb3 > 0) {
              float k3 = row[u][0];
#pragma unroll
              for (int c = 1; c < D; ++c) k3 = c == ax3 ? row[u][c] : k3;
              atomicAdd(&h3[cd * nb3 + bucket_of(k3, a.params[gq], nb3)], 1u);
            }
          }
        } else if (q < gs->cap[cd - 8u]) {
          d = lo + gs->off[cd - 8u] + q;
          out = stg;
        }
        if (d < 0) {
          sbad = 1u;
          continue;
        }
#pragma unroll
        for (int c = 0; c < NCOL; ++c) out[i64(c) * nc + d] = row[u][c];
      }
      __syncthreads();
    }
  }
  __syncthreads();
  if (tid == 0 && sbad) g3_bad(a.err, gs);
  if (nb3 <= 0) return;
  u32* hn3 = g.hist3 + (kG3Gg * s + fg) * nb3;
  if (LEVEL < 2) {  // the inserted rows' level-(l+3) counts
    for (int i = tid; i < NG * nb3; i += NT)
      if (h3[i]) atomicAdd(&hn3[i], h3[i]);
    return;
  }
  // LEVEL 2 is the last writer of its two great-grandchildren: complete -> add the counts;
  // otherwise (this or an earlier step failed) recount them from their slots, so the levels after
  // stay consistent for a build that will be redone anyway
  if (tid == 0) incomplete = 0u;
  __syncthreads();
  if (tid < NG) {
    const u32 placed = atomicAdd(&gs->zc[fg + tid][0], 0u) + atomicAdd(&gs->ins[fg + tid], 0u);
    if (i64(placed) != a.seg_n[gg0 + tid]) atomicOr(&incomplete, 1u);
  }
  __syncthreads();
  if (!incomplete) {
    for (int i = tid; i < NG * nb3; i += NT)
      if (h3[i]) atomicAdd(&hn3[i], h3[i]);
    return;
  }
  if (tid == 0 && n > 0) g3_bad(a.err, gs);
  for (int i = tid; i < NG * nb3; i += NT) h3[i] = 0u;
  __syncthreads();
  for (int k = 0; k < NG; ++k) {
    const i64 gq = gg0 + k;
    const BucketParams p3 = a.params[gq];
    const float* col = a.dst + i64(ax3) * nc + a.seg_lo[gq];
    for (i64 e = tid; e < a.seg_n[gq]; e += NT) atomicAdd(&h3[k * nb3 + bucket_of(col[e], p3, nb3)], 1u);
  }
  __syncthreads();
  for (int i = tid; i < NG * nb3; i += NT) hn3[i] = h3[i];
}

// Multi-block resolve of levels l+1 and l+2 (sampled triples of few, large segments, e.g. the
// 16 segments of level 4: one workgroup per node would leave most CUs idle while it streams its
// band rows three times). Each step runs on K blocks per node and meets the next one at a
// kernel boundary:
//   k_g3_mh  band-row histogram (LDS, flushed to the node's global histogram);
//   k_g3_ms  per node: the median's rank among its band rows (exact counts), its bin;
//   k_g3_mc  the bin's composites appended to the node's candidate list;
//   k_g3_mp  per node: the exact pivot (radix select), the children's cells;
//   k_g3_mr  every band row routed on (the median out, appends / inserts by per-chunk reservation);
//   k_g3_fin per great-grandchild: complete, or (a failed segment) its histogram recounted.
constexpr int kG3MCand = 4096;  // candidates of a node's median bin (multi-block resolve)

struct G3Node {  // per node of a multi-block resolve: [segment][slot], slot 0-1 children, 2-5 grandchildren
  u32 ok, m, t, bin, rank, cnt, ccnt, pad;
  unsigned long long piv;
};

// The node's exact median rank among its staged rows (thread 0 only): *ok false if the segment is
// bad or the band missed (then *miss).
template <int LEVEL>
__device__ __forceinline__ void g3_node_rank(const LevelArgs& a, const G3Seg* gs, i64 h, int x, bool* ok, bool* miss,
                                             u32* m_out, u32* t_out) {
  const int tag = LEVEL == 0 ? 0 : (LEVEL == 1 ? 1 + x : 3 + x);
  const i64 hn = LEVEL == 0 ? h : (LEVEL == 1 ? 2 * h + 1 + x : 4 * h + 3 + x);
  const i64 n = a.seg_n[h], nn = a.seg_n[hn];
  bool good = n > 0 && gs->bad == 0u;
  const u32 m = gs->zc[8 + tag][0];
  i64 left = 0;
  if (LEVEL == 0) {
    const SegState st = a.state[h];
    left = st.cnt_less;
    good = good && m == st.cnt_mid;
  } else if (LEVEL == 1) {  // certain and resolved rows of the child's left grandchild
    left = i64(gs->zc[4 * x][0]) + gs->zc[4 * x + 1][0] + gs->ins[4 * x] + gs->ins[4 * x + 1] + gs->zc[8 + 3 + 2 * x][0];
  } else {
    left = i64(gs->zc[2 * x][0]) + gs->ins[2 * x];
  }
  const i64 tt = nn / 2 - left;
  const bool hit = m <= gs->cap[tag] && tt >= 0 && tt < i64(m);
  *miss = good && !hit;
  *ok = good && hit;
  *m_out = m;
  *t_out = u32(tt);
}

// Bucketing of a node's band rows: its band, narrowed by its exact cell.
template <int LEVEL>
__device__ __forceinline__ BucketParams g3_res_params(const LevelArgs& a, const G3Seg* gs, i64 hn, int x, int ax) {
  const float* cl = a.cells + hn * 2 * a.dim;
  const u32 A = LEVEL == 1 ? gs->a1[x] : gs->a2[x], B = LEVEL == 1 ? gs->b1[x] : gs->b2[x];
  const float flo = fmaxf(g3_lo_of(A), cl[2 * ax]);
  const float fhi = fminf(g3_hi_of(B), cl[2 * ax + 1]);
  return make_params(flo, fhi > flo ? fhi : flo, kG3ResBins);
}

template <int LEVEL>
__global__ __launch_bounds__(kBlock) void k_g3_mh(LevelArgs a, G3Args g, int K) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int NODES = LEVEL == 1 ? 2 : 4;
  __shared__ u32 hres[kG3ResBins];
  __shared__ BucketParams bp;
  __shared__ u32 sm, sgo;
  const i64 s = blockIdx.x / (NODES * K);
  const int x = int(blockIdx.x / K % NODES), part = int(blockIdx.x % K);
  const i64 h = a.heap0 + s;
  const G3Seg* gs = g.g3 + g.seg0 + s;
  const int ax = LEVEL == 1 ? a.next_axis : g.axis2;
  const i64 hn = LEVEL == 1 ? 2 * h + 1 + x : 4 * h + 3 + x;
  const int tag = LEVEL == 1 ? 1 + x : 3 + x;
  for (int i = threadIdx.x; i < kG3ResBins; i += kBlock) hres[i] = 0u;
  if (threadIdx.x == 0) {
    sgo = a.seg_n[h] > 0 && gs->bad == 0u;
    sm = min(gs->zc[8 + tag][0], gs->cap[tag]);
    bp = g3_res_params<LEVEL>(a, gs, hn, x, ax);
  }
  __syncthreads();
  if (!sgo) return;
  const u32 m = sm, per = (m + u32(K) - 1) / u32(K);
  const u32 e0 = min(m, u32(part) * per), e1 = min(m, e0 + per);
  const float* kc = g.stage + i64(ax) * a.ncol + a.seg_lo[h] + gs->off[tag];
  const BucketParams p = bp;
  for (u32 b0 = e0; b0 < e1; b0 += kBlock * 8) {
    float k[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const u32 e = b0 + u * kBlock + threadIdx.x;
      k[u] = kc[e < e1 ? e : e0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b0 + u * kBlock + threadIdx.x < e1) atomicAdd(&hres[bucket_of(k[u], p, kG3ResBins)], 1u);
  }
  __syncthreads();
  u32* out = g.mhist + ((g.seg0 + s) * 6 + (LEVEL == 1 ? 0 : 2) + x) * kG3ResBins;
  for (int i = threadIdx.x; i < kG3ResBins; i += kBlock)
    if (hres[i]) atomicAdd(&out[i], hres[i]);
}

template <int LEVEL>
__global__ __launch_bounds__(kBlock) void k_g3_ms(LevelArgs a, G3Args g) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int NODES = LEVEL == 1 ? 2 : 4;
  __shared__ u32 ssum[kBlock / 64], sok, sm, st_, sbin, srank, scnt;
  const i64 s = blockIdx.x / NODES;
  const int x = int(blockIdx.x % NODES), slot = (LEVEL == 1 ? 0 : 2) + x;
  const i64 h = a.heap0 + s;
  G3Seg* gs = g.g3 + g.seg0 + s;
  G3Node* nd = g.nodes + (g.seg0 + s) * 6 + slot;
  const int tid = threadIdx.x;
  if (tid == 0) {
    bool ok, miss;
    u32 m, t;
    g3_node_rank<LEVEL>(a, gs, h, x, &ok, &miss, &m, &t);
    if (miss) g3_bad(a.err, gs);
    sok = ok;
    sm = m;
    st_ = t;
    sbin = 0xffffffffu;
  }
  __syncthreads();
  const u32 t = st_;
  if (sok) {
    const u32* hb = g.mhist + ((g.seg0 + s) * 6 + slot) * kG3ResBins;
    constexpr int per = kG3ResBins / kBlock;
    u32 v[per], sum = 0;
#pragma unroll
    for (int i = 0; i < per; ++i) {
      v[i] = hb[tid * per + i];
      sum += v[i];
    }
    const u32 incl = dev::wave_incl_scan(sum);
    if (dev::lane() == 63) ssum[tid / 64] = incl;
    __syncthreads();
    u32 ex = incl - sum;
    for (int k2 = 0; k2 < tid / 64; ++k2) ex += ssum[k2];
    if (t >= ex && t < ex + sum) {
      u32 c = ex;
      int i = 0;
      while (i + 1 < per && t >= c + v[i]) c += v[i++];
      sbin = u32(tid * per + i);
      srank = t - c;
      scnt = v[i];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const bool ok = sok && sbin != 0xffffffffu;
    if (sok && !ok) g3_bad(a.err, gs);  // (the histogram does not hold the rank: inconsistent)
    nd->ok = ok;
    nd->m = sm;
    nd->t = t;
    nd->bin = sbin;
    nd->rank = srank;
    nd->cnt = scnt;
    nd->ccnt = 0u;
  }
}

template <int NCOL, int LEVEL>
__global__ __launch_bounds__(kBlock) void k_g3_mc(LevelArgs a, G3Args g, int K) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int NODES = LEVEL == 1 ? 2 : 4;
  constexpr int D = NCOL - 1;
  __shared__ BucketParams bp;
  __shared__ G3Node snd;
  const i64 s = blockIdx.x / (NODES * K);
  const int x = int(blockIdx.x / K % NODES), part = int(blockIdx.x % K), slot = (LEVEL == 1 ? 0 : 2) + x;
  const i64 h = a.heap0 + s;
  const G3Seg* gs = g.g3 + g.seg0 + s;
  G3Node* nd = g.nodes + (g.seg0 + s) * 6 + slot;
  const int ax = LEVEL == 1 ? a.next_axis : g.axis2;
  const i64 hn = LEVEL == 1 ? 2 * h + 1 + x : 4 * h + 3 + x;
  const int tag = LEVEL == 1 ? 1 + x : 3 + x;
  if (threadIdx.x == 0) {
    snd = *nd;
    bp = g3_res_params<LEVEL>(a, gs, hn, x, ax);
  }
  __syncthreads();
  if (!snd.ok || snd.cnt > u32(kG3MCand)) return;  // (too many: the select streams them instead)
  const u32 m = snd.m, per = (m + u32(K) - 1) / u32(K);
  const u32 e0 = min(m, u32(part) * per), e1 = min(m, e0 + per);
  const i64 r0 = a.seg_lo[h] + gs->off[tag];
  const float* kc = g.stage + i64(ax) * a.ncol + r0;
  const u32* ic = reinterpret_cast<const u32*>(g.stage) + i64(D) * a.ncol + r0;
  u64* cand = g.cand + ((g.seg0 + s) * 6 + slot) * kG3MCand;
  const BucketParams p = bp;
  for (u32 b0 = e0; b0 < e1; b0 += kBlock) {  // uniform trip count: ballots below
    const u32 e = b0 + threadIdx.x;
    bool mine = false;
    float kf = 0.0f;
    if (e < e1) {
      kf = kc[e];
      mine = bucket_of(kf, p, kG3ResBins) == snd.bin;
    }
    const u64 bm = __ballot(mine);
    if (!bm) continue;
    const int leader = __ffsll((long long)bm) - 1;
    u32 base = 0;
    if (dev::lane() == leader) base = atomicAdd(&nd->ccnt, u32(__popcll(bm)));
    base = u32(__shfl(int(base), leader, 64));
    if (mine) cand[base + mbcnt(bm)] = composite_key(kf, ic[e]);
  }
}

template <int NCOL, int LEVEL>
__global__ __launch_bounds__(kG3Threads) void k_g3_mp(LevelArgs a, G3Args g) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int NT = kG3Threads;
  constexpr int NODES = LEVEL == 1 ? 2 : 4;
  constexpr int D = NCOL - 1;
  __shared__ G3Node snd;
  __shared__ BucketParams bp;
  const i64 s = blockIdx.x / NODES;
  const int x = int(blockIdx.x % NODES), slot = (LEVEL == 1 ? 0 : 2) + x;
  const i64 h = a.heap0 + s;
  const G3Seg* gs = g.g3 + g.seg0 + s;
  G3Node* nd = g.nodes + (g.seg0 + s) * 6 + slot;
  const int ax = LEVEL == 1 ? a.next_axis : g.axis2;
  const i64 hn = LEVEL == 1 ? 2 * h + 1 + x : 4 * h + 3 + x;
  const int tag = LEVEL == 1 ? 1 + x : 3 + x;
  const int tid = threadIdx.x;
  if (tid == 0) {
    snd = *nd;
    bp = g3_res_params<LEVEL>(a, gs, hn, x, ax);
  }
  __syncthreads();
  if (!snd.ok) return;
  const u32 m = snd.m, cnt = snd.cnt, bin = snd.bin;
  const bool fits = cnt <= u32(kG3MCand);
  const i64 r0 = a.seg_lo[h] + gs->off[tag];
  const float* kc = g.stage + i64(ax) * a.ncol + r0;
  const u32* ic = reinterpret_cast<const u32*>(g.stage) + i64(D) * a.ncol + r0;
  const u64* cand = g.cand + ((g.seg0 + s) * 6 + slot) * kG3MCand;
  const BucketParams p = bp;
  const u64 piv = g3_block_select<NT>(
      [&](auto f) {
        if (fits) {
          for (u32 e = tid; e < cnt; e += NT) f(cand[e]);
        } else {
          for (u32 e = tid; e < m; e += NT) {
            const float kf = kc[e];
            if (bucket_of(kf, p, kG3ResBins) == bin) f(composite_key(kf, ic[e]));
          }
        }
      },
      snd.rank);
  if (tid == 0) nd->piv = piv;
  const float pk = from_orderable(u32(piv >> 32));
  const float* cl = a.cells + hn * 2 * D;
  for (int q = tid; q < 2 * D; q += NT) {
    const float v0 = cl[q];
    a.cells[(2 * hn + 1) * 2 * D + q] = q == 2 * ax + 1 ? pk : v0;
    a.cells[(2 * hn + 2) * 2 * D + q] = q == 2 * ax ? pk : v0;
  }
}

template <int NCOL, int LEVEL>
__global__ __launch_bounds__(kBlock) void k_g3_mr(LevelArgs a, G3Args g, int K) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  constexpr int NT = kBlock;
  constexpr int D = NCOL - 1;
  constexpr int NODES = LEVEL == 1 ? 2 : 4;
  constexpr int NG = 8 / NODES;
  constexpr int R = 4;
  __shared__ u32 h3[NG * kTripleBins];
  __shared__ u32 lc[16], lbase[16], sbad;
  __shared__ G3Node snd;
  const i64 s = blockIdx.x / (NODES * K);
  const int x = int(blockIdx.x / K % NODES), part = int(blockIdx.x % K), slot = (LEVEL == 1 ? 0 : 2) + x;
  const i64 h = a.heap0 + s;
  G3Seg* gs = g.g3 + g.seg0 + s;
  const int tid = threadIdx.x;
  const int nb3 = g.bins3;
  const i64 nc = a.ncol;
  const i64 hn = LEVEL == 1 ? 2 * h + 1 + x : 4 * h + 3 + x;
  const int tag = LEVEL == 1 ? 1 + x : 3 + x;
  const int fg = NG * x;
  const i64 gg0 = 8 * h + 7 + fg;
  float* __restrict__ stg = g.stage;
  const i64 lo = a.seg_lo[h];
  const i64 nn = a.seg_n[hn], nlo = a.seg_lo[hn];
  for (int i = tid; i < NG * nb3; i += NT) h3[i] = 0u;
  if (tid < 16) lc[tid] = 0u;
  if (tid == 0) {
    snd = g.nodes[(g.seg0 + s) * 6 + slot];
    sbad = 0u;
  }
  __syncthreads();
  if (!snd.ok) return;
  const u64 piv = snd.piv;
  const u32 m = snd.m, per = (m + u32(K) - 1) / u32(K);
  const u32 e0 = min(m, u32(part) * per), e1 = min(m, e0 + per);
  const i64 r0 = lo + gs->off[tag];
  const int ax1 = a.next_axis, ax2 = g.axis2, ax3 = g.axis3;
  u32 A2[4], B2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    A2[i] = gs->a2[i];
    B2[i] = gs->b2[i];
  }
  auto dest = [&](const float* row) -> u32 {
    float k1 = row[0], k2 = row[0];
#pragma unroll
    for (int c = 1; c < D; ++c) {
      k1 = c == ax1 ? row[c] : k1;
      k2 = c == ax2 ? row[c] : k2;
    }
    const u32 id = __float_as_uint(row[D]);
    const u64 ck = composite_key(LEVEL == 1 ? k1 : k2, id);
    if (ck == piv) {
      const i64 mpos = nlo + nn / 2;
#pragma unroll
      for (int c = 0; c < D; ++c) a.out_pts[mpos * D + c] = row[c];
      a.out_ids[mpos] = id;
      return 15u;
    }
    const u32 side = ck < piv ? 0u : 1u;
    if (LEVEL == 2) return side;
    const u32 gi = 2 * u32(x) + side;
    const u32 o2 = orderable(k2);
    if (o2 >= A2[gi] && o2 <= B2[gi]) return 11u + gi;
    return 2 * gi + (o2 > B2[gi] ? 1u : 0u) - u32(fg);
  };
  for (u32 b0 = e0; b0 < e1; b0 += NT * R) {
    float row[R][NCOL];
    u32 code[R], rk[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const u32 e = b0 + u * NT + tid;
      const u32 ei = e < e1 ? e : e0;
#pragma unroll
      for (int c = 0; c < NCOL; ++c) row[u][c] = stg[i64(c) * nc + r0 + ei];
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      code[u] = b0 + u * NT + tid < e1 ? dest(row[u]) : 15u;
      rk[u] = code[u] < 15u ? atomicAdd(&lc[code[u]], 1u) : 0u;
    }
    __syncthreads();
    if (tid < 15) {  // one reservation per destination per chunk
      const u32 c = lc[tid];
      if (c) lbase[tid] = atomicAdd(tid < 8 ? &gs->ins[fg + tid] : &gs->zc[tid][0], c);
      lc[tid] = 0u;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const u32 cd = code[u];
      if (cd >= 15u) continue;
      const u32 q = lbase[cd] + rk[u];
      float* out = a.dst;
      i64 d = -1;
      if (cd < 8u) {
        const i64 gq = gg0 + cd;
        const i64 pos = i64(gs->zc[fg + cd][0]) + q;
        if (pos < a.seg_n[gq]) {
          d = a.seg_lo[gq] + pos;
          if (nb3 > 0) {
            float k3 = row[u][0];
#pragma unroll
            for (int c = 1; c < D; ++c) k3 = c == ax3 ? row[u][c] : k3;
            atomicAdd(&h3[cd * nb3 + bucket_of(k3, a.params[gq], nb3)], 1u);
          }
        }
      } else if (q < gs->cap[cd - 8u]) {
        d = lo + gs->off[cd - 8u] + q;
        out = stg;
      }
      if (d < 0) {
        sbad = 1u;
        continue;
      }
#pragma unroll
      for (int c = 0; c < NCOL; ++c) out[i64(c) * nc + d] = row[u][c];
    }
    __syncthreads();
  }
  __syncthreads();
  if (tid == 0 && sbad) g3_bad(a.err, gs);
  if (nb3 <= 0) return;
  u32* hn3 = g.hist3 + (kG3Gg * s + fg) * nb3;
  for (int i = tid; i < NG * nb3; i += NT)
    if (h3[i]) atomicAdd(&hn3[i], h3[i]);
}

// One workgroup per great-grandchild after a multi-block resolve: every row placed, or (a failed
// segment) its level-(l+3) histogram recounted from its slots.
__global__ __launch_bounds__(kBlock) void k_g3_fin(LevelArgs a, G3Args g) {
  if (dev::build_failed(a.err)) return;  // the build already failed (a miss): it is redone
  __shared__ u32 h3[kTripleBins];
  __shared__ u32 incomplete;
  const i64 s = blockIdx.x / kG3Gg;
  const int k = int(blockIdx.x % kG3Gg);
  const i64 h = a.heap0 + s;
  G3Seg* gs = g.g3 + g.seg0 + s;
  const i64 gq = 8 * h + 7 + k;
  const int nb3 = g.bins3;
  if (threadIdx.x == 0) {
    incomplete = i64(gs->zc[k][0]) + gs->ins[k] != a.seg_n[gq];
    if (incomplete && a.seg_n[h] > 0) g3_bad(a.err, gs);
  }
  __syncthreads();
  if (!incomplete || nb3 <= 0) return;
  for (int i = threadIdx.x; i < nb3; i += kBlock) h3[i] = 0u;
  __syncthreads();
  const BucketParams p3 = a.params[gq];
  const float* col = a.dst + i64(g.axis3) * a.ncol + a.seg_lo[gq];
  for (i64 e = threadIdx.x; e < a.seg_n[gq]; e += kBlock) atomicAdd(&h3[bucket_of(col[e], p3, nb3)], 1u);
  __syncthreads();
  u32* out = g.hist3 + (kG3Gg * s + k) * nb3;
  for (int i = threadIdx.x; i < nb3; i += kBlock) out[i] = h3[i];
}

// =====================================================================================
// Tail levels: the last three global levels of a segment (<= 16 Ki rows) in ONE workgroup.
// The segment's rows stay where the previous scatter put them; every row is read once per
// level (only that level's key column, coalesced, one row per lane per item) and once more
// when it moves, so the three levels cost 3 x 4 + 16 B read and 16 B written per row instead
// of a triple's two key sweeps, its 12-zone scatter (8 + 12 + 32 B) and five small kernels
// between them. Per level, for the level's 1 / 2 / 4 sub-segments at once:
//   bins      a linear histogram of the key over the sub-segment's cell (LDS atomics), a
//             block scan, and the bin holding the median rank (n_s / 2) of each sub-segment;
//   select    the median bin's rows ((key, id) composite) ranked by one wave per sub-segment
//             (<= 64 candidates), or a block-wide radix select over the composite key (8-bit
//             digits, any number of candidates: heavy duplicates);
//   classify  every live row goes left / right of its sub-segment's pivot (a row's id is read
//             only when its key equals the pivot key); the median row is written to its
//             output slot; the children's cells are set.
// Then every row gets its position in its leaf from one LDS atomic on its wave's leaf counter
// plus the waves' prefix, and each column is staged through LDS in leaf order and written
// back with coalesced stores (the 7 median slots carry garbage in the scratch columns; the
// subtree kernel reads only leaf ranges).
constexpr int kTailThreads = 1024;
constexpr int kTailBins = 4096;  // bins of a level, split evenly among its sub-segments
constexpr int kTailCand = 64;    // median-bin candidates one wave ranks

struct TailArgs {
  const float* src;
  float* dst;
  i64 ncol;
  const i64* seg_lo;
  const i64* seg_n;
  float* cells;  // heap-indexed [h][dim][2]
  i64 heap0;     // first segment (of this part) at level L
  int level;     // L: the first tail level
  int depth0;
  float* out_pts;
  u32* out_ids;
  u32* err;
  unsigned long long* stamps;  // diagnostic (PKD_TAIL_STAMPS=1): [block][kTailStampSlots] s_memtime, else null
  int pipe;                    // move phase: next column's loads in flight, two stage buffers (2 x CAP words)
};
constexpr int kTailStampSlots = 24, kTailStampBlocks = 2048;
__device__ __forceinline__ void tail_stamp(const TailArgs& a, int slot) {
  if (a.stamps != nullptr && blockIdx.x < kTailStampBlocks && __builtin_amdgcn_readfirstlane(threadIdx.x) < 64)
    a.stamps[blockIdx.x * kTailStampSlots + slot] = __builtin_amdgcn_s_memtime();
}

// exclusive scan over the 1024 threads of a block (one value each); *total = the sum.
// Caller: a barrier between two uses (wsum is reused).
__device__ __forceinline__ u32 block_excl_scan1024(u32 v, u32* wsum, u32* total, int tid) {
  const int w = tid / 64, ln = tid & 63;
  const u32 incl = dev::wave_incl_scan(v);
  if (ln == 63) wsum[w] = incl;
  __syncthreads();
  const u32 wi = dev::wave_incl_scan(ln < kTailThreads / 64 ? wsum[ln] : 0u);
  const u32 before = w > 0 ? u32(__shfl(wi, w - 1, 64)) : 0u;
  *total = u32(__shfl(wi, kTailThreads / 64 - 1, 64));
  return before + incl - v;
}

// SLIM (D >= 3): two key register sets (level 2's keys reuse level 0's, loaded when level 2
// starts) and no id registers (a row's id is read from its column only where a key equals the
// pivot key or the row is a median-bin candidate): 32 fewer registers per 16 items, so the
// 16-item shape of the 1 B build spills 120 instead of 212 bytes per lane (the 12-item one none).
// IDS: ids in registers (default unless SLIM); SLIM with IDS keeps the two key sets and the ids.
// LEV = 4 (8-D builds: 17 global levels leave 13 between the top and the tail, three triples
// and a 4-level tail instead of two triples, two pairs and a 3-level tail): the same steps for
// one more level (8 sub-segments at the last one, 16 leaves), SLIM: level t's keys in register
// set t & 1, reloaded for levels 2 and 3 (each issued when the level before it starts).
template <int D, int ITEMS, int WPE, bool SLIM = false, bool IDS = !SLIM, int LEV = 3>
__global__ __launch_bounds__(kTailThreads) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_tail3(TailArgs a) {
  constexpr int T = kTailThreads, W = T / 64, CAP = T * ITEMS, NB = kTailBins, G = ITEMS / 4;
  static_assert(!SLIM || D >= 3, "slim registers need three distinct level axes");
  static_assert(LEV == 3 || LEV == 4, "3 or 4 tail levels");
  static_assert(LEV == 3 || D < 3 || SLIM, "4 levels keep two key register sets");
  constexpr int NS = 1 << (LEV - 1), NLEAF = 1 << LEV, NNODE = NLEAF - 1, NALL = 2 * NLEAF - 1;
  // columns kept in registers: every column for D < 3, else the three levels' key columns (SLIM: two sets)
  constexpr int KC = D < 3 ? D : (SLIM ? 2 : 3);
  constexpr u32 kDead = 0xffffffffu, kMed = 0x80000000u;  // absent row / median of tail node (low bits)
  static_assert(ITEMS % 4 == 0, "16-B groups of 4 rows");
  static_assert(CAP >= NB, "the stage buffer holds the bins");
  extern __shared__ __align__(16) u32 stage[];  // CAP words: the output columns; bins / counters alias it
  u32* bins = stage;
  __shared__ u32 ckey[NS][kTailCand], cid[NS][kTailCand];
  __shared__ u32 ccnt[NS], sbst[NS], srank[NS], wsum[W];
  __shared__ unsigned long long spiv[NS];
  __shared__ float scell[2][NLEAF][D][2];  // cells of the level's sub-segments / of their children
  __shared__ BucketParams sprm[NS];
  __shared__ i64 nlo[NALL];                // segment starts of the tail's nodes and leaves (heap order below h)
  __shared__ u32 nn[NALL];
  __shared__ u32 sbig, failed;
  dev::build_failed_issue(a.err, &failed);  // tested after the first barrier (level 0)
  const int tid = threadIdx.x, w = tid / 64, ln = dev::lane();
  const i64 h = a.heap0 + blockIdx.x;
  const i64 lo = a.seg_lo[h];
  const int n = int(a.seg_n[h]);
  if (n <= 0) return;
  const int shift = int(lo & 3);  // rows are read in 16-B aligned groups of 4 from lo - shift
  if (n + shift > CAP) {  // the host sizes ITEMS from the largest segment; never expected
    if (tid == 0) atomicOr(a.err, 16u);
    return;
  }
  tail_stamp(a, 0);
  const i64 nc = a.ncol;
  // Item i = 4 g + j of a thread is row (g * T + tid) * 4 + j - shift of the segment: one 16-B
  // load per group of 4 rows. Rows are addressed through buffer descriptors (one per column,
  // wave-uniform): the lane offset tid * 16 is the only per-lane address register, g's
  // g * 16 KiB the scalar offset.
  const u32 vo = u32(tid) * 16u;
  const i64 alo = lo - shift;
  const int recs = (shift + n + 3) & ~3;
  auto col = [&](const float* base, int c) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + i64(c) * nc + alo), 0, recs * 4, 0x00020000);
  };
  auto ld4 = [&](const __amdgpu_buffer_rsrc_t& r, int g) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, vo, u32(g * T * 16), 0);
  };
  // every row's level keys and id, loaded at once (the whole segment in flight)
  int axis_of[LEV];
#pragma unroll
  for (int t = 0; t < LEV; ++t) axis_of[t] = (a.depth0 + a.level + t) % D;
  // the nodes' geometry and the root cell into LDS BEFORE the key loads are issued: their LDS
  // stores wait for their own global loads, and the load counter is in order, so behind the keys'
  // loads they made wave 0 (and with it the first barrier) wait for the whole segment's keys and
  // ids; ahead of them, level 0 starts as soon as its own key column is in (the compiler barrier
  // keeps the order)
  {  // (all three loads in flight together, then the stores)
    i64 vlo = 0;
    u32 vn = 0;
    float vc = 0.0f;
    if (tid < NALL) {  // node k (heap order below h: 0 = h, 1-2 children, ..., NNODE.. the leaves)
      const int lev = 31 - __builtin_clz(u32(tid) + 1u);
      const i64 hk = (h + 1) * (i64(1) << lev) - 1 + (tid - ((1 << lev) - 1));
      vlo = a.seg_lo[hk];
      vn = u32(a.seg_n[hk]);
    }
    if (tid < 2 * D) vc = a.cells[h * 2 * D + tid];
    if (tid < NALL) {
      nlo[tid] = vlo;
      nn[tid] = vn;
    }
    if (tid < 2 * D) (&scell[0][0][0][0])[tid] = vc;
  }
  asm volatile("" ::: "memory");
  float xs[KC][ITEMS];
  u32 ids[IDS ? ITEMS : 1];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const auto r = col(a.src, D < 3 ? k : axis_of[k]);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const auto v = ld4(r, g);
#pragma unroll
      for (int j = 0; j < 4; ++j) xs[k][4 * g + j] = __uint_as_float(v[j]);
    }
  }
  const auto rid = col(a.src, D);
  if constexpr (IDS) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const auto v = ld4(rid, g);
#pragma unroll
      for (int j = 0; j < 4; ++j) ids[4 * g + j] = v[j];
    }
  }
  auto id_of = [&](int i) -> u32 {  // item i's id: a register, or (SLIM) one dword load
    if constexpr (!IDS) return __builtin_amdgcn_raw_buffer_load_b32(rid, vo + u32(i % 4) * 4u, u32(i / 4 * T * 16), 0);
    else return ids[i];
  };
  // path: the row's sub-segment at the current level (while a level bins, its bin: the
  // sub-segment is bin >> lgB); kDead for absent rows, kMed | node for the tail's medians
  u32 path[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int r = (i / 4 * T + tid) * 4 + i % 4 - shift;
    path[i] = (r >= 0 && r < n) ? 0u : kDead;
  }
#pragma unroll
  for (int t = 0; t < LEV; ++t) {
    // the thread index, opaque per level: addresses derived from it (LDS and global, of the
    // few-thread steps) are recomputed per level instead of held in registers across levels
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int wq = tq / 64, lq = tq & 63;
    const int S = 1 << t, B = NB >> t, lgB = 12 - t;
    static_assert(NB == 4096, "lgB");
    const int axis = axis_of[t];
    const int kx = D < 3 ? axis : (SLIM ? (t & 1) : t);  // register set of this level's keys
    if (SLIM && t + 1 >= 2 && t + 1 < LEV) {  // level t+1's keys into level t-1's (dead) registers, issued
      const auto r = col(a.src, axis_of[t + 1]);  // a whole level ahead of their use
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const auto v = ld4(r, g);
#pragma unroll
        for (int j = 0; j < 4; ++j) xs[(t + 1) & 1][4 * g + j] = __uint_as_float(v[j]);
      }
    }
    for (int b = tq; b < NB; b += T) bins[b] = 0;
    if (tq < NS) {
      ccnt[tq] = 0;
      sbst[tq] = 0xffffffffu;
      spiv[tq] = ~0ull;
    }
    if (t == 0) {
      __syncthreads();  // nn / scell
      if (failed) return;  // the build already failed (a miss): it is redone
    }
    if (tq < S) {
      const float* c = &scell[t & 1][tq][axis][0];
      sprm[tq] = make_params(c[0], c[1], B);
    }
    __syncthreads();
    if (t < 3) tail_stamp(a, 1 + 4 * t);  // (level 3 of a 4-level tail: counted in move.rank)
    // ---- bins ----
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (path[i] < kMed) {
        const u32 sp = path[i];
        path[i] = sp * u32(B) + bucket_of(xs[kx][i], sprm[sp], B);
        atomicAdd(&bins[path[i]], 1u);
      }
    }
    __syncthreads();
    {
      u32 c[NB / T], sum = 0;
#pragma unroll
      for (int j = 0; j < NB / T; ++j) {
        c[j] = bins[tq * (NB / T) + j];
        sum += c[j];
      }
      u32 total;
      const u32 ex = block_excl_scan1024(sum, wsum, &total, tq);
      const int sp = tq * (NB / T) / B;  // B is a multiple of NB / T: a thread's bins share a sub-segment
      u32 start = 0;
      for (int q = 0; q < sp; ++q) start += nn[S - 1 + q];
      u32 run = ex - start;
      const u32 m = nn[S - 1 + sp] / 2;
#pragma unroll
      for (int j = 0; j < NB / T; ++j) {
        if (run <= m && m < run + c[j]) {
          sbst[sp] = u32(tq * (NB / T) + j);
          srank[sp] = m - run;
        }
        run += c[j];
      }
    }
    __syncthreads();
    if (t < 3) tail_stamp(a, 2 + 4 * t);  // (level 3 of a 4-level tail: counted in move.rank)
    // ---- candidates of the median bins: (key, id) straight from registers ----
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const u32 sp = path[i] >> lgB;
      if (path[i] < kMed && path[i] == sbst[sp]) {
        const u32 k = atomicAdd(&ccnt[sp], 1u);
        if (k < u32(kTailCand)) {
          ckey[sp][k] = orderable(xs[kx][i]);
          cid[sp][k] = id_of(i);
        }
      }
    }
    __syncthreads();
    if (tq == 0) {
      u32 big = 0;
      for (int q = 0; q < S; ++q) big |= ccnt[q] > u32(kTailCand) ? 1u : 0u;
      sbig = big;
    }
    if (wq < S) {  // wave s ranks sub-segment s's candidates (results unused if any list overflowed)
      const int sp = wq;
      const int m = int(min(ccnt[sp], u32(kTailCand)));
      const u64 ck = lq < m ? (u64(ckey[sp][lq]) << 32) | u64(cid[sp][lq]) : ~0ull;
      u32 rank = 0;
#pragma unroll 1
      for (int j = 0; j < m; ++j) rank += dev::shfl_u64(ck, j) < ck ? 1u : 0u;
      if (lq < m && rank == srank[sp] && ccnt[sp] <= u32(kTailCand)) spiv[sp] = ck;
    }
    __syncthreads();
    if (sbig) {
      // radix select over the composite (key, id) of every sub-segment's median-bin rows,
      // 8 bits per pass from the top (ids are distinct, so 8 passes leave one row)
      if (tq < NS) spiv[tq] = 0;
#pragma unroll 1
      for (int pass = 0; pass < 8; ++pass) {
        const int sh = 56 - 8 * pass;
        const u64 known = pass == 0 ? 0ull : (~0ull << (sh + 8));  // digits fixed by earlier passes
        for (int b = tq; b < NS * 256; b += T) bins[b] = 0;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const u32 sp = path[i] >> lgB;
          if (path[i] < kMed && path[i] == sbst[sp]) {
            const u64 ck = (u64(orderable(xs[kx][i])) << 32) | u64(id_of(i));
            if (((ck ^ spiv[sp]) & known) == 0) atomicAdd(&bins[sp * 256 + u32((ck >> sh) & 255u)], 1u);
          }
        }
        __syncthreads();
        if (wq < S) {  // wave s: digits 4 lq .. 4 lq + 3 of sub-segment s
          const int sp = wq;
          u32 c4[4], sum = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            c4[j] = bins[sp * 256 + 4 * lq + j];
            sum += c4[j];
          }
          u32 run = dev::wave_incl_scan(sum) - sum;
          const u32 r = srank[sp];
          u32 found = 0xffffffffu, nr = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (run <= r && r < run + c4[j]) {
              found = u32(4 * lq + j);
              nr = r - run;
            }
            run += c4[j];
          }
          if (found != 0xffffffffu) {
            spiv[sp] |= u64(found) << sh;
            srank[sp] = nr;
          }
        }
        __syncthreads();
      }
    }
    if (t < 3) tail_stamp(a, 3 + 4 * t);  // (level 3 of a 4-level tail: counted in move.rank)
    // ---- classify: left / right of the pivot; the median row is marked (written with the columns) ----
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (path[i] >= kMed) continue;
      const u32 sp = path[i] >> lgB;
      const u64 pv = spiv[sp];
      const u32 ok = orderable(xs[kx][i]), pk = u32(pv >> 32);
      if (ok != pk) {  // the key decides (the id is read only on a key tie with the pivot)
        path[i] = 2 * sp + (ok > pk ? 1u : 0u);
      } else {
        const u64 ck = (u64(ok) << 32) | u64(id_of(i));
        path[i] = ck == pv ? (kMed | u32(S - 1 + sp)) : 2 * sp + (ck > pv ? 1u : 0u);
      }
    }
    if (tq < 2 * S) {  // children cells: the pivot key bounds the split axis
      const int sp = tq / 2, side = tq & 1;
      const float pkf = from_orderable(u32(spiv[sp] >> 32));
      const i64 hs = (h + 1) * S - 1 + sp;
      float* gc = a.cells + (2 * hs + 1 + side) * 2 * D;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        float clo = scell[t & 1][sp][c][0], chi = scell[t & 1][sp][c][1];
        if (c == axis) {
          if (side == 0) chi = pkf;
          else clo = pkf;
        }
        scell[(t + 1) & 1][tq][c][0] = clo;
        scell[(t + 1) & 1][tq][c][1] = chi;
        gc[2 * c] = clo;
        gc[2 * c + 1] = chi;
      }
    }
    __syncthreads();
    if (t < 3) tail_stamp(a, 4 + 4 * t);  // (level 3 of a 4-level tail: counted in move.rank)
  }
  // ---- move: position inside the leaf (one LDS counter per 16 lanes and leaf), then each
  // column staged through LDS in leaf order and written back coalesced ----
  constexpr int kGroups = W * 4;
  static_assert(CAP >= kGroups * NLEAF, "counters in the stage buffer");
  __shared__ u32 gbase[kGroups][NLEAF];
  u32* gcnt = stage;
  const int grp = tid / 16;
  for (int k = tid; k < kGroups * NLEAF; k += T) gcnt[k] = 0;
  __syncthreads();
  // (leaf << 24) | rank among the 16-lane group's rows of that leaf, in place of the leaf index
#pragma unroll
  for (int i = 0; i < ITEMS; ++i)
    if (path[i] < kMed) path[i] = (path[i] << 24) | atomicAdd(&gcnt[grp * NLEAF + path[i]], 1u);
  __syncthreads();
  if (tid < NLEAF) {
    const u32 first = u32(nlo[NNODE + tid] - lo);
    u32 off = first;
    for (int k = 0; k < kGroups; ++k) {
      gbase[k][tid] = off;
      off += gcnt[k * NLEAF + tid];
    }
    if (off - first != nn[NNODE + tid]) atomicOr(a.err, 16u);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < ITEMS; ++i)
    if (path[i] < kMed) path[i] = (path[i] & 0xffffffu) + gbase[grp][path[i] >> 24];
  tail_stamp(a, 13);
  // column c's register set (a level's keys), or -1: loaded
  auto kreg_of = [&](int c) {
    int kreg = -1;
#pragma unroll
    for (int k = 0; k < KC; ++k)  // (SLIM: set k holds the keys of the last level t with t & 1 == k)
      if ((D < 3 ? k : (SLIM ? axis_of[((LEV - 1) & 1) == k ? LEV - 1 : LEV - 2] : axis_of[k])) == c) kreg = k;
    return kreg;
  };
  auto loaded = [&](int c) { return c == D ? !IDS : kreg_of(c) < 0; };
  auto load_col = [&](int c, u32 (&v)[ITEMS]) {
    const auto r = col(a.src, c);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const auto q = ld4(r, g);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * g + j] = q[j];
    }
  };
  // pipe: the next loaded column's loads are issued before this column is staged and stored, and
  // the columns alternate between two stage buffers (one barrier per column instead of two): the
  // load latency and the barrier no longer serialise the D + 1 columns of the one workgroup per CU
  const bool pipe = a.pipe != 0;
  u32 pre[ITEMS];
  if (pipe) {
    int c0 = 0;
    while (c0 <= D && !loaded(c0)) ++c0;
    if (c0 <= D) load_col(c0, pre);
  }
#pragma unroll
  for (int c = 0; c <= D; ++c) {
    // column c: from registers (a level's keys or the ids), else loaded
    const int kreg = kreg_of(c);
    u32* sb = stage + (pipe ? (c & 1) * CAP : 0);
    u32 v[ITEMS];
    if (c == D && IDS) {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) v[i] = ids[IDS ? i : 0];
    } else if (kreg >= 0 && c < D) {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        u32 x = 0;
#pragma unroll
        for (int k = 0; k < KC; ++k) x = k == kreg ? __float_as_uint(xs[k][i]) : x;
        v[i] = x;
      }
    } else if (pipe) {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) v[i] = pre[i];
      int cn = c + 1;
      while (cn <= D && !loaded(cn)) ++cn;
      if (cn <= D) load_col(cn, pre);
    } else {
      load_col(c, v);
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (path[i] < kMed) {
        sb[path[i] + u32(shift)] = v[i];  // stage index = column row - alo: 16-B groups align
      } else if (path[i] != kDead) {  // a tail median: straight to its output slot
        const int k = int(path[i] & 15u);
        const i64 slot = nlo[k] + nn[k] / 2;
        if (c < D) a.out_pts[slot * D + c] = __uint_as_float(v[i]);
        else a.out_ids[slot] = v[i];
      }
    }
    __syncthreads();
    const auto dr = col(a.dst, c);
    // 16-B stores of the aligned groups of 4 rows inside the segment (a quarter of the store
    // and LDS-read instructions of one word per lane); the <= 2 edge groups word by word (their
    // other words belong to neighbouring segments)
    using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
    const int ng = (n + shift + 3) >> 2;
#pragma unroll 2
    for (int q = tid; q < ng; q += T) {
      const int j0 = 4 * q;
      if (j0 >= shift && j0 + 3 < n + shift) {
        const u32x4 v4 = *reinterpret_cast<const u32x4*>(sb + j0);
        __builtin_amdgcn_raw_buffer_store_b128(v4, dr, u32(j0) * 4u, 0, 0);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = j0 + e;
          if (j >= shift && j < n + shift) __builtin_amdgcn_raw_buffer_store_b32(sb[j], dr, u32(j) * 4u, 0, 0);
        }
      }
    }
    // (pipe: the next column writes the other buffer; this one is rewritten two columns on,
    // after the next column's barrier, which every thread reaches only once its reads here are done)
    if (!pipe) __syncthreads();
    tail_stamp(a, 14 + c);
  }
}

size_t tail_lds_bytes(int items, bool pipe) {  // k_tail3's dynamic LDS (pipe: two stage buffers)
  return size_t(items) * kTailThreads * 4 * (pipe ? 2 : 1);
}

unsigned long long* tail_stamp_buffer() {  // PKD_TAIL_STAMPS=1 (diagnostic): allocated once, else null
  static unsigned long long* p = [] {
    unsigned long long* q = nullptr;
    if (std::getenv("PKD_TAIL_STAMPS")) {
      PKD_HIP_CHECK(hipMalloc(&q, size_t(kTailStampBlocks) * kTailStampSlots * 8));
      PKD_HIP_CHECK(hipMemset(q, 0, size_t(kTailStampBlocks) * kTailStampSlots * 8));
    }
    return q;
  }();
  return p;
}

// Calls f(std::integral_constant<int, dim + 1>) for dim <= 8 (rows in registers), else
// f(std::integral_constant<int, 0>) (runtime dim).
template <class F>
void with_ncol(int dim, F&& f) {
  switch (dim) {
    case 1: f(std::integral_constant<int, 2>{}); break;
    case 2: f(std::integral_constant<int, 3>{}); break;
    case 3: f(std::integral_constant<int, 4>{}); break;
    case 4: f(std::integral_constant<int, 5>{}); break;
    case 5: f(std::integral_constant<int, 6>{}); break;
    case 6: f(std::integral_constant<int, 7>{}); break;
    case 7: f(std::integral_constant<int, 8>{}); break;
    case 8: f(std::integral_constant<int, 9>{}); break;
    default: f(std::integral_constant<int, 0>{}); break;
  }
}

// Columns per load round of the runtime-dim partition: more bytes in flight per thread for
// wide rows (1M x 64D 2.67 -> 2.56 ms with 16, 500k x 128D 2.76 -> 2.62 ms with 32; 16D
// keeps 8).
int colgroup_for(int ncols, const Tuning& t) {
  if (t.colgroup > 0) return t.colgroup;
  return ncols >= 96 ? 32 : (ncols >= 48 ? 16 : 8);
}

size_t tiled_prep_lds(int dim) { return size_t(2 * dim) * 4 + size_t(dim) * (kPrepRows + 1) * 4; }

int pow2_floor(i64 v) {
  int p = 1;
  while (i64(p) * 2 <= v) p *= 2;
  return p;
}

int global_bins(i64 nmax) { return std::max(32, std::min(kMaxBins, pow2_floor(std::max<i64>(1, nmax / 24)))); }

}  // namespace

// ---------------------------------------------------------------------------------------
// Knob defaults, with their measurements:
// * hist_div 2: the first-level histogram's 4096-bin flush per block is its cost beyond the
//   key read; half the blocks: 100M x 3D k_hist 130 -> 115 us.
// * scan_div: the key sweeps run on ~1024 blocks at every size (half the partition grid from
//   64 M points, all of it below): their per-block histogram flush (2 x next_bins global atomics)
//   scales with blocks. 100 M x 3D: 9.12-9.18 ms vs 9.24 on 2048 blocks; 12.5 M: 1.427 vs 1.44 on
//   512 (profiles/r4_scan_grid_ab.txt). Round 2's reading at 100 M, on pairs:
//   the sweep stays bandwidth-bound (100M x 3D k_scan 1.57 -> 1.51 ms).
// * level_blocks: 4096 blocks from 40 M points, 2048 from 20 M, 1024 below (round 5, 50 M 4.85 ->
//   4.78 ms, 25 M 2.535 -> 2.51 ms, 12.5 M best at 1024: profiles/r5_level_blocks.txt); before: four rounds of 4 workgroups per CU for builds >= 64 M points (round 5, with
//   the sampled triples: 100 M x 3D 8.678 -> 8.641 ms against two rounds, 6144 and 8192 in
//   between, 16384 slower; 100 M x 8D 20.11 -> 19.79 ms, 1 B neutral: profiles/r5_level_blocks.txt),
//   one round below: at 12.5 M points (a
//   rank's share of 100 M on 8 GPUs) 1024 blocks build 7% faster than 2048, 1280 or 768
//   (profiles/r1_level_blocks_sweep.txt).
// * split: from level 2 (a pair boundary), 4 parts on 4 HIP streams for builds of >= 64 M
//   points (50 M: time-neutral, 25 M: +3%, 12.5 M: +7%; profiles/r2_split_build.txt).
const char* ab_knob(const char* name) {
  const char* v = std::getenv(name);
  if (v == nullptr) return nullptr;
  const char* ab = std::getenv("PKD_AB");  // read per call: knobs are read at builder construction only
  if (ab != nullptr && std::string(ab) == "1") return v;
  static std::mutex mu;
  static std::vector<std::string> noted;
  std::lock_guard<std::mutex> lk(mu);
  if (std::find(noted.begin(), noted.end(), name) == noted.end()) {
    noted.emplace_back(name);
    std::fprintf(stderr, "pkdtree: %s is an A/B knob, ignored without PKD_AB=1\n", name);
  }
  return nullptr;
}

Tuning Tuning::from_env() {
  auto env_i = [](const char* k, i64 d) -> i64 {  // public knobs
    const char* e = std::getenv(k);
    return e ? std::atoll(e) : d;
  };
  auto ab_i = [](const char* k, i64 d) -> i64 {  // A/B knobs
    const char* e = ab_knob(k);
    return e ? std::atoll(e) : d;
  };
  Tuning t;
  const char* impl = std::getenv("PKD_SUBTREE_IMPL");
  if (impl) throw std::invalid_argument("PKD_SUBTREE_IMPL was removed: one subtree kernel ships (k_subtree_rank)");
  t.split = env_i("PKD_SPLIT", 1) != 0;
  t.split_trace = std::getenv("PKD_SPLIT_TRACE") != nullptr;
  t.top = env_i("PKD_TOP", 1) != 0;
  t.implicit_ids = ab_i("PKD_IMPLICIT_IDS", 1) != 0;
  t.narrow = ab_i("PKD_NARROW", 1) != 0;
  t.pairs = ab_i("PKD_PAIR", 1) != 0;
  t.triples = ab_i("PKD_TRIPLE", 1) != 0;
  t.triple_from = int(ab_i("PKD_TRIPLE_FROM", 3));
  t.atomic_ranks = int(ab_i("PKD_PART_ATOMIC", -1));
  t.atomic_ranks3 = int(ab_i("PKD_PART3_ATOMIC", -1));
  t.prefix = ab_i("PKD_PART_PREFIX", 1) != 0;
  t.tail = ab_i("PKD_TAIL", 1) != 0;
  t.tail4 = ab_i("PKD_TAIL4", 1) != 0;
  t.tail4_min_dim = int(ab_i("PKD_TAIL4_MIN_DIM", t.tail4_min_dim));
  t.tail_pipe = ab_i("PKD_TAIL_PIPE", 1) != 0;
  t.g3_stage = int(ab_i("PKD_G3_STAGE", 2));
  t.part3_stage = ab_i("PKD_PART3_STAGE", 1) != 0;
  t.wide_ki = int(ab_i("PKD_WIDE_KI", t.wide_ki));
  t.xcd_map = ab_i("PKD_XCD_MAP", 1) != 0;
  t.colgroup = int(ab_i("PKD_COLGROUP", 0));
  t.hist_div = int(std::max<i64>(1, ab_i("PKD_HIST_DIV", 2)));
  t.scan_div = int(std::max<i64>(0, ab_i("PKD_SCAN_DIV", 0)));
  const int pb = int(ab_i("PKD_PAIR_BINS", kPairBins));
  t.pair_bins = (pb >= 64 && pb <= kPairBins && (pb & (pb - 1)) == 0) ? pb : kPairBins;
  t.level_blocks = std::max<i64>(0, ab_i("PKD_LEVEL_BLOCKS", 0));
  t.stage2_min = std::max<i64>(1, ab_i("PKD_STAGE2_MIN", kRefineCap));
  t.split_level = int(ab_i("PKD_SPLIT_LEVEL", 2));
  t.split_parts = int(ab_i("PKD_SPLIT_PARTS", 4));
  t.split_streams = int(ab_i("PKD_SPLIT_STREAMS", 4));
  t.split_min_n = ab_i("PKD_SPLIT_MIN_N", i64(64) << 20);
  t.split_min_n_3d = ab_i("PKD_SPLIT_MIN_N_3D", ab_knob("PKD_SPLIT_MIN_N") ? t.split_min_n : i64(512) << 20);
  t.top_min_n = ab_i("PKD_TOP_MIN_N", t.top_min_n);
  t.top_sample_log2 = int(ab_i("PKD_TOP_SAMPLE", t.top_sample_log2));
  if (const char* z = ab_knob("PKD_TOP_Z")) t.top_z = float(std::atof(z));
  t.top_blocks = int(ab_i("PKD_TOP_BLOCKS", 0));
  t.top_diag = int(ab_i("PKD_TOP_DIAG", 0));
  t.g3 = ab_i("PKD_G3", t.g3 ? 1 : 0) != 0;
  t.g3_min_segs = int(std::max<i64>(1, ab_i("PKD_G3_MIN_SEGS", t.g3_min_segs)));
  t.g3_min_rows = std::max<i64>(4096, ab_i("PKD_G3_MIN_ROWS", t.g3_min_rows));
  t.g3_sample = std::max<i64>(1024, ab_i("PKD_G3_SAMPLE", t.g3_sample));
  t.g3_div_min = int(std::max<i64>(1, ab_i("PKD_G3_DIV_MIN", t.g3_div_min)));
  t.g3_multi_below = std::max<i64>(1, ab_i("PKD_G3_MULTI_BELOW", t.g3_multi_below));
  t.g3_sample_blocks = std::max<i64>(1, ab_i("PKD_G3_SAMPLE_BLOCKS", t.g3_sample_blocks));
  t.g3_min_n = std::max<i64>(0, ab_i("PKD_G3_MIN_N", t.g3_min_n));
  t.tail_slim12 = ab_i("PKD_TAIL_SLIM12", t.tail_slim12);
  t.g3_max_dim = int(ab_i("PKD_G3_MAX_DIM", t.g3_max_dim));
  if (const char* z = ab_knob("PKD_G3_Z")) t.g3_z = float(std::atof(z));
  return t;
}

int default_subtree_max(int dim) { return subtree_capacity(dim); }

struct SplitStreams {
  std::mutex mu;
  int device = -1;
  std::vector<hipStream_t> side;  // streams 1..S-1 (stream 0 is the caller's)
  hipEvent_t fork = nullptr;
  std::vector<hipEvent_t> join;
  ~SplitStreams() {
    for (hipStream_t s : side) (void)hipStreamDestroy(s);
    for (hipEvent_t e : join) (void)hipEventDestroy(e);
    if (fork) (void)hipEventDestroy(fork);
  }
};

SplitStreams* GpuBuilder::split_streams_for(hipStream_t stream) const {
  if (!split_ || split_parts_ < 2) return nullptr;
  int dev = 0;
  PKD_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(split_->mu);
  if (split_->device == dev) return split_.get();
  if (split_->device >= 0) return nullptr;  // created for another device: build unsplit
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  PKD_HIP_CHECK(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone) return nullptr;  // no stream creation inside a capture
  for (int k = 1; k < split_streams_; ++k) {
    hipStream_t s = nullptr;
    PKD_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    split_->side.push_back(s);
    hipEvent_t e = nullptr;
    PKD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    split_->join.push_back(e);
  }
  PKD_HIP_CHECK(hipEventCreateWithFlags(&split_->fork, hipEventDisableTiming));
  split_->device = dev;
  return split_.get();
}

GpuBuilder::GpuBuilder(i64 n, int dim, BuildOptions opt)
    : n_(n), dim_(dim), opt_(opt), tune_(Tuning::from_env()) {

  if (dim <= 0) throw std::invalid_argument("pkdtree: dim must be > 0");
  if (n < 0 || n >= (i64(1) << 32)) throw std::invalid_argument("pkdtree: n must be in [0, 2^32)");
  nsub_ = opt.subtree_max > 0 ? std::min(opt.subtree_max, subtree_capacity_max(dim)) : subtree_capacity(dim);
  // High dims: narrow columns (the global levels move lg + 2 columns instead of dim + 1) and the
  // key-slot subtree kernel, whose LDS holds only its own levels' keys, so segments are larger
  if (dim > 8 && tiled_prep_lds(dim) <= size_t(96 * 1024) && tune_.narrow) {
    const int capn = subtree_capacity_narrow(dim);
    const int cap = opt.subtree_max > 0 ? std::min(opt.subtree_max, capn) : capn;
    int lg = 0;
    while (cap > 0 && (n_ >> lg) > cap) ++lg;
    if (cap > 0 && 2 * (lg + 2) < dim + 1) {
      narrow_ = true;
      nsub_ = cap;
    }
  }
  lg_ = 0;
  while ((n_ >> lg_) > nsub_) ++lg_;
  heap_nodes_ = (i64(1) << (lg_ + 1)) - 1;
  // Sampled top levels: full-column AoS builds large enough that one scatter pass plus the
  // sample and the band fix-up beat the paired levels 0..3 (level 4 must still be global).
  top_ = tune_.top && opt.allow_top && dim >= 2 && dim <= 8 && !narrow_ && n_ >= tune_.top_min_n && lg_ >= top4::kLevels + 1;
  max_bins_ = 0;
  max_hist_ = 1;
  const i64 level_blocks =
      tune_.level_blocks > 0 ? tune_.level_blocks
                             : (n_ >= 40000000 ? 2 * kLevelBlocks : (n_ >= 20000000 ? kLevelBlocks : kLevelBlocks / 2));
  scan_div_ = tune_.scan_div > 0 ? tune_.scan_div : int(std::max<i64>(1, level_blocks / (kLevelBlocks / 2)));
  // The level plan: with the sampled top (levels 0..3 by top4::run, pairing from level 4) for the
  // AoS / caller-column entry points, and without it for the entry points that start at level 0
  // (build_rows, build_from_soa, strided or row-id input): there levels 0..3 pair up as usual.
  i64 g3_segs = 0, g3_multi_segs = 0;
  // A triple from level l may be sampled (k_g3_*): rows in registers, a large build, many large
  // segments. Level l's own median bucket is taken from the fused histogram as is (a second stage
  // is skipped: its rows are the staged tag-0 rows, ranked exactly by k_g3_res<0>).
  auto g3_ok = [&](const LevelPlan& lp) {
    return tune_.g3 && opt.allow_top && !narrow_ && dim >= 2 && dim <= std::min(8, tune_.g3_max_dim) &&
           n_ >= tune_.g3_min_n && lp.segs >= tune_.g3_min_segs && lp.nmax >= tune_.g3_min_rows;
  };
  auto make_plan = [&](bool with_top) {
    std::vector<LevelPlan> lv;
    for (int l = 0; l < lg_; ++l) {
      LevelPlan lp;
      lp.level = l;
      lp.segs = i64(1) << l;
      lp.nmax = n_ >> l;
      lp.bins = global_bins(lp.nmax);
      lp.next_bins = (l + 1 < lg_) ? global_bins(n_ >> (l + 1)) : 0;
      // 2048 blocks per level (a whole number of rounds at 2 or 4 resident blocks per CU on
      // 256 CUs) while segments are few; one block per segment below that.
      // rows per block-chunk of the partition kernel used for this dim (runtime-dim rows are
      // wide, so their blocks take 1024-row chunks and more blocks share a segment)
      const i64 chunk = dim <= 8 ? i64(kChunk) : i64(kBlock) * 4;
      lp.bps = int(std::max<i64>(1, std::min<i64>(level_blocks / lp.segs, (lp.nmax + chunk - 1) / chunk)));
      lp.axis = (opt.depth0 + l) % dim;
      // expected middle zone nmax / bins larger than the LDS refine: split the median bucket
      lp.stage2 = lp.nmax / lp.bins > tune_.stage2_min;
      if (lp.stage2) max_hist2_ = std::max<i64>(max_hist2_, lp.segs * kBins2);
      lv.push_back(lp);
      max_bins_ = std::max(max_bins_, lp.bins);
      max_hist_ = std::max<i64>(max_hist_, lp.segs * lp.bins);
    }
    // Levels l, l+1, l+2 move in ONE fused scatter pass (a triple) when rows fit the register
    // path and neither l+1 nor l+2 needs a second-stage histogram (their median buckets are
    // narrowed by the two key sweeps k_scan / k_scan2 and k_refine alone); otherwise l and l+1
    // pair up. A triple never straddles the split level of a split build.
    const bool pairs = dim <= 8 && tune_.pairs;
    const bool may_split = tune_.split && opt.allow_split && n_ >= tune_.split_min(dim);
    auto cap_bins = [&](int l, int cap) {  // level l's bins, fused into the previous pass's LDS
      if (l >= lg_) return;
      LevelPlan& g = lv[size_t(l)];
      g.bins = std::min(g.bins, cap);
      lv[size_t(l - 1)].next_bins = g.bins;
    };
    // The last three global levels: one workgroup per segment (k_tail3) when a segment fits its
    // 1024 threads x 8 / 12 / 16 rows (always, below the subtree capacity of 2048) and rows fit
    // registers (dim <= 8, full columns).
    // (A split build's parts start at split_level: the tail may not begin above it.)
    const bool may_split0 = tune_.split && opt.allow_split && n_ >= tune_.split_min(dim);
    if (tune_.tail && pairs && !narrow_ && lg_ >= 5 && (!may_split0 || lg_ - tail_lev_ >= tune_.split_level)) {
      const i64 nl = (n_ >> (lg_ - tail_lev_)) + 3;  // + the 16-B alignment shift of the segment start
      tail_items_ = nl <= 8 * 1024 ? 8 : (nl <= 12 * 1024 ? 12 : (nl <= 16 * 1024 ? 16 : 0));
      if (tail_items_ > 0) {
        tail_ = lg_ - tail_lev_;
        for (int l = tail_; l < lg_; ++l) lv[size_t(l)].tail = true;
      }
    }
    const int lgrp = tail_ >= 0 ? tail_ : lg_;  // levels the pairs / triples cover
    const int lfirst = with_top ? top4::kLevels : 0;
    if (with_top)
      for (int l = 0; l < top4::kLevels; ++l) lv[size_t(l)].sampled = true;
    for (int l = lfirst; pairs && l + 1 < lgrp;) {
      // (four levels left: two pairs, not a triple and a lone level, whose single-level pass moves
      // every row for one level: 100M x 8D level 13 alone took 1.7 ms)
      // (a sampled triple needs no histogram of levels l+1, l+2, so their second stages do not matter)
      const bool tri = tune_.triples && l >= tune_.triple_from && l + 2 < lgrp && lgrp - l != 4 &&
                       ((!lv[size_t(l + 1)].stage2 && !lv[size_t(l + 2)].stage2) || g3_ok(lv[size_t(l)]));
      int next = l + (tri ? 3 : 2);
      if (may_split && l < tune_.split_level && tune_.split_level < next) next = tune_.split_level;  // a pass ends there
      if (next - l == 3) {
        lv[size_t(l)].triple = true;
        cap_bins(l + 2, tune_.pair_bins);   // k_scan2: 4 grandchild histograms in LDS
        cap_bins(l + 3, kTripleBins);       // k_partition3: 8 great-grandchild histograms in LDS
      } else if (next - l == 2) {
        lv[size_t(l)].pair = true;
        cap_bins(l + 2, tune_.pair_bins);   // the pair's scatter fuses 4 grandchild histograms in LDS
      }
      l = next;
    }
    if (tail_ > 0) lv[size_t(tail_ - 1)].next_bins = 0;  // k_tail3 bins its levels itself
    // Sampled triples: full-column rows in registers, segments many and large enough (the fix-up
    // kernels run one workgroup per node; the staging regions must fit a segment), and level l's
    // median bucket exact from the fused histogram alone (no second stage).
    for (int l = 0; l < lg_; ++l) {
      LevelPlan& lp = lv[size_t(l)];
      if (!(lp.triple && g3_ok(lp))) continue;
      lp.g3 = true;
      // sample rows per segment: g3_sample, or 1 / 24 of a larger segment (the staged fraction falls
      // as 1 / sqrt(sample) while the sample's own reads grow linearly)
      const i64 want = std::max<i64>(tune_.g3_sample, lp.nmax / 24);
      lp.g3_div = int(std::max<i64>(tune_.g3_div_min, lp.nmax / want));
      const i64 windows = std::max<i64>(1, lp.nmax / (64 * i64(lp.g3_div)));
      lp.g3_sblocks = int(std::max<i64>(1, std::min<i64>(tune_.g3_sample_blocks / lp.segs, windows / 64)));
      if (lp.segs < tune_.g3_multi_below) {  // few nodes: K blocks each for the resolve of levels l+1, l+2
        lp.g3_k1 = int(std::max<i64>(2, 1024 / (2 * lp.segs)));
        lp.g3_k2 = int(std::max<i64>(2, 1024 / (4 * lp.segs)));
        g3_multi_segs = std::max(g3_multi_segs, lp.segs);
      }
      g3_ = true;
      g3_segs = std::max(g3_segs, lp.segs);
    }
    return lv;
  };
  // A 4-level tail where it leaves one row-moving pass fewer between the top and the tail (100 M x
  // 8D: 17 levels = 4 sampled + 3 triples + 4, instead of 4 + 2 triples + 2 pairs + 3): both plans
  // are laid out and their passes counted. Rows of 5..9 columns (the 4-level kernel keeps two key
  // register sets), segments of <= 16 Ki rows at its first level.
  auto passes = [&](const std::vector<LevelPlan>& lv) {
    int c = 0;
    const int lend = tail_ >= 0 ? tail_ : lg_;
    for (int l = 0; l < lend; ++c) l += lv[size_t(l)].sampled ? top4::kLevels : (lv[size_t(l)].triple ? 3 : (lv[size_t(l)].pair ? 2 : 1));
    return c;
  };
  if (tune_.tail4 && tune_.tail && dim >= tune_.tail4_min_dim && dim >= 3 && dim <= 8 && !narrow_ && lg_ >= 9 &&
      (n_ >> (lg_ - 4)) + 3 <= 16 * 1024) {
    tail_lev_ = 3;
    const int p3 = passes(make_plan(top_));
    const bool had3 = tail_ >= 0;
    tail_ = -1;
    tail_lev_ = 4;
    const int p4 = passes(make_plan(top_));
    if (!(had3 && tail_ >= 0 && p4 < p3)) tail_lev_ = 3;
    tail_ = -1;
    tail_items_ = 0;
    g3_ = false;
    g3_segs = g3_multi_segs = 0;
  }
  levels_ = make_plan(top_);
  if (top_) levels_nt_ = make_plan(false);
  for (const auto* plan : {&levels_, &levels_nt_})
    for (const LevelPlan& lp : *plan) {
      max_bins_ = std::max(max_bins_, lp.bins);
      max_hist_ = std::max<i64>(max_hist_, lp.segs * lp.bins);
    }
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + std::max<size_t>(bytes, 1));
    return o;
  };
  ncol_ = std::max<i64>(64, (n + 63) / 64 * 64);  // 256-B aligned columns (vector stores)
  const size_t colbytes = size_t(dim + 1) * size_t(ncol_) * 4;
  off_cols_a_ = take(colbytes);
  off_cols_b_ = take(colbytes);
  off_seg_lo_ = take(size_t(heap_nodes_) * 8);
  off_seg_n_ = take(size_t(heap_nodes_) * 8);
  off_state_ = take(size_t(heap_nodes_) * sizeof(SegState));
  off_params_ = take(size_t(heap_nodes_) * sizeof(BucketParams));
  off_cells_ = take(size_t(heap_nodes_) * size_t(2 * dim) * 4);
  off_hist0_ = take(size_t(max_hist_) * 4);
  off_hist1_ = take(size_t(max_hist_) * 4);
  off_hist2_ = take(size_t(std::max<i64>(max_hist2_, 1)) * 4);
  off_bbox_ = take(size_t(2 * dim) * 4 * (1 + kMaxBoxParts));  // final box + per-block partials
  off_err_ = take(16);
  i64 max_grid = 1;
  for (const auto* plan : {&levels_, &levels_nt_})
    for (const LevelPlan& lp : *plan) max_grid = std::max<i64>(max_grid, lp.segs * lp.bps);
  off_bcnt_ = take(size_t(max_grid) * 4 * 4 * 2);  // per-block counts + bases (prefix placement)
  if (top_) off_top_ = take(top4::workspace_bytes());
  if (g3_) {
    off_stage_ = take(colbytes);
    off_g3_ = take(size_t(g3_segs) * sizeof(G3Seg));
    off_g3_hist_ = take(size_t(g3_segs) * 6 * kG3Bins * 4);
    if (g3_multi_segs > 0) {
      off_g3_nodes_ = take(size_t(g3_multi_segs) * 6 * sizeof(G3Node));
      off_g3_mhist_ = take(size_t(g3_multi_segs) * 6 * kG3ResBins * 4);
      off_g3_cand_ = take(size_t(g3_multi_segs) * 6 * kG3MCand * 8);
    }
  }
  {
    const Tuning& sc = tune_;
    const int L = sc.split_level;
    const bool paired = lg_ >= 2 && (levels_[0].pair || levels_[0].triple);
    bool boundary = false;  // L starts a pass (single level, pair or triple)
    for (int l = 0; l < lg_;) {
      boundary = boundary || l == L;
      l += levels_[size_t(l)].triple ? 3 : (levels_[size_t(l)].pair ? 2 : 1);
    }
    if (sc.split && opt.allow_split && paired && !narrow_ && dim <= 8 && n_ >= sc.split_min(dim) && L >= 2 && boundary &&
        L < lg_ && sc.split_parts >= 2 && sc.split_streams >= 1) {
      const int P = std::min(pow2_floor(sc.split_parts), 1 << L);
      split_level_ = L;
      split_parts_ = P;
      split_streams_ = std::max(1, std::min(sc.split_streams, P));
      size_t hw = 1, h2w = 1, bw = 1;
      for (int l = L; l < lg_; ++l) {  // the part's share of every per-segment array
        const LevelPlan& lp = levels_[size_t(l)];
        const i64 sp = lp.segs / P;
        if (l > L) hw = std::max(hw, size_t(sp) * size_t(lp.bins));
        if (lp.stage2) h2w = std::max(h2w, size_t(sp) * size_t(kBins2));
        const i64 chunk = i64(kChunk);
        const i64 pb = std::max<i64>(1, std::min<i64>(i64(lp.bps) * P / std::max(1, std::min(sc.split_streams, P)),
                                                      (lp.nmax + chunk - 1) / chunk));
        bw = std::max(bw, size_t(sp) * size_t(std::max<i64>(pb, lp.bps)) * 8);
      }
      split_hist_ = hw;
      split_hist2_ = h2w;
      split_bcnt_ = bw;
      split_set_bytes_ = align_up(2 * hw * 4) + align_up(h2w * 4) + align_up(bw * 4);
      off_split_ = take(split_set_bytes_ * size_t(split_streams_));
      split_ = std::make_shared<SplitStreams>();
    }
  }
  ws_bytes_ = off;
}

std::string GpuBuilder::describe() const {
  std::ostringstream os;
  os << "GpuBuilder(n=" << n_ << ", dim=" << dim_ << ", global_levels=" << lg_ << ", subtree_max=" << nsub_
     << ", workspace=" << ws_bytes_ << "B";
  if (split_parts_ > 1)
    os << ", split at level " << split_level_ << " into " << split_parts_ << " parts on " << split_streams_ << " streams";
  os << ")";
  for (const auto& lp : levels_)
    os << "\n  L" << lp.level << " segs=" << lp.segs << " nmax=" << lp.nmax << " bins=" << lp.bins
       << " next_bins=" << lp.next_bins << " bps=" << lp.bps << " axis=" << lp.axis << (lp.stage2 ? " stage2" : "")
       << (lp.pair ? " pair" : "") << (lp.triple ? " triple" : "") << (lp.tail ? " tail" : "")
       << (lp.sampled ? " sampled" : "") << (lp.g3 ? " g3" : "");
  return os.str();
}

namespace {
// acc[0] |= err[0]; acc[1] += builds with any error bit; acc[2] += builds with the miss bit
// (one thread: stream-ordered after the build, no host round trip).
__global__ void k_accumulate_error(const u32* __restrict__ err, u32* __restrict__ acc) {
  if (threadIdx.x != 0) return;
  const u32 e = err[0];
  acc[0] |= e;
  acc[1] += e != 0u ? 1u : 0u;
  acc[2] += (e & top4::kErrBit) ? 1u : 0u;
}
}  // namespace

void GpuBuilder::accumulate_error(const void* workspace, u32* acc, hipStream_t stream) const {
  k_accumulate_error<<<1, 64, 0, stream>>>(error_word(workspace), acc);
  PKD_LAUNCH_CHECK();
}

u32 GpuBuilder::read_error(const void* workspace, hipStream_t stream, u32* detail) const {
  u32 e[4] = {0, 0, 0, 0};
  PKD_HIP_CHECK(hipMemcpyAsync(e, static_cast<const char*>(workspace) + off_err_, 16, hipMemcpyDeviceToHost, stream));
  PKD_HIP_CHECK(hipStreamSynchronize(stream));
  if (detail) {
    detail[0] = e[1];
    detail[1] = e[2];
    detail[2] = e[3];
  }
  return e[0];
}

std::vector<u32> GpuBuilder::g3_report(const void* workspace, hipStream_t stream) const {
  std::vector<u32> out;
  int last = -1;
  for (const auto& lp : levels_)
    if (lp.g3) last = lp.level;
  if (last < 0 || n_ == 0) return out;
  const i64 segs = levels_[size_t(last)].segs;
  std::vector<G3Seg> g(static_cast<size_t>(segs));
  std::vector<i64> sn(static_cast<size_t>(segs));
  const char* ws = static_cast<const char*>(workspace);
  PKD_HIP_CHECK(hipMemcpyAsync(g.data(), ws + off_g3_, size_t(segs) * sizeof(G3Seg), hipMemcpyDeviceToHost, stream));
  PKD_HIP_CHECK(hipMemcpyAsync(sn.data(), ws + off_seg_n_ + size_t(segs - 1) * 8, size_t(segs) * 8,
                               hipMemcpyDeviceToHost, stream));
  PKD_HIP_CHECK(hipStreamSynchronize(stream));
  out.push_back(u32(last));
  for (i64 s = 0; s < segs; ++s) {
    const G3Seg& q = g[size_t(s)];
    out.push_back(u32(sn[size_t(s)]));
    for (int t = 0; t < 7; ++t) out.push_back(q.zc[8 + t][0]);
    for (int z = 0; z < 8; ++z) out.push_back(q.zc[z][0]);
    for (int z = 0; z < 8; ++z) out.push_back(q.ins[z]);
    out.push_back(q.bad);
  }
  return out;
}

float* GpuBuilder::soa_input(void* workspace) const {
  return reinterpret_cast<float*>(static_cast<char*>(workspace) + off_cols_a_);
}

void GpuBuilder::build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids,
                       void* workspace, hipStream_t stream) const {
  prep_and_run(pts, dim_, false, ids, id_base, out_pts, out_ids, workspace, stream);
}

void GpuBuilder::build_rows(const float* rows, float* out_pts, u32* out_ids, void* workspace,
                            hipStream_t stream) const {
  prep_and_run(rows, dim_ + 1, true, nullptr, 0, out_pts, out_ids, workspace, stream);
}

void GpuBuilder::prep_and_run(const float* pts, int rs, bool ids_in_row, const u32* ids, u32 id_base,
                              float* out_pts, u32* out_ids, void* workspace, hipStream_t stream) const {
  if (n_ == 0) return;
  TraceRange tr("pkd.build");
  char* ws = static_cast<char*>(workspace);
  float* colsA = reinterpret_cast<float*>(ws + off_cols_a_);
  u32* bbox = reinterpret_cast<u32*>(ws + off_bbox_);
  u32* part = bbox + 2 * dim_;
  const bool tiled = dim_ > 8 && tiled_prep_lds(dim_) <= size_t(96 * 1024);  // LDS transpose tiles
  const int grid = tiled ? int(std::min<i64>(kMaxBoxParts, std::max<i64>(1, (n_ + kPrepRows - 1) / kPrepRows)))
                         : int(std::min<i64>(kMaxBoxParts, std::max<i64>(1, (n_ + kBlock - 1) / kBlock)));
  const size_t lds = tiled ? tiled_prep_lds(dim_) : size_t(2 * dim_) * 4;
  if (tiled) {
    ensure_dynamic_lds(reinterpret_cast<const void*>(&k_prep_tiled), 96 * 1024);
  }
  // High-dim AoS input: only the global levels' keys, the ids and the input row index travel
  // through the global levels (lg_ + 2 columns instead of dim + 1); the subtree kernel and the
  // median writes gather whole rows from the input, which outlives the build.
  const bool narrow = narrow_ && tiled;
  if (top_ && !ids_in_row && rs == dim_) {  // levels 0..3 straight from the AoS input (no prep pass)
    run_top(pts, nullptr, ids, id_base, out_pts, out_ids, ws, stream);
    return;
  }
  const bool vec3 = dim_ == 3 && !ids_in_row && rs == 3 && (reinterpret_cast<uintptr_t>(pts) % 16 == 0) &&
                    (ids == nullptr || reinterpret_cast<uintptr_t>(ids) % 16 == 0);
  if (vec3) {
    const int g = int(std::min<i64>(2048, std::max<i64>(1, (n_ / 16 + kBlock - 1) / kBlock)));
    // generated ids are synthesised by the first pair's kernels instead of written here
    // (-4 B written and -4 B read per point); the first level must be a pair for that
    const std::vector<LevelPlan>& plan0 = top_ ? levels_nt_ : levels_;  // (this entry starts at level 0)
    const bool implicit = ids == nullptr && lg_ >= 2 && (plan0[0].pair || plan0[0].triple) && tune_.implicit_ids;
    k_prep3v<<<g, kBlock, 0, stream>>>(pts, ids, id_base, colsA, n_, ncol_, part, implicit ? 0 : 1);
    PKD_LAUNCH_CHECK();
    k_bbox_reduce<<<2 * dim_, kBlock, 0, stream>>>(part, g, dim_, bbox);
    PKD_LAUNCH_CHECK();
    run_levels(out_pts, out_ids, ws, stream, implicit, id_base);
    return;
  }
  switch (dim_) {
    case 1: k_prep<1><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    case 2: k_prep<2><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    case 3: k_prep<3><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    case 4: k_prep<4><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    case 5: k_prep<5><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    case 6: k_prep<6><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    case 7: k_prep<7><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    case 8: k_prep<8><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_); break;
    default:
      if (tiled)
        k_prep_tiled<<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0,
                                                    ncol_, narrow ? 1 : 0, lg_, opt_.depth0);
      else k_prep<0><<<grid, kBlock, lds, stream>>>(pts, ids, id_base, colsA, n_, dim_, part, rs, ids_in_row ? 1 : 0, ncol_);
      break;
  }
  PKD_LAUNCH_CHECK();
  k_bbox_reduce<<<2 * dim_, kBlock, 0, stream>>>(part, grid, dim_, bbox);
  PKD_LAUNCH_CHECK();
  run_levels(out_pts, out_ids, ws, stream, false, 0, narrow ? pts : nullptr, rs);
}

// Levels 0..3 by the sampled top pass (top4.hpp), then the remaining levels from level 4: from
// the AoS input (pts) or from SoA columns (in_cols: dim coordinate columns + the id column,
// stride ncol_, not the workspace's own columns), no prep or bounding-box pass either way.
void GpuBuilder::run_top(const float* pts, const float* in_cols, const u32* ids, u32 id_base, float* out_pts,
                         u32* out_ids, char* ws, hipStream_t stream) const {
  float* colsA = reinterpret_cast<float*>(ws + off_cols_a_);
  u32* err = reinterpret_cast<u32*>(ws + off_err_);
  zero_u32(err, 4, stream);
  top4::Geom g{};
  for (int h = 0; h < top4::kHeap; ++h) {  // the heap geometry of k_geometry, levels 0..4
    int l = 0;
    while (((h + 1) >> (l + 1)) > 0) ++l;
    const i64 j = h + 1 - (i64(1) << l);
    i64 lo = 0, m = n_;
    for (int b = l - 1; b >= 0; --b) {
      if ((j >> b) & 1) {
        lo = lo + m / 2 + 1;
        m = m - m / 2 - 1;
      } else {
        m = m / 2;
      }
      if (m < 0) m = 0;
    }
    g.lo[h] = lo;
    g.n[h] = m;
  }
  for (int l = 0; l <= top4::kLevels; ++l) g.axis[l] = (opt_.depth0 + l) % dim_;
  g.dim = dim_;
  top4::IO io{};
  io.pts = pts;
  io.in_cols = in_cols;
  io.in_ncol = ncol_;
  io.ids = ids;
  io.id_base = id_base;
  io.n = n_;
  io.cols = colsA;
  io.stage = reinterpret_cast<float*>(ws + off_cols_b_);
  io.ncol = ncol_;
  io.out_pts = out_pts;
  io.out_ids = out_ids;
  io.cells = reinterpret_cast<float*>(ws + off_cells_);
  io.params = reinterpret_cast<BucketParams*>(ws + off_params_);
  io.bins4 = levels_[size_t(top4::kLevels)].bins;
  io.err = err;
  io.ws = ws + off_top_;
  top4::Tune tt;
  tt.sample_log2 = tune_.top_sample_log2;
  tt.z = tune_.top_z;
  tt.scatter_blocks = tune_.top_blocks;
  tt.diag = tune_.top_diag;
  tt.salt = top_salt_++;
  {
    TraceRange trt("pkd.top4");
    top4::run(g, io, tt, stream);
  }
  if (tt.diag) return;  // timing diagnostic: no tree
  run_levels(out_pts, out_ids, ws, stream, false, 0, nullptr, 0, nullptr, top4::kLevels);
}

void GpuBuilder::build_from_soa(float* out_pts, u32* out_ids, void* workspace, hipStream_t stream) const {
  if (n_ == 0) return;
  if (narrow_) throw std::runtime_error("pkdtree: build_from_soa needs the full-column layout (set PKD_NARROW=0)");
  TraceRange tr("pkd.build");
  char* ws = static_cast<char*>(workspace);
  float* colsA = reinterpret_cast<float*>(ws + off_cols_a_);
  u32* bbox = reinterpret_cast<u32*>(ws + off_bbox_);
  u32* part = bbox + 2 * dim_;
  const int grid = int(std::min<i64>(2048, std::max<i64>(1, (n_ + kBlock - 1) / kBlock)));
  k_bbox_soa<<<grid, kBlock, 0, stream>>>(colsA, n_, dim_, part, ncol_);
  PKD_LAUNCH_CHECK();
  k_bbox_reduce<<<2 * dim_, kBlock, 0, stream>>>(part, grid, dim_, bbox);
  PKD_LAUNCH_CHECK();
  run_levels(out_pts, out_ids, ws, stream);
}

void GpuBuilder::build_columns(float* cols, float* out_pts, u32* out_ids, void* workspace, hipStream_t stream,
                               const float* root_cell) const {
  if (n_ == 0) return;
  if (narrow_) throw std::runtime_error("pkdtree: build_columns needs the full-column layout (dim <= 8)");
  if (reinterpret_cast<uintptr_t>(cols) % 256 != 0) throw std::invalid_argument("pkdtree: columns must be 256-B aligned");
  TraceRange tr("pkd.build");
  char* ws = static_cast<char*>(workspace);
  if (top_ && cols != reinterpret_cast<float*>(ws + off_cols_a_)) {  // sampled top levels from the columns
    run_top(nullptr, cols, nullptr, 0, out_pts, out_ids, ws, stream);
    return;
  }
  if (g3_ && !top_ && cols != reinterpret_cast<float*>(ws + off_cols_a_)) {
    // a sampled triple may miss (error bit top4_band_miss_bit()): its rebuild reads the caller's
    // columns again, so the levels run on a copy instead of clobbering them
    PKD_HIP_CHECK(hipMemcpyAsync(ws + off_cols_a_, cols, size_t(dim_ + 1) * size_t(ncol_) * 4, hipMemcpyDeviceToDevice,
                                 stream));
    cols = reinterpret_cast<float*>(ws + off_cols_a_);
  }
  if (root_cell) {  // the caller's box of the points: no bounding-box pass over the columns
    k_cell_root<<<1, 64, 0, stream>>>(root_cell, dim_, reinterpret_cast<float*>(ws + off_cells_),
                                      reinterpret_cast<BucketParams*>(ws + off_params_), opt_.depth0 % dim_,
                                      lg_ > 0 ? (top_ ? levels_nt_ : levels_)[0].bins : 1);
    PKD_LAUNCH_CHECK();
    run_levels(out_pts, out_ids, ws, stream, false, 0, nullptr, 0, cols, 0, true);
    return;
  }
  u32* bbox = reinterpret_cast<u32*>(ws + off_bbox_);
  u32* part = bbox + 2 * dim_;
  const int grid = int(std::min<i64>(2048, std::max<i64>(1, (n_ + kBlock - 1) / kBlock)));
  k_bbox_soa<<<grid, kBlock, 0, stream>>>(cols, n_, dim_, part, ncol_);
  PKD_LAUNCH_CHECK();
  k_bbox_reduce<<<2 * dim_, kBlock, 0, stream>>>(part, grid, dim_, bbox);
  PKD_LAUNCH_CHECK();
  run_levels(out_pts, out_ids, ws, stream, false, 0, nullptr, 0, cols);
}

void GpuBuilder::run_levels(float* out_pts, u32* out_ids, char* ws, hipStream_t stream, bool implicit_ids,
                            u32 id_base, const float* in_rows, i64 in_rs, float* cols_a, int first_level,
                            bool root_ready) const {
  const int narrow_k = in_rows ? lg_ : 0;  // key columns of the narrow layout
  const u32 g3_salt = g3_ ? g3_salt_++ : 0u;  // this build's sample positions (sampled triples)
  // levels 0..3 already built by the sampled top, or the plan that pairs them from level 0
  const std::vector<LevelPlan>& levels = (top_ && first_level == 0) ? levels_nt_ : levels_;
  float* colsA = cols_a ? cols_a : reinterpret_cast<float*>(ws + off_cols_a_);
  float* colsB = reinterpret_cast<float*>(ws + off_cols_b_);
  i64* seg_lo = reinterpret_cast<i64*>(ws + off_seg_lo_);
  i64* seg_n = reinterpret_cast<i64*>(ws + off_seg_n_);
  SegState* state = reinterpret_cast<SegState*>(ws + off_state_);
  BucketParams* params = reinterpret_cast<BucketParams*>(ws + off_params_);
  float* cells = reinterpret_cast<float*>(ws + off_cells_);
  u32* hist[2] = {reinterpret_cast<u32*>(ws + off_hist0_), reinterpret_cast<u32*>(ws + off_hist1_)};
  u32* bbox = reinterpret_cast<u32*>(ws + off_bbox_);
  u32* err = reinterpret_cast<u32*>(ws + off_err_);
  if (first_level == 0) zero_u32(err, 4, stream);

  k_geometry<<<int((heap_nodes_ + kBlock - 1) / kBlock), kBlock, 0, stream>>>(seg_lo, seg_n, heap_nodes_, n_);
  PKD_LAUNCH_CHECK();
  const int axis0 = opt_.depth0 % dim_;
  if (first_level == 0 && !root_ready) {
    k_root<<<1, 64, 0, stream>>>(bbox, dim_, cells, params, axis0, lg_ > 0 ? levels[0].bins : 1);
    PKD_LAUNCH_CHECK();
  }

  // Levels [l0, l1) of segment range `part` of `nparts` (at level l: segments
  // [part * segs / nparts, (part + 1) * segs / nparts)) on stream `st`. The per-segment arrays
  // indexed by the level-relative segment (histograms, stage-2 histograms, block counts) come
  // from `hs`; only level l0 > 0 reads its histogram from the shared arrays, where the
  // previous (unsplit) pass wrote it.
  struct HistSet {
    u32* h[2];
    u32* h2;
    u32* bcnt;
  };
  // Zone ranks of the scatter passes: LDS atomics below 64 M points, wave ballots above
  // (A/B in profiles/r3_partition_subtree_experiments.txt); knob -1 = by size.
  auto atomic_ranks = [&](int knob) { return knob >= 0 ? knob != 0 : n_ < (i64(64) << 20); };
  // triples: wave ballots + LDS-staged stores from 10 M points at rows of <= 5 columns (3-D
  // 12.5 M 1.415 -> 1.387 ms, 50 M 4.74 -> 4.41; 2 M - 8 M 1-2 % slower), else from 64 M (8-D
  // 5 M - 30 M are 2-4 % slower with ballots); profiles/r6_ballot_sizes.txt
  auto atomic_ranks3 = [&](int knob) {
    return knob >= 0 ? knob != 0 : n_ < (dim_ <= 4 ? i64(10) << 20 : i64(64) << 20);
  };
  auto run_range = [&](int base, int l0, int l1, int part, int nparts, hipStream_t st, const HistSet& hs,
                       float*& src, float*& dst) {
    auto hist_of = [&](int l) -> u32* {  // `base`: the level where the part's own arrays start
      if (base > 0 && l == base)
        return hist[l & 1] + size_t(part) * size_t(levels[size_t(l)].segs / nparts) * size_t(levels[size_t(l)].bins);
      return hs.h[(l - base) & 1];
    };
    // A part's kernels run next to split_streams_ - 1 others: its blocks per segment scale by
    // parts / streams so the concurrent grids together match the unsplit level's grid.
    auto bps_of = [&](int l) -> int {
      const LevelPlan& lp = levels[size_t(l)];
      if (nparts == 1) return lp.bps;
      const i64 chunk = dim_ <= 8 ? i64(kChunk) : i64(kBlock) * 4;
      const i64 want = i64(lp.bps) * nparts / std::max(1, split_streams_);
      return int(std::max<i64>(1, std::min<i64>(want, (lp.nmax + chunk - 1) / chunk)));
    };
    auto level_args = [&](int l) {
      const LevelPlan& lp = levels[size_t(l)];
      LevelArgs a;
      a.src = src;
      a.dst = dst;
      a.ncol = ncol_;
      a.dim = dim_;
      a.seg_lo = seg_lo;
      a.seg_n = seg_n;
      a.state = state;
      a.params = params;
      a.cells = cells;
      a.heap0 = lp.segs - 1 + i64(part) * (lp.segs / nparts);
      a.bps = bps_of(l);
      a.axis = lp.axis;
      a.next_axis = (opt_.depth0 + l + 1) % dim_;
      a.bins = lp.bins;
      a.next_bins = lp.next_bins;
      a.hist = hist_of(l);
      a.hist_next = l + 1 < lg_ ? hist_of(l + 1) : nullptr;
      a.out_pts = out_pts;
      a.out_ids = out_ids;
      a.err = err;
      a.block_reserve = (lp.segs <= 8 && lp.bps > 4) ? 1 : 0;  // only where cursor contention is high
      a.small_done = 0;
      a.hist2 = hs.h2;
      a.id_implicit = (implicit_ids && l == 0) ? 1 : 0;
      a.xcd = tune_.xcd_map ? 1 : 0;
      a.narrow = in_rows ? 1 : 0;
      a.kcol = a.narrow ? l : a.axis;
      a.nkcol = a.narrow ? std::min(l + 1, narrow_k) : a.next_axis;
      a.idcol = a.narrow ? narrow_k : dim_;
      a.ncols = a.narrow ? narrow_k + 2 : dim_ + 1;
      a.colgroup = colgroup_for(a.ncols - 1, tune_);
      a.in_rows = in_rows;
      a.in_rs = in_rs;
      a.id_base0 = id_base;
      return a;
    };
    auto refine = [&](LevelArgs& a, i64 segs) {
      a.small_done = dim_ <= 8 ? 1 : 0;
      if (a.small_done) {
        const int g = int((segs + 3) / 4);
        with_ncol(dim_, [&](auto nc) {
          constexpr int NC = decltype(nc)::value > 0 ? decltype(nc)::value : 9;
          k_refine_both<NC, kRefineCap><<<g + int(segs), kBlock, size_t(kRefineCap) * 12, st>>>(a, segs, g);
        });
      } else {
        k_refine<kRefineCap><<<int(segs), kBlock, size_t(kRefineCap) * 12, st>>>(a);
      }
      PKD_LAUNCH_CHECK();
    };
    static const char* const kLevelNames[] = {"pkd.level0", "pkd.level1", "pkd.level2", "pkd.level3",
                                              "pkd.level4", "pkd.level5", "pkd.level6", "pkd.level7",
                                              "pkd.level8", "pkd.level9", "pkd.level10", "pkd.level11+"};
    const int lend = tail_ >= 0 ? std::min(l1, tail_) : l1;
    for (int l = l0; l < lend;) {
      const LevelPlan& lp = levels[size_t(l)];
      const i64 segs = lp.segs / nparts;  // this part's segments at level l
      TraceRange trl(kLevelNames[std::min(l, 11)]);  // a pair's range carries its first level
      LevelArgs a = level_args(l);
      if (l == first_level) {  // no previous pass fused this level's histogram
        zero_u32(hist[l & 1], lp.segs * lp.bins, st);
        LevelArgs ah = a;  // like k_scan: fewer blocks, fewer histogram flush atomics
        ah.bps = std::max(1, a.bps / tune_.hist_div);
        k_hist<<<int(lp.segs * ah.bps), kBlock, size_t(lp.bins) * 4, st>>>(ah, hist[l & 1]);
        PKD_LAUNCH_CHECK();
      }
      k_select<<<int(segs), kBlock, 0, st>>>(a);
      PKD_LAUNCH_CHECK();
      if (lp.stage2 && !lp.g3) {
        zero_u32(a.hist2, segs * kBins2, st);
        k_hist2<<<int(segs * a.bps), kBlock, 0, st>>>(a);
        PKD_LAUNCH_CHECK();
        k_select2<<<int(segs), kBlock, 0, st>>>(a);
        PKD_LAUNCH_CHECK();
      }
      const int grid = int(segs * a.bps);
      if (lp.g3) {
        const LevelPlan& lr = levels[size_t(l + 2)];
        G3Args ga;
        ga.g3 = reinterpret_cast<G3Seg*>(ws + off_g3_);
        ga.shist = reinterpret_cast<u32*>(ws + off_g3_hist_);
        ga.stage = reinterpret_cast<float*>(ws + off_stage_);
        ga.seg0 = i64(part) * segs;
        ga.axis2 = lr.axis;
        ga.axis3 = (opt_.depth0 + l + 3) % dim_;
        ga.bins3 = lr.next_bins;
        ga.hist3 = l + 3 < lg_ ? hist_of(l + 3) : nullptr;
        ga.sample_div = lp.g3_div;
        ga.sblocks = lp.g3_sblocks;
        ga.z = tune_.g3_z;
        ga.salt = g3_salt * 0x9e3779b9u + u32(l);
        const bool multi = lp.g3_k1 > 1;
        ga.nodes = multi ? reinterpret_cast<G3Node*>(ws + off_g3_nodes_) : nullptr;
        ga.mhist = multi ? reinterpret_cast<u32*>(ws + off_g3_mhist_) : nullptr;
        ga.cand = multi ? reinterpret_cast<u64*>(ws + off_g3_cand_) : nullptr;
        zero_u32(ga.shist + ga.seg0 * 6 * kG3Bins, segs * 6 * kG3Bins, st);
        const int sgrid = int(segs * lp.g3_sblocks);
        k_g3_sample<1><<<sgrid, kBlock, 0, st>>>(a, ga);
        PKD_LAUNCH_CHECK();
        k_g3_band<1><<<int(segs), kBlock, 0, st>>>(a, ga);
        PKD_LAUNCH_CHECK();
        k_g3_sample<2><<<sgrid, kBlock, 0, st>>>(a, ga);
        PKD_LAUNCH_CHECK();
        k_g3_band<2><<<int(segs), kBlock, 0, st>>>(a, ga);
        PKD_LAUNCH_CHECK();
        with_ncol(dim_, [&](auto nc) {
          constexpr int NC = decltype(nc)::value;
          if constexpr (NC >= 3) {
            constexpr int KI = NC <= 5 ? 8 : 4;
            const size_t lds3 = size_t(std::max(1, kG3Gg * ga.bins3)) * 4;
            // staged tile of NH parts: NC x kBlock * KI / NH floats + a zone byte per row
            auto lds_stg = [&](int nh) { return size_t((std::max(1, (kG3Gg * ga.bins3 + 1) / 2) + 3) & ~3) * 4 +
                                                size_t(kBlock * KI / nh) * (4 * NC + 1); };
            const bool stg16 = (lp.nmax + a.bps - 1) / a.bps < 65536;  // 16-bit histogram counts suffice
            bool wide8 = false;  // rows of >= 6 columns: 8 rows per thread and chunk, stored in 4 parts
            if constexpr (NC > 5) {
              if (tune_.wide_ki == 8 && stg16 && !atomic_ranks3(tune_.atomic_ranks3)) {
                k_g3_part<NC, 8, false, 4><<<grid, kBlock, size_t((std::max(1, (kG3Gg * ga.bins3 + 1) / 2) + 3) & ~3) * 4 +
                                                             size_t(kBlock * 2) * (4 * NC + 1), st>>>(a, ga);
                wide8 = true;
              }
            }
            if (wide8) {
            } else if (atomic_ranks3(tune_.atomic_ranks3)) k_g3_part<NC, KI, true><<<grid, kBlock, lds3, st>>>(a, ga);
            else if (!stg16) k_g3_part<NC, KI, false><<<grid, kBlock, lds3, st>>>(a, ga);
            else if (tune_.g3_stage == 1) k_g3_part<NC, KI, false, 1><<<grid, kBlock, lds_stg(1), st>>>(a, ga);
            else if (tune_.g3_stage == 2) k_g3_part<NC, KI, false, 2><<<grid, kBlock, lds_stg(2), st>>>(a, ga);
            else k_g3_part<NC, KI, false><<<grid, kBlock, lds3, st>>>(a, ga);
            PKD_LAUNCH_CHECK();
            k_g3_res<NC, 0><<<int(segs), kG3Threads, 0, st>>>(a, ga);
            PKD_LAUNCH_CHECK();
            if (lp.g3_k1 > 1) {  // few large segments: every step of levels l+1, l+2 on K blocks per node
              const int k1 = lp.g3_k1, k2 = lp.g3_k2;
              k_g3_mh<1><<<int(2 * segs * k1), kBlock, 0, st>>>(a, ga, k1);
              k_g3_ms<1><<<int(2 * segs), kBlock, 0, st>>>(a, ga);
              k_g3_mc<NC, 1><<<int(2 * segs * k1), kBlock, 0, st>>>(a, ga, k1);
              k_g3_mp<NC, 1><<<int(2 * segs), kG3Threads, 0, st>>>(a, ga);
              k_g3_mr<NC, 1><<<int(2 * segs * k1), kBlock, 0, st>>>(a, ga, k1);
              k_g3_mh<2><<<int(4 * segs * k2), kBlock, 0, st>>>(a, ga, k2);
              k_g3_ms<2><<<int(4 * segs), kBlock, 0, st>>>(a, ga);
              k_g3_mc<NC, 2><<<int(4 * segs * k2), kBlock, 0, st>>>(a, ga, k2);
              k_g3_mp<NC, 2><<<int(4 * segs), kG3Threads, 0, st>>>(a, ga);
              k_g3_mr<NC, 2><<<int(4 * segs * k2), kBlock, 0, st>>>(a, ga, k2);
              k_g3_fin<<<int(kG3Gg * segs), kBlock, 0, st>>>(a, ga);
              PKD_LAUNCH_CHECK();
            } else {
              k_g3_res<NC, 1><<<int(2 * segs), kG3Threads, 0, st>>>(a, ga);
              PKD_LAUNCH_CHECK();
              k_g3_res<NC, 2><<<int(4 * segs), kG3Threads, 0, st>>>(a, ga);
              PKD_LAUNCH_CHECK();
            }
          }
        });
        std::swap(src, dst);
        l += 3;
        continue;
      }
      if (lp.triple) {
        const LevelPlan& lq = levels[size_t(l + 1)];
        const LevelPlan& lr = levels[size_t(l + 2)];
        const i64 segs1 = lq.segs / nparts, segs2 = lr.segs / nparts;
        const int gs = int((segs + 3) / 4), gs1 = int((segs1 + 3) / 4);
        LevelArgs b = level_args(l + 1);
        LevelArgs c = level_args(l + 2);
        TripleArgs ta;
        ta.bins1 = lq.bins;
        ta.axis2 = lr.axis;
        ta.bins2 = lr.bins;
        ta.hist2 = hist_of(l + 2);
        ta.axis3 = (opt_.depth0 + l + 3) % dim_;
        ta.bins3 = lr.next_bins;
        ta.hist3 = l + 3 < lg_ ? hist_of(l + 3) : nullptr;
        with_ncol(dim_, [&](auto nc) {
          constexpr int NC = decltype(nc)::value;
          if constexpr (NC > 0) {
            LevelArgs as = a;  // the key sweeps' own block split (their histogram flush scales with blocks)
            as.bps = std::max(1, a.bps / scan_div_);
            k_scan<NC><<<int(segs * as.bps), kBlock, size_t(2 * lp.next_bins + 64) * 4, st>>>(as);
            PKD_LAUNCH_CHECK();
            k_pivot_both<NC><<<gs + int(segs), kBlock, 0, st>>>(a, segs, gs);
            PKD_LAUNCH_CHECK();
            k_select<<<int(segs1), kBlock, 0, st>>>(b);
            PKD_LAUNCH_CHECK();
            k_scan2<NC><<<int(segs * as.bps), kBlock, size_t(4 * lr.bins + 64) * 4, st>>>(as, ta);
            PKD_LAUNCH_CHECK();
            k_pivot_both<NC><<<gs1 + int(segs1), kBlock, 0, st>>>(b, segs1, gs1);
            PKD_LAUNCH_CHECK();
            k_select<<<int(segs2), kBlock, 0, st>>>(c);
            PKD_LAUNCH_CHECK();
            constexpr int KI = NC <= 5 ? 8 : 4;
            const size_t lds3 = size_t(std::max(1, 8 * ta.bins3)) * 4;
            // the ballot form's stores through an LDS tile (as k_g3_part): 16-bit histogram counts + the tile
            const size_t lds_stg = size_t((std::max(1, (8 * ta.bins3 + 1) / 2) + 3) & ~3) * 4 +
                                   size_t(kBlock * KI / 2) * (4 * NC + 1);
            const bool stg16 = (lp.nmax + a.bps - 1) / a.bps < 65536;
            bool wide8 = false;  // rows of >= 6 columns: 8 rows per thread and chunk, stored in 4 parts
            if constexpr (NC > 5) {
              if (tune_.wide_ki == 8 && stg16 && tune_.part3_stage && !atomic_ranks3(tune_.atomic_ranks3)) {
                k_partition3<NC, 8, false, 4><<<grid, kBlock, size_t((std::max(1, (8 * ta.bins3 + 1) / 2) + 3) & ~3) * 4 +
                                                                size_t(kBlock * 2) * (4 * NC + 1), st>>>(a, ta);
                wide8 = true;
              }
            }
            if (wide8) {
            } else if (atomic_ranks3(tune_.atomic_ranks3)) k_partition3<NC, KI, true><<<grid, kBlock, lds3, st>>>(a, ta);
            else if (stg16 && tune_.part3_stage) k_partition3<NC, KI, false, 2><<<grid, kBlock, lds_stg, st>>>(a, ta);
            else k_partition3<NC, KI, false><<<grid, kBlock, lds3, st>>>(a, ta);
            PKD_LAUNCH_CHECK();
          }
        });
        refine(c, segs2);
        std::swap(src, dst);
        l += 3;
        continue;
      }
      if (lp.pair) {
        const LevelPlan& lq = levels[size_t(l + 1)];
        const i64 segs1 = lq.segs / nparts;
        const size_t lds_a = size_t(2 * lp.next_bins + 64) * 4;
        const int gs = int((segs + 3) / 4);
        with_ncol(dim_, [&](auto nc) {
          constexpr int NC = decltype(nc)::value;
          if constexpr (NC > 0) {
            LevelArgs as = a;  // the scan's own block split (its histogram flush scales with blocks)
            as.bps = std::max(1, a.bps / scan_div_);
            k_scan<NC><<<int(segs * as.bps), kBlock, lds_a, st>>>(as);
            PKD_LAUNCH_CHECK();
            k_pivot_both<NC><<<gs + int(segs), kBlock, 0, st>>>(a, segs, gs);
            PKD_LAUNCH_CHECK();
          }
        });
        LevelArgs b = level_args(l + 1);
        k_select<<<int(segs1), kBlock, 0, st>>>(b);
        PKD_LAUNCH_CHECK();
        PairArgs pa;
        pa.stage2_1 = lq.stage2 ? 1 : 0;
        pa.bins1 = lq.bins;
        pa.axis2 = (opt_.depth0 + l + 2) % dim_;
        pa.bins2 = lq.next_bins;
        pa.hist2n = l + 2 < lg_ ? hist_of(l + 2) : hist_of(l);
        // the second-stage pass of level l+1 reads what the block-reserve count pass would:
        // it also counts each block's certain rows, and the scatter writes from prefix offsets
        const bool pfx = lq.stage2 && a.block_reserve && tune_.prefix;
        if (pfx) {
          pa.bcnt = hs.bcnt;
          pa.bbase = pa.bcnt + size_t(grid) * 4;
        }
        if (lq.stage2) {
          zero_u32(b.hist2, segs1 * kBins2, st);
          k_hist2p<<<grid, kBlock, 0, st>>>(a, pa);
          PKD_LAUNCH_CHECK();
          k_select2<<<int(segs1), kBlock, 0, st>>>(b);
          PKD_LAUNCH_CHECK();
        }
        if (pfx) {
          k_block_bases<<<int(segs), kBlock, 0, st>>>(a, pa);
          PKD_LAUNCH_CHECK();
        }
        const size_t lds_b = size_t(std::max(1, 4 * lq.next_bins)) * 4;
        with_ncol(dim_, [&](auto nc) {
          constexpr int NC = decltype(nc)::value;
          if constexpr (NC > 0) {
            constexpr int KI = NC <= 5 ? 8 : 4;
            // 16-B row loads (4 consecutive rows of a column per lane): one load instruction per
            // 4 rows per column; the pass is bound by requests in flight per CU, not by HBM
            // (profiles/r2_split_build.txt, CU masks). 100M x 3D 12.73 -> 12.52 ms one-stream,
            // 12.22 -> 12.12 split.
            if (atomic_ranks(tune_.atomic_ranks)) {
              if (pfx) k_partition2<NC, KI, true, true><<<grid, kBlock, lds_b, st>>>(a, pa);
              else k_partition2<NC, KI, false, true><<<grid, kBlock, lds_b, st>>>(a, pa);
            } else {
              if (pfx) k_partition2<NC, KI, true><<<grid, kBlock, lds_b, st>>>(a, pa);
              else k_partition2<NC, KI, false><<<grid, kBlock, lds_b, st>>>(a, pa);
            }
          }
        });
        PKD_LAUNCH_CHECK();
        refine(b, segs1);
        std::swap(src, dst);
        l += 2;
        continue;
      }
      const size_t lds = size_t(std::max(1, 2 * lp.next_bins)) * 4;
      with_ncol(dim_, [&](auto nc) {
        constexpr int NC = decltype(nc)::value;
        if (NC > 0 && NC <= 5) k_partition<NC, 8><<<grid, kBlock, lds, st>>>(a);
        else k_partition<NC, 4><<<grid, kBlock, lds, st>>>(a);
      });
      PKD_LAUNCH_CHECK();
      refine(a, segs);
      std::swap(src, dst);
      l += 1;
    }
    if (tail_ >= 0 && l1 == lg_) {  // the last three levels of this part's segments
      TraceRange trt("pkd.tail");
      const LevelPlan& lp = levels[size_t(tail_)];
      const i64 segs = lp.segs / nparts;
      TailArgs ta{src, dst, ncol_, seg_lo, seg_n, cells, lp.segs - 1 + i64(part) * segs, tail_, opt_.depth0,
                  out_pts, out_ids, err, tail_stamp_buffer(), tune_.tail_pipe ? 1 : 0};
      const size_t lds = tail_lds_bytes(tail_items_, tune_.tail_pipe);
      with_ncol(dim_, [&](auto nc) {
        constexpr int D = decltype(nc)::value - 1;
        if constexpr (D >= 1) {
          auto go = [&](auto kern) {
            ensure_dynamic_lds(reinterpret_cast<const void*>(kern), int(lds));
            kern<<<int(segs), kTailThreads, lds, st>>>(ta);
          };
          // one 1024-thread workgroup per CU (128 registers): the two-per-CU shape (64 registers)
          // spills and was slower (100M x 3D k_tail3 1.41 vs 1.32 ms, profiles/r3_tail.txt)
          // (16 items: two key sets and ids on demand, else the 128 registers spill)
          if constexpr (D >= 3) {
            if (tail_lev_ == 4) {  // (two key register sets: the SLIM shape, ids read where keys tie)
              if (tail_items_ == 8) go(&k_tail3<D, 8, 4, true, false, 4>);
              else if (tail_items_ == 12) go(&k_tail3<D, 12, 4, true, false, 4>);
              else go(&k_tail3<D, 16, 4, true, false, 4>);
              return;
            }
          }
          if constexpr (D >= 3) {
            if (tail_items_ == 8) go(&k_tail3<D, 8, 4>);
            else if (tail_items_ == 12 && tune_.tail_slim12 == 0) go(&k_tail3<D, 12, 4>);
            else if (tail_items_ == 12 && tune_.tail_slim12 == 1) go(&k_tail3<D, 12, 4, true>);
            else if (tail_items_ == 12) go(&k_tail3<D, 12, 4, true, true>);
            else go(&k_tail3<D, 16, 4, true>);
          } else {
            if (tail_items_ == 8) go(&k_tail3<D, 8, 4>);
            else if (tail_items_ == 12) go(&k_tail3<D, 12, 4>);
            else go(&k_tail3<D, 16, 4>);
          }
        }
      });
      PKD_LAUNCH_CHECK();
      std::swap(src, dst);
    }
  };
  auto subtree = [&](int part, int nparts, hipStream_t st, const float* src) {
    const i64 leaves = i64(1) << lg_;
    const i64 heap0 = leaves - 1 + i64(part) * (leaves / nparts);
    TraceRange trs("pkd.subtree");
    // the largest segment of level lg_ holds floor(n / 2^lg_) points (a child never exceeds half its parent)
    const int nmax = int(std::min<i64>(nsub_, n_ >> lg_));
    launch_subtree(src, ncol_, dim_, seg_lo, seg_n, cells, heap0, leaves / nparts, opt_.depth0 + lg_, nmax, out_pts,
                   out_ids, err, st, in_rows ? narrow_k : -1, in_rows, in_rs);
  };

  float* src = colsA;
  float* dst = colsB;
  const HistSet whole{{hist[0], hist[1]}, reinterpret_cast<u32*>(ws + off_hist2_), reinterpret_cast<u32*>(ws + off_bcnt_)};
  SplitStreams* sp = (split_parts_ > 1 && !in_rows) ? split_streams_for(stream) : nullptr;
  if (!sp) {
    run_range(0, first_level, lg_, 0, 1, stream, whole, src, dst);
    subtree(0, 1, stream, src);
    return;
  }
  // Split build: the top levels on `stream`, then every part's remaining levels and subtree
  // kernel on its own stream (fork / join through events, so it also captures into a graph).
  run_range(0, 0, split_level_, 0, 1, stream, whole, src, dst);
  PKD_HIP_CHECK(hipEventRecord(sp->fork, stream));
  for (hipStream_t s2 : sp->side) PKD_HIP_CHECK(hipStreamWaitEvent(s2, sp->fork, 0));
  const int P = split_parts_;
  std::vector<hipStream_t> pst(size_t(P), stream);
  std::vector<HistSet> phs(size_t(P), whole);
  std::vector<float*> psrc(size_t(P), src), pdst(size_t(P), dst);
  for (int p = 0; p < P; ++p) {
    const int k = p % split_streams_;
    pst[size_t(p)] = k == 0 ? stream : sp->side[size_t(k - 1)];
    char* set = ws + off_split_ + size_t(k) * split_set_bytes_;
    u32* h0 = reinterpret_cast<u32*>(set);
    u32* h1 = h0 + split_hist_;
    u32* h2 = reinterpret_cast<u32*>(set + align_up(2 * split_hist_ * 4));
    u32* bc = reinterpret_cast<u32*>(set + align_up(2 * split_hist_ * 4) + align_up(split_hist2_ * 4));
    phs[size_t(p)] = HistSet{{h0, h1}, h2, bc};
  }
  // PKD_SPLIT_TRACE=1 (debug, synchronises): when each part's first and last kernel ran,
  // relative to the fork, printed to stderr
  const bool trace = tune_.split_trace;
  std::vector<hipEvent_t> tev;
  auto tmark = [&](hipStream_t st2) {
    if (!trace) return;
    hipEvent_t e = nullptr;
    PKD_HIP_CHECK(hipEventCreate(&e));
    PKD_HIP_CHECK(hipEventRecord(e, st2));
    tev.push_back(e);
  };
  tmark(stream);
  // Part p's remaining levels, then its subtree kernel, on stream p % split_streams_ (all parts
  // start at the fork and run in lockstep; PKD_SPLIT_TRACE shows it)
  for (int p = 0; p < P; ++p) {
    tmark(pst[size_t(p)]);
    run_range(split_level_, split_level_, lg_, p, P, pst[size_t(p)], phs[size_t(p)], psrc[size_t(p)], pdst[size_t(p)]);
    tmark(pst[size_t(p)]);
    subtree(p, P, pst[size_t(p)], psrc[size_t(p)]);
    tmark(pst[size_t(p)]);
  }
  for (size_t k = 0; k < sp->side.size(); ++k) {
    PKD_HIP_CHECK(hipEventRecord(sp->join[k], sp->side[k]));
    PKD_HIP_CHECK(hipStreamWaitEvent(stream, sp->join[k], 0));
  }
  if (trace) {
    PKD_HIP_CHECK(hipStreamSynchronize(stream));
    std::ostringstream os;
    os << "split trace (ms after the fork; part: start / subtree start / end):";
    for (size_t i = 1; i + 2 < tev.size(); i += 3) {
      float t0 = 0, t1 = 0, t2 = 0;
      PKD_HIP_CHECK(hipEventElapsedTime(&t0, tev[0], tev[i]));
      PKD_HIP_CHECK(hipEventElapsedTime(&t1, tev[0], tev[i + 1]));
      PKD_HIP_CHECK(hipEventElapsedTime(&t2, tev[0], tev[i + 2]));
      os << " [" << (i - 1) / 3 << ": " << t0 << " / " << t1 << " / " << t2 << "]";
    }
    std::fprintf(stderr, "%s\n", os.str().c_str());
    for (hipEvent_t e : tev) (void)hipEventDestroy(e);
  }
}

std::vector<u32> GpuBuilder::top_band_report(const void* workspace, hipStream_t stream) const {
  std::vector<u32> r;
  if (!top_) return r;
  u32 b[top4::kNodes][3];
  top4::band_report(static_cast<const char*>(workspace) + off_top_, stream, b);
  for (int x = 0; x < top4::kNodes; ++x)
    for (int k = 0; k < 3; ++k) r.push_back(b[x][k]);
  return r;
}

// Diagnostic: mean cycles of each k_tail3 phase (PKD_TAIL_STAMPS=1) over the recorded blocks.
std::string tail_stamp_report() {
  unsigned long long* d = tail_stamp_buffer();
  if (!d) return "tail stamps disabled (set PKD_TAIL_STAMPS=1)";
  std::vector<unsigned long long> h(size_t(kTailStampBlocks) * kTailStampSlots);
  PKD_HIP_CHECK(hipDeviceSynchronize());
  PKD_HIP_CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  static const char* names[kTailStampSlots] = {"start", "L0.load", "L0.bins", "L0.select", "L0.classify", "L1.load",
                                               "L1.bins", "L1.select", "L1.classify", "L2.load", "L2.bins",
                                               "L2.select", "L2.classify", "move.rank", "col0", "col1", "col2", "col3",
                                               "col4", "col5", "col6", "col7", "col8", "x"};
  double acc[kTailStampSlots] = {};
  int cnt[kTailStampSlots] = {};
  for (int b = 0; b < kTailStampBlocks; ++b) {
    const unsigned long long* s = &h[size_t(b) * kTailStampSlots];
    for (int i = 1; i < kTailStampSlots; ++i)
      if (s[i] && s[i - 1]) {
        acc[i] += double(s[i] - s[i - 1]);
        ++cnt[i];
      }
  }
  std::ostringstream os;
  os << "tail stamps (mean cycles per phase):";
  for (int i = 1; i < kTailStampSlots; ++i)
    if (cnt[i]) os << " " << names[i] << "=" << long(acc[i] / cnt[i]);
  return os.str();
}

}  // namespace pkdtree
