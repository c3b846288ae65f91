// Reference-mode builder on the GPU: the reference's own (quirky) tree, by SELECTION.
//
// build_tree_rec (kdtree_sequential.cpp:30-66, kdtree_mpi.cpp:60-100) sorts only the FIRST
// n - 1 points of every subrange on the node's axis (:46-48), takes list[n/2] as the median and
// recurses on [0, n/2) and [n/2 + 1, n). Nothing needs a sort to reproduce that:
// with m = n / 2 and ranks taken among the n - 1 sortable rows of the segment,
//   * the median is rank m (n = 2: no sortable rank m, the untouched last row is the median);
//   * the left child [0, m) holds ranks 0 .. m - 1, and ITS last row (which the next level
//     leaves out of its sort) is rank m - 1, the left maximum;
//   * the right child [m + 1, n) holds ranks m + 1 .. n - 2 followed by the parent's last row,
//     which stays the right child's last row.
// So every level is an exact rank-m selection per segment with the invariant "the segment's
// last position holds its excluded row": rows never need a full order, only the left maximum
// and the median need exact places. Level-synchronous, on a u32 permutation of the input rows:
//   global levels (segments > kFinCap rows), per level:
//     k_ref_keys      the level's key of every sortable row (gathered through the permutation)
//                     and each segment's key range
//     k_ref_hist      a value-linear histogram of each segment's keys over its range
//     k_ref_select    the buckets b1 <= b2 holding ranks m - 1 and m
//     k_ref_part      every sortable row moves once: left of b1 / inside [b1, b2] / right of b2,
//                     with wave ballots and one reservation per zone and chunk; the last row
//                     keeps its slot; the left zone's maximum and the right zone's minimum are
//                     kept (composite (key, row))
//     k_ref_refine    one workgroup per segment: exact (key, row) ranks m - 1 and m inside the
//                     middle zone (MSD radix select), the middle rows placed around them
//   k_ref_finish      one workgroup per segment of <= kFinCap rows finishes all remaining levels
//                     in LDS: each sub-segment's sortable rows ranked through a per-sub-segment
//                     bucket histogram (buckets = the sub-segment's own slot range) and exact
//                     comparisons inside a bucket, then moved to their ranks
//   k_ref_gather      output rows through the final permutation.
// Ties. std::sort is unstable, so when equal keys meet where the tree is decided the reference
// binary's tree depends on its library's sort internals. Exactly three adjacent-rank pairs of a
// segment decide its tree: (m - 1, m) and (m, m + 1) pick the median and the two child sets,
// (m - 2, m - 1) picks the left child's excluded last row; the order of every other row is
// re-sorted by the next level anyway. A tie on any of those pairs is COUNTED (ties_word()): the
// tree is then the (key, row)-ordered one, which may differ from the binary's, and callers fall
// back to the CPU std::sort builder (kdtree_gpu / kdtree_dist --mode reference, KDTree.build).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "device_utils.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {

namespace {

constexpr int kBlock = 256;
constexpr int kFinCap = 2048;     // largest segment the LDS finish takes
constexpr int kFinThreads = 1024;  // its workgroup: kFinCap / kFinThreads rows per thread (1024: the per-level
                                   // barrier / LDS-latency chains are 4x shorter than with 256 threads)
constexpr int kFinItems = kFinCap / kFinThreads;
constexpr int kItems = 8;         // rows per thread per partition chunk
constexpr int kChunk = kBlock * kItems;
constexpr int kRefineCap = 4096;  // middle rows selected in LDS (more: streamed from global)
// Deciding ties: words[0] counts the tied segments; the median slots of the first kTieSlots of them
// are listed from words[kTieOff] on, so the host can redo exactly those subtrees and their
// ancestors' sorts (reference_repair, cpu_tree.hpp) instead of the whole tree.
constexpr u32 kTieOff = 16;
__device__ __forceinline__ void note_tie(u32* ties, u32 slot) {
  const u32 k = atomicAdd(ties, 1u);
  if (k < ReferenceBuilder::kTieSlots) ties[kTieOff + k] = slot;
}

struct RefSeg {
  u32 lo, n;              // slot range of the segment
  u32 kmin, kmax;         // orderable key range of its sortable rows on the level's axis
  u32 b1, b2;             // buckets of ranks m - 1 and m
  u32 L, M;               // sortable rows below b1 / inside [b1, b2]
  u32 cur[3];             // zone cursors of the partition
  u32 pad;
  u64 left_max;           // largest composite of the left zone (0: empty)
  u64 right_min;          // smallest composite of the right zone (~0: empty)
};

__host__ __device__ inline void seg_geometry(i64 n, int l, i64 j, i64* lo_out, i64* n_out) {
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

// Value-linear bucket of an orderable key's float value over [value(kmin), value(kmax)]:
// (x - lo) * B / span, clamped and truncated. Subtraction, multiplication by a positive constant
// (no FMA: -ffp-contract=off), clamping and truncation are all monotone, so any key order is kept
// and ranks stay exact. Buckets linear in the key's BIT PATTERN instead would crowd the rows of
// any range spanning several binary exponents (every cell around 0) into a few buckets, whose
// select then streams thousands of rows (a 10 M build's refines and LDS finish: 2-5x slower).
struct RefBk {
  float lo, scale;
};
__device__ __forceinline__ RefBk ref_scale(u32 kmin, u32 kmax, u32 B) {
  const float lo = from_orderable(kmin), span = from_orderable(kmax) - lo;
  return RefBk{lo, (span > 0.0f && span < INFINITY) ? float(B) / span : 0.0f};
}
__device__ __forceinline__ u32 ref_bucket_v(float x, RefBk p, u32 B) {
  const float t = fminf(fmaxf((x - p.lo) * p.scale, 0.0f), float(B - 1));
  return u32(t);
}
__device__ __forceinline__ u32 ref_bucket_s(u32 k, RefBk p, u32 B) { return ref_bucket_v(from_orderable(k), p, B); }
__device__ __forceinline__ u32 ref_bucket(u32 k, u32 kmin, u32 kmax, u32 B) {
  return ref_bucket_s(k, ref_scale(kmin, kmax, B), B);
}

__device__ __forceinline__ u64 comp(u32 key, u32 row) { return (u64(key) << 32) | row; }

__global__ __launch_bounds__(kBlock) void k_ref_init(u32* __restrict__ perm, i64 n) {
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += i64(gridDim.x) * kBlock) perm[p] = u32(p);
}

// Segment descriptors of level l (geometry, cleared ranges and cursors) and a zeroed histogram.
__global__ __launch_bounds__(kBlock) void k_ref_seg_init(RefSeg* __restrict__ seg, i64 S, i64 n_total, int l,
                                                         u32* __restrict__ hist, i64 hwords) {
  for (i64 i = i64(blockIdx.x) * kBlock + threadIdx.x; i < hwords; i += i64(gridDim.x) * kBlock) hist[i] = 0u;
  for (i64 s = i64(blockIdx.x) * kBlock + threadIdx.x; seg != nullptr && s < S; s += i64(gridDim.x) * kBlock) {
    i64 lo = 0, m = 0;
    seg_geometry(n_total, l, s, &lo, &m);
    RefSeg r{};
    r.lo = u32(lo);
    r.n = u32(m);
    r.kmin = 0xffffffffu;
    r.kmax = 0u;
    r.left_max = 0ull;
    r.right_min = ~0ull;
    seg[s] = r;
  }
}

// The sortable rows [lo, lo + n - 1) of segment s, split over bps blocks.
__device__ __forceinline__ void block_part(const RefSeg& r, int part, int bps, u32* b0, u32* b1) {
  const u32 sortable = r.n > 0 ? r.n - 1 : 0u;
  const u32 per = (sortable + u32(bps) - 1) / u32(bps);
  *b0 = min(sortable, u32(part) * per);
  *b1 = min(sortable, *b0 + per);
}

__global__ __launch_bounds__(kBlock) void k_ref_keys(const float* __restrict__ pts, int dim, int axis,
                                                     const u32* __restrict__ perm, RefSeg* __restrict__ seg, int bps,
                                                     u32* __restrict__ keys) {
  const i64 s = blockIdx.x / bps;
  const int part = blockIdx.x % bps;
  const RefSeg r = seg[s];
  u32 b0, b1;
  block_part(r, part, bps, &b0, &b1);
  u32 mn = 0xffffffffu, mx = 0u;
  constexpr int U = 4;  // gathers in flight per thread
  for (u32 e0 = b0; e0 < b1; e0 += kBlock * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32 e = e0 + u32(u * kBlock) + threadIdx.x;
      v[u] = e < b1 ? pts[i64(perm[r.lo + e]) * dim + axis] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32 e = e0 + u32(u * kBlock) + threadIdx.x;
      if (e < b1) {
        const u32 k = orderable(v[u]);
        keys[r.lo + e] = k;
        mn = min(mn, k);
        mx = max(mx, k);
      }
    }
  }
  mn = dev::wave_min_u32(mn);
  mx = dev::wave_max_u32(mx);
  if (dev::lane() == 0 && mn <= mx) {
    atomicMin(&seg[s].kmin, mn);
    atomicMax(&seg[s].kmax, mx);
  }
}

__global__ __launch_bounds__(kBlock) void k_ref_hist(const u32* __restrict__ keys, const RefSeg* __restrict__ seg,
                                                     int bps, int B, u32* __restrict__ hist) {
  extern __shared__ u32 h[];
  const i64 s = blockIdx.x / bps;
  const int part = blockIdx.x % bps;
  const RefSeg r = seg[s];
  for (int b = threadIdx.x; b < B; b += kBlock) h[b] = 0u;
  __syncthreads();
  u32 b0, b1;
  block_part(r, part, bps, &b0, &b1);
  for (u32 e = b0 + threadIdx.x; e < b1; e += kBlock)
    atomicAdd(&h[ref_bucket(keys[r.lo + e], r.kmin, r.kmax, u32(B))], 1u);
  __syncthreads();
  u32* out = hist + s * i64(B);
  for (int b = threadIdx.x; b < B; b += kBlock)
    if (h[b]) atomicAdd(&out[b], h[b]);
}

// Bucket holding the rank-th element of h[0, B) (B <= 4096; one wave): *below = rows before it.
__device__ __forceinline__ u32 wave_find(const u32* h, int B, u32 rank, u32* below) {
  const int per = (B + 63) / 64, ln = dev::lane();
  u32 s = 0;
  for (int i = 0; i < per; ++i) {
    const int b = ln * per + i;
    s += b < B ? h[b] : 0u;
  }
  const u32 incl = dev::wave_incl_scan(s), excl = incl - s;
  const u64 m = __ballot(rank >= excl && rank < incl);
  if (!m) {
    *below = __shfl(incl, 63, 64);
    return u32(B);
  }
  const int src = __ffsll((long long)m) - 1;
  u32 bin = 0, bel = 0;
  if (ln == src) {
    u32 c = excl;
    int b = ln * per;
    while (b + 1 < ln * per + per && b + 1 < B && rank >= c + h[b]) c += h[b++];
    bin = u32(b);
    bel = c;
  }
  *below = u32(__shfl(int(bel), src, 64));
  return u32(__shfl(int(bin), src, 64));
}

// One workgroup per segment: the buckets of ranks m - 1 and m (every thread sums B / 256
// consecutive buckets, one block scan, the owning threads walk their buckets).
// The next level's descriptors of segment s's children (geometry, cleared cursors and ranges):
// written for every segment of a level, so no separate initialisation launch is needed (the
// children's key ranges are filled in by this level's refine).
__device__ __forceinline__ void ref_children_init(RefSeg* __restrict__ nsg, i64 s, const RefSeg& r) {
  if (nsg == nullptr || threadIdx.x != 0) return;
  const u32 m = r.n / 2;
  RefSeg c{};
  c.kmin = 0xffffffffu;
  c.kmax = 0u;
  c.left_max = 0ull;
  c.right_min = ~0ull;
  c.lo = r.lo;
  c.n = m;
  nsg[2 * s] = c;
  c.lo = r.lo + m + 1;
  c.n = r.n > m ? r.n - m - 1 : 0u;
  nsg[2 * s + 1] = c;
}

// The buckets of ranks m - 1 and m of segment s from its histogram h (global, or the LDS of the
// histogram block itself): every thread sums B / 256 consecutive buckets, one block scan, the
// owning threads walk their buckets. All threads of the block call it.
__device__ __forceinline__ void ref_select_body(RefSeg* __restrict__ seg, i64 s, const RefSeg& r, int B, const u32* h,
                                                u32* __restrict__ err) {
  __shared__ u32 wsum[kBlock / 64];
  __shared__ u32 res[4];  // b1, L, b2, rows up to the end of b2
  if (r.n < 3) return;    // (uniform: every thread holds the same r)
  const u32 m = r.n / 2;
  const int per = B >= kBlock ? B / kBlock : 1;
  const int t = threadIdx.x, b0 = t * per;
  u32 c = 0;
  if (b0 < B)
    for (int i = 0; i < per; ++i) c += h[b0 + i];
  const u32 incl = dev::wave_incl_scan(c);
  if (dev::lane() == 63) wsum[t / 64] = incl;
  __syncthreads();
  u32 ex = incl - c;
  for (int w = 0; w < t / 64; ++w) ex += wsum[w];
  if (t < 4) res[t] = 0xffffffffu;
  __syncthreads();
  for (int q = 0; q < 2; ++q) {
    const u32 rank = m - 1 + u32(q);
    if (c > 0 && rank >= ex && rank < ex + c) {
      u32 below = ex;
      int b = b0;
      while (rank >= below + h[b]) below += h[b++];
      res[2 * q] = u32(b);
      res[2 * q + 1] = q == 0 ? below : below + h[b];
    }
  }
  __syncthreads();
  if (t == 0) {
    if (res[0] >= u32(B) || res[2] >= u32(B) || res[3] < res[1]) {
      atomicOr(err, 1u);
      return;
    }
    seg[s].b1 = res[0];
    seg[s].L = res[1];
    seg[s].b2 = res[2];
    seg[s].M = res[3] - res[1];
  }
}

// One workgroup per segment: the buckets of ranks m - 1 and m (and, nsg != nullptr, the next
// level's descriptors).
__global__ __launch_bounds__(kBlock) void k_ref_select(RefSeg* __restrict__ seg, int B, const u32* __restrict__ hist,
                                                       u32* __restrict__ err, RefSeg* __restrict__ nsg) {
  const i64 s = blockIdx.x;
  const RefSeg r = seg[s];
  ref_children_init(nsg, s, r);
  ref_select_body(seg, s, r, B, hist + s * i64(B), err);
}

// Every sortable row once: zone 0 (bucket < b1) -> [lo, lo + L), zone 1 -> [lo + L, lo + L + M)
// with its composite in midc, zone 2 -> [lo + L + M, lo + n - 1); the last row keeps its slot.
__global__ __launch_bounds__(kBlock) void k_ref_part(const u32* __restrict__ keys, const u32* __restrict__ src,
                                                     u32* __restrict__ dst, u64* __restrict__ midc,
                                                     RefSeg* __restrict__ seg, int bps, int B) {
  __shared__ u32 wc[kBlock / 64][3];
  __shared__ u32 zb[kBlock / 64][3];
  __shared__ u64 red[kBlock / 64][2];
  const i64 s = blockIdx.x / bps;
  const int part = blockIdx.x % bps;
  const RefSeg r = seg[s];
  const int w = threadIdx.x / 64, ln = dev::lane();
  if (part == 0 && threadIdx.x == 0 && r.n > 0) dst[r.lo + r.n - 1] = src[r.lo + r.n - 1];
  u32 b0, b1;
  block_part(r, part, bps, &b0, &b1);
  u64 lmax = 0ull, rmin = ~0ull;
  for (u32 c0 = b0; c0 < b1; c0 += kChunk) {
    u32 key[kItems], row[kItems], z[kItems], rk[kItems];
    u32 cnt[3] = {0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      const u32 e = c0 + u32(w * 64 * kItems + i * 64 + ln);
      const bool valid = e < b1;
      key[i] = valid ? keys[r.lo + e] : 0u;
      row[i] = valid ? src[r.lo + e] : 0u;
      const u32 b = ref_bucket(key[i], r.kmin, r.kmax, u32(B));
      z[i] = !valid ? 3u : (b < r.b1 ? 0u : (b <= r.b2 ? 1u : 2u));
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const u64 mq = __ballot(z[i] == u32(q));
        if (z[i] == u32(q)) rk[i] = cnt[q] + dev::mbcnt(mq);
        cnt[q] += u32(__popcll(mq));
      }
      const u64 cp = comp(key[i], row[i]);
      if (z[i] == 0u) lmax = cp > lmax ? cp : lmax;
      if (z[i] == 2u) rmin = cp < rmin ? cp : rmin;
    }
    if (ln < 3) wc[w][ln] = cnt[ln];
    __syncthreads();
    if (threadIdx.x < 3) {
      const int q = threadIdx.x;
      u32 t = 0;
      for (int k = 0; k < kBlock / 64; ++k) t += wc[k][q];
      u32 base = t ? atomicAdd(&seg[s].cur[q], t) : 0u;
      for (int k = 0; k < kBlock / 64; ++k) {
        zb[k][q] = base;
        base += wc[k][q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      if (z[i] > 2u) continue;
      const u32 off = zb[w][z[i]] + rk[i];
      const u32 pos = r.lo + (z[i] == 0u ? 0u : (z[i] == 1u ? r.L : r.L + r.M)) + off;
      dst[pos] = row[i];
      if (z[i] == 1u) midc[pos] = comp(key[i], row[i]);
    }
    __syncthreads();  // wc / zb are rewritten by the next chunk
  }
  lmax = dev::wave_max_u64(lmax);
  rmin = dev::wave_min_u64(rmin);
  if (ln == 0) {
    red[w][0] = lmax;
    red[w][1] = rmin;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; ++k) {
      lmax = red[k][0] > lmax ? red[k][0] : lmax;
      rmin = red[k][1] < rmin ? red[k][1] : rmin;
    }
    if (lmax) atomicMax((unsigned long long*)&seg[s].left_max, (unsigned long long)lmax);
    if (rmin != ~0ull) atomicMin((unsigned long long*)&seg[s].right_min, (unsigned long long)rmin);
  }
}

// rank-th smallest (0-based) of the composites visited by each(f): MSD radix select, 8-bit
// digits below the highest bit in which the candidates differ (every thread of the block calls
// it and visits its share).
template <class Each>
__device__ u64 block_select(Each each, u32 rank) {
  __shared__ __align__(16) u32 hist[256];
  __shared__ u64 rmn[kBlock / 64], rmx[kBlock / 64];
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
  for (int k = 1; k < kBlock / 64; ++k) {
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
    hist[threadIdx.x] = 0u;
    __syncthreads();
    each([&](u64 v) {
      if ((v & himask) == prefix) atomicAdd(&hist[u32(v >> sh) & dmask], 1u);
    });
    __syncthreads();
    if (threadIdx.x < 64) {
      u32 below = 0;
      const u32 b = wave_find(hist, 256, rank, &below);
      if (threadIdx.x == 0) {
        info[0] = b;
        info[1] = below;
      }
    }
    __syncthreads();
    prefix |= u64(info[0] & dmask) << sh;
    rank -= info[1];
    hb = sh - 1;
  }
  return prefix;
}

// One workgroup per segment: ranks m - 1 and m inside the middle zone, the middle rows placed
// around them (left of the left maximum / right of the median), the median written to both
// permutation buffers (its slot is final), and the three deciding pairs checked for ties.
__global__ __launch_bounds__(kBlock) void k_ref_refine(const RefSeg* __restrict__ seg, const u64* __restrict__ midc,
                                                       u32* __restrict__ dst, u32* __restrict__ other,
                                                       u32* __restrict__ ties) {
  __shared__ u64 buf[kRefineCap];
  __shared__ u32 cl, cr;
  __shared__ u64 rpred[kBlock / 64], rsucc[kBlock / 64];
  const RefSeg r = seg[blockIdx.x];
  if (r.n < 3) return;
  const u32 m = r.n / 2, L = r.L, M = r.M;
  const u32 base = r.lo + L;
  const bool in_lds = M <= u32(kRefineCap);
  if (in_lds)
    for (u32 e = threadIdx.x; e < M; e += kBlock) buf[e] = midc[base + e];
  if (threadIdx.x == 0) {
    cl = 0;
    cr = 0;
  }
  __syncthreads();
  auto each = [&](auto f) {
    if (in_lds) {
      for (u32 e = threadIdx.x; e < M; e += kBlock) f(buf[e]);
    } else {
      for (u32 e = threadIdx.x; e < M; e += kBlock) f(midc[base + e]);
    }
  };
  const u64 c1 = block_select(each, m - 1 - L);
  const u64 c2 = block_select(each, m - L);
  u64 pred = r.left_max, succ = r.right_min;  // ranks m - 2 and m + 1 (0 / ~0: none)
  each([&](u64 v) {
    if (v < c1) pred = v > pred ? v : pred;
    if (v > c2) succ = v < succ ? v : succ;
  });
  pred = dev::wave_max_u64(pred);
  succ = dev::wave_min_u64(succ);
  if (dev::lane() == 0) {
    rpred[threadIdx.x / 64] = pred;
    rsucc[threadIdx.x / 64] = succ;
  }
  __syncthreads();
  // place: [lo + L, lo + m - 1) left of c1, lo + m - 1 = c1, lo + m = c2, (lo + m, lo + L + M) right of c2
  each([&](u64 v) {
    u32 pos;
    if (v < c1) pos = base + atomicAdd(&cl, 1u);
    else if (v == c1) pos = r.lo + m - 1;
    else if (v == c2) pos = r.lo + m;
    else pos = r.lo + m + 1 + atomicAdd(&cr, 1u);
    dst[pos] = u32(v);
    if (v == c2) other[pos] = u32(v);  // the median's slot is final: both buffers
  });
  if (threadIdx.x == 0) {
    for (int k = 0; k < kBlock / 64; ++k) {
      pred = rpred[k] > pred ? rpred[k] : pred;
      succ = rsucc[k] < succ ? rsucc[k] : succ;
    }
    const u32 k1 = u32(c1 >> 32), k2 = u32(c2 >> 32);
    bool tie = k1 == k2;
    if (m >= 2 && pred != 0ull && u32(pred >> 32) == k1) tie = true;       // rank m - 2 vs the left's last
    if (m + 1 <= r.n - 2 && succ != ~0ull && u32(succ >> 32) == k2) tie = true;  // rank m + 1 vs the median
    if (tie) note_tie(ties, r.lo + m);
  }
}

// LDS min / max of a key into smin[sl] / smax[sl] (every lane calls it): the lanes that share
// the first active lane's sub-segment -- all of them at the first finish levels, where a few
// sub-segments span the block -- combine with wave reductions and one atomic pair; the others
// issue their own.
__device__ __forceinline__ void seg_minmax(u32* smin, u32* smax, int sl, bool act, u32 key) {
  const u64 am = __ballot(act);
  if (!am) return;
  const int leader = __ffsll((long long)am) - 1;
  const int lsl = __shfl(sl, leader, 64);
  const bool same = act && sl == lsl;
  const u32 wmn = dev::wave_min_u32(same ? key : 0xffffffffu), wmx = dev::wave_max_u32(same ? key : 0u);
  if (dev::lane() == leader) {
    atomicMin(&smin[lsl], wmn);
    atomicMax(&smax[lsl], wmx);
  }
  if (act && !same) {
    atomicMin(&smin[sl], key);
    atomicMax(&smax[sl], key);
  }
}

// One workgroup per segment of level lf (<= kFinCap rows): every remaining level in LDS. Each
// sub-segment [sl, sl + sn) with sn >= 3 ranks its sortable rows (all but its last slot) by
// (key, slot): buckets are the sub-segment's own slots [sl, sl + sn - 1), value-linear over its
// key range, so one block scan serves every sub-segment; rows move to sl + rank.
__global__ __launch_bounds__(kFinThreads) void k_ref_finish(const float* __restrict__ pts, int dim, int depth0,
                                                            u32* __restrict__ perm, i64 n_total, int lf, int levels,
                                                            u32* __restrict__ ties) {
  __shared__ u32 P[2][kFinCap], K[kFinCap];
  __shared__ u32 H[kFinCap + 1];
  __shared__ u32 smin[kFinCap], smax[kFinCap];
  u32* tk = smin;  // bucket-ordered keys: smin / smax are dead once the buckets are known
  __shared__ unsigned short tp[kFinCap], SL[kFinCap], SN[kFinCap];
  __shared__ u32 wsum[kFinThreads / 64];
  i64 lo64 = 0, m64 = 0;
  seg_geometry(n_total, lf, blockIdx.x, &lo64, &m64);
  if (m64 <= 1) return;
  const int M = int(m64);
  const u32 lo = u32(lo64);
  const int tid = threadIdx.x;
  for (int p = tid; p < M; p += kFinThreads) {
    P[0][p] = perm[lo + p];
    SL[p] = 0;
    SN[p] = (unsigned short)M;
  }
  int cur = 0;
  __syncthreads();
  for (int l = lf; l < levels; ++l) {
    const int axis = (depth0 + l) % dim;
    // 1. keys of the sortable rows, sub-segment key ranges, empty histogram
    for (int p = tid; p < M; p += kFinThreads) {
      smin[p] = 0xffffffffu;
      smax[p] = 0u;
    }
    for (int p = tid; p <= M; p += kFinThreads) H[p] = 0u;
    __syncthreads();
    u32 key[kFinItems], slot[kFinItems];
    bool srt[kFinItems];
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = tid + i * kFinThreads;
      srt[i] = false;
      key[i] = 0;
      int sl = 0;
      if (p < M) {
        const int sn = SN[p];
        sl = SL[p];
        srt[i] = sn >= 3 && p != sl + sn - 1;
        if (srt[i]) key[i] = orderable(pts[i64(P[cur][p]) * dim + axis]);
      }
      seg_minmax(smin, smax, sl, srt[i], key[i]);
    }
    __syncthreads();
    // 2. bucket counts (bucket = a slot of the sub-segment's sortable range)
    u32 bk[kFinItems];
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = tid + i * kFinThreads;
      bk[i] = 0;
      slot[i] = 0;
      if (srt[i]) {
        const int sl = SL[p], sn = SN[p];
        bk[i] = u32(sl) + ref_bucket(key[i], smin[sl], smax[sl], u32(sn - 1));
        slot[i] = atomicAdd(&H[bk[i]], 1u);
      }
    }
    __syncthreads();
    // 3. exclusive scan of H[0, M) (H[M] = total)
    {
      constexpr int C = kFinItems;
      u32 x[C], s = 0;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int b = tid * C + j;
        x[j] = b < M ? H[b] : 0u;
        s += x[j];
      }
      const u32 incl = dev::wave_incl_scan(s);
      if (dev::lane() == 63) wsum[tid / 64] = incl;
      __syncthreads();
      u32 run = incl - s;
      for (int w = 0; w < tid / 64; ++w) run += wsum[w];
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int b = tid * C + j;
        if (b < M) H[b] = run;
        run += x[j];
      }
      if (tid == kFinThreads - 1) H[M] = run;
    }
    __syncthreads();
    // 4. rows in bucket order; rank = rows of the sub-segment in lower buckets (+ the bucket's
    // smaller rows below)
    u32 rank[kFinItems], st[kFinItems], cnt[kFinItems];
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = tid + i * kFinThreads;
      rank[i] = 0;
      st[i] = 0;
      cnt[i] = 0;
      if (srt[i]) {
        const int sl = SL[p];
        st[i] = H[bk[i]];
        cnt[i] = H[bk[i] + 1] - st[i];
        rank[i] = st[i] - H[sl];
        tk[st[i] + slot[i]] = key[i];
        tp[st[i] + slot[i]] = (unsigned short)p;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = tid + i * kFinThreads;
      for (u32 j = 0; j < cnt[i]; ++j) {
        const u32 q = st[i] + j;
        const u32 kq = tk[q];
        rank[i] += (kq < key[i] || (kq == key[i] && int(tp[q]) < p)) ? 1u : 0u;
      }
    }
    // 5. move: sortable rows to sl + rank, the others stay
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = tid + i * kFinThreads;
      if (p >= M) continue;
      const int np = srt[i] ? int(SL[p]) + int(rank[i]) : p;
      P[cur ^ 1][np] = P[cur][p];
      K[np] = key[i];
    }
    __syncthreads();
    cur ^= 1;
    // 6. ties on the deciding pairs of every sub-segment (checked by its first slot's thread),
    // then the next level's sub-segments
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = tid + i * kFinThreads;
      if (p >= M) continue;
      const int sl = SL[p], sn = SN[p];
      if (p == sl && sn >= 3) {
        const int m = sn / 2;
        const u32* kk = K + sl;
        bool tie = kk[m - 1] == kk[m];
        if (m >= 2 && kk[m - 2] == kk[m - 1]) tie = true;
        if (m + 1 <= sn - 2 && kk[m] == kk[m + 1]) tie = true;
        if (tie) note_tie(ties, lo + u32(sl) + u32(m));
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = tid + i * kFinThreads;
      if (p >= M) continue;
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
  for (int p = tid; p < M; p += kFinThreads) perm[lo + p] = P[cur][p];
}

// Rows out in slot order: one thread per output ELEMENT (slot p, coordinate c), so a wave reads
// and writes runs of consecutive floats of a row (a thread per row strode a whole row between
// lanes: 500 k x 128D 0.82 ms); 4 elements per thread in flight.
__global__ __launch_bounds__(kBlock) void k_ref_gather(const float* __restrict__ pts, const u32* __restrict__ ids,
                                                       u32 id_base, int dim, const u32* __restrict__ perm, i64 n,
                                                       float* __restrict__ out_pts, u32* __restrict__ out_ids) {
  const i64 total = n * dim, stride = i64(gridDim.x) * kBlock;
  constexpr int U = 4;
  for (i64 e0 = i64(blockIdx.x) * kBlock + threadIdx.x; e0 < total; e0 += U * stride) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 e = e0 + u * stride;
      const i64 p = e / dim, c = e - p * dim;
      v[u] = e < total ? pts[i64(perm[p]) * dim + c] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 e = e0 + u * stride;
      if (e < total) out_pts[e] = v[u];
    }
  }
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += stride) {
    const i64 r = perm[p];
    out_ids[p] = ids ? ids[r] : id_base + u32(r);
  }
}

// ---- row path (dim <= 8): rows move as SoA columns (dim coordinates + the input row index),
// so a level reads its keys contiguously and the medians go straight to the output -------------
// cols(c, p): column c of slot p; column dim holds the input row index bits.
struct RowCols {
  float* c;
  i64 ncol;
  __device__ __forceinline__ float& at(int col, u32 p) const { return c[i64(col) * ncol + p]; }
};

// Block-wide min / max (every thread calls it; red: LDS [kBlock / 64][2]); valid in thread 0.
__device__ __forceinline__ void block_minmax(u32* mn, u32* mx, u32 (*red)[2]) {
  u32 a = dev::wave_min_u32(*mn), b = dev::wave_max_u32(*mx);
  __syncthreads();
  if (dev::lane() == 0) {
    red[threadIdx.x / 64][0] = a;
    red[threadIdx.x / 64][1] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k < kBlock / 64; ++k) {
      a = min(a, red[k][0]);
      b = max(b, red[k][1]);
    }
  *mn = a;
  *mx = b;
}

// AoS input -> SoA columns; the key range of level 0's sortable rows [0, n - 1).
__global__ __launch_bounds__(kBlock) void k_rr_prep(const float* __restrict__ pts, i64 n, int dim, int axis0,
                                                    RowCols out, RefSeg* __restrict__ seg0) {
  __shared__ u32 red[kBlock / 64][2];
  u32 mn = 0xffffffffu, mx = 0u;
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += i64(gridDim.x) * kBlock) {
    for (int c = 0; c < dim; ++c) {
      const float v = pts[p * dim + c];
      out.at(c, u32(p)) = v;
      if (c == axis0 && p + 1 < n) {
        mn = min(mn, orderable(v));
        mx = max(mx, orderable(v));
      }
    }
    out.at(dim, u32(p)) = __uint_as_float(u32(p));
  }
  block_minmax(&mn, &mx, red);
  if (threadIdx.x == 0 && seg0 && mn <= mx) {
    atomicMin(&seg0->kmin, mn);
    atomicMax(&seg0->kmax, mx);
  }
}

// Histogram of a level's sortable keys: every block's LDS histogram is STORED (all B bins,
// coalesced) -- straight into the segment's histogram when the segment has one block, else into
// per-block partials that k_rr_hred sums. (Flushing with global atomics cost ~4 M atomics a level:
// 256 blocks x 16 Ki bins; 30 us of a 10 M level's 36.)
__global__ __launch_bounds__(kBlock) void k_rr_hist(RowCols src, int axis, RefSeg* __restrict__ seg, int bps,
                                                    int B, u32* __restrict__ out, u32* __restrict__ err,
                                                    RefSeg* __restrict__ nsg, int fuse_select) {
  extern __shared__ u32 h[];
  const i64 s = blockIdx.x / bps;
  const int part = blockIdx.x % bps;
  const RefSeg r = seg[s];
  for (int b = threadIdx.x; b < B; b += kBlock) h[b] = 0u;
  __syncthreads();
  u32 b0, b1;
  block_part(r, part, bps, &b0, &b1);
  const RefBk sc = ref_scale(r.kmin, r.kmax, u32(B));
  const float* kc = src.c + i64(axis) * src.ncol + r.lo;
  constexpr int U = 4;
  for (u32 e0 = b0; e0 < b1; e0 += kBlock * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32 e = e0 + u32(u * kBlock) + threadIdx.x;
      v[u] = kc[e < b1 ? e : b0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32 e = e0 + u32(u * kBlock) + threadIdx.x;
      if (e < b1) atomicAdd(&h[ref_bucket_v(v[u], sc, u32(B))], 1u);
    }
  }
  __syncthreads();
  if (fuse_select) {  // (bps == 1) the block holds its segment's whole histogram: select right here
    ref_children_init(nsg, s, r);
    ref_select_body(seg, s, r, B, h, err);
    return;
  }
  u32* o = out + i64(blockIdx.x) * B;  // (block = segment when bps == 1)
  for (int b = threadIdx.x; b < B; b += kBlock) o[b] = h[b];
}

// Segment histograms from the blocks' partials: one thread per (segment, bin).
__global__ __launch_bounds__(kBlock) void k_rr_hred(const u32* __restrict__ part, int bps, int B, i64 total,
                                                    u32* __restrict__ hist) {
  const i64 i = i64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= total) return;
  const i64 s = i / B, b = i % B;
  const u32* p = part + (s * bps) * B + b;
  u32 sum = 0;
  for (int k = 0; k < bps; ++k) sum += p[i64(k) * B];
  hist[i] = sum;
}

// Per-block partials of a row-path partition (no same-address atomics across blocks): the
// children's next-axis ranges and the zones' extreme composites, reduced by k_rr_refine.
struct PartPartial {
  u32 lmn, lmx, rmn, rmx;
  u64 lmax, rmin;
};

// The row-path partition: as k_ref_part, moving every column; the children's key ranges on the
// next level's axis are collected (left zone -> left child, right zone and the last row -> right
// child; the middle rows' share is added by k_rr_refine).
template <int NC>
__global__ __launch_bounds__(kBlock) void k_rr_part(RowCols src, RowCols dst, int axis, int naxis,
                                                    RefSeg* __restrict__ seg, int bps, int B,
                                                    PartPartial* __restrict__ partials) {
  constexpr int kI = NC <= 5 ? 8 : 4;  // rows per thread per chunk
  __shared__ u32 wc[kBlock / 64][3];
  __shared__ u32 zb[kBlock / 64][3];
  __shared__ u64 red[kBlock / 64][2];
  __shared__ u32 red2[kBlock / 64][2];
  const i64 s = blockIdx.x / bps;
  const int part = blockIdx.x % bps;
  const RefSeg r = seg[s];
  const int w = threadIdx.x / 64, ln = dev::lane();
  u32 lmn = 0xffffffffu, lmx = 0u, rmn = 0xffffffffu, rmx = 0u;  // children's next-axis ranges
  if (part == 0 && threadIdx.x == 0 && r.n > 0) {  // the last row keeps its slot (the right child's last)
    const u32 p = r.lo + r.n - 1;
    for (int c = 0; c < NC; ++c) dst.at(c, p) = src.at(c, p);
    rmn = rmx = orderable(src.at(naxis, p));
  }
  u32 b0, b1;
  block_part(r, part, bps, &b0, &b1);
  const RefBk sc = ref_scale(r.kmin, r.kmax, u32(B));
  u64 lmax = 0ull, rmin = ~0ull;
  constexpr int kCh = kBlock * kI;
  for (u32 c0 = b0; c0 < b1; c0 += kCh) {
    float v[kI][NC];
    u32 z[kI], rk[kI];
    u32 cnt[3] = {0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < kI; ++i) {
      const u32 e = c0 + u32(w * 64 * kI + i * 64 + ln);
      const bool valid = e < b1;
      const u32 pe = r.lo + (valid ? e : b0);
#pragma unroll
      for (int c = 0; c < NC; ++c) v[i][c] = src.at(c, pe);
      float kf = v[i][0], nf = v[i][0];
#pragma unroll
      for (int c = 1; c < NC - 1; ++c) {
        kf = c == axis ? v[i][c] : kf;
        nf = c == naxis ? v[i][c] : nf;
      }
      const u32 key = orderable(kf);
      const u32 b = ref_bucket_v(kf, sc, u32(B));
      z[i] = !valid ? 3u : (b < r.b1 ? 0u : (b <= r.b2 ? 1u : 2u));
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const u64 mq = __ballot(z[i] == u32(q));
        if (z[i] == u32(q)) rk[i] = cnt[q] + dev::mbcnt(mq);
        cnt[q] += u32(__popcll(mq));
      }
      const u64 cp = comp(key, __float_as_uint(v[i][NC - 1]));
      const u32 nk = orderable(nf);
      if (z[i] == 0u) {
        lmax = cp > lmax ? cp : lmax;
        lmn = min(lmn, nk);
        lmx = max(lmx, nk);
      }
      if (z[i] == 2u) {
        rmin = cp < rmin ? cp : rmin;
        rmn = min(rmn, nk);
        rmx = max(rmx, nk);
      }
    }
    if (ln < 3) wc[w][ln] = cnt[ln];
    __syncthreads();
    if (threadIdx.x < 3) {
      const int q = threadIdx.x;
      u32 t = 0;
      for (int k = 0; k < kBlock / 64; ++k) t += wc[k][q];
      u32 base = t ? atomicAdd(&seg[s].cur[q], t) : 0u;
      for (int k = 0; k < kBlock / 64; ++k) {
        zb[k][q] = base;
        base += wc[k][q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kI; ++i) {
      if (z[i] > 2u) continue;
      const u32 pos = r.lo + (z[i] == 0u ? 0u : (z[i] == 1u ? r.L : r.L + r.M)) + zb[w][z[i]] + rk[i];
#pragma unroll
      for (int c = 0; c < NC; ++c) dst.at(c, pos) = v[i][c];
    }
    __syncthreads();  // wc / zb are rewritten by the next chunk
  }
  block_minmax(&lmn, &lmx, red2);
  block_minmax(&rmn, &rmx, red2);
  lmax = dev::wave_max_u64(lmax);
  rmin = dev::wave_min_u64(rmin);
  if (ln == 0) {
    red[w][0] = lmax;
    red[w][1] = rmin;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; ++k) {
      lmax = red[k][0] > lmax ? red[k][0] : lmax;
      rmin = red[k][1] < rmin ? red[k][1] : rmin;
    }
    partials[blockIdx.x] = PartPartial{lmn, lmx, rmn, rmx, lmax, rmin};
  }
}

// Row-path refine (one workgroup per segment): the partition's block partials are reduced; the
// middle zone is copied to the same slots of src (dead there since the partition), then every
// middle row is read from src and written to its place in dst; the median row goes straight to
// the output; the children's next-axis ranges are stored (this workgroup is their only writer).
// Middle zones of <= 64 rows (the deep levels) are ranked by one wave without a barrier.
// Middle zones of <= 64 rows (every segment of the deep levels): one wave per segment, four per
// block, no barrier. Each lane holds one middle row (loads before stores: in place), ranks it
// against the others by shuffles and writes it to its final place.
template <int NC>
__device__ __forceinline__ void rr_refine_wave(const RefSeg& r, i64 s, RowCols dst, int axis, int naxis,
                                               RefSeg* __restrict__ nseg, const PartPartial* __restrict__ partials,
                                               int bps, const u32* __restrict__ ids, u32 id_base,
                                               float* __restrict__ out_pts, u32* __restrict__ out_ids,
                                               u32* __restrict__ ties) {
  constexpr int D = NC - 1;
  const int ln = dev::lane();
  const u32 m = r.n / 2, L = r.L, M = r.M;
  u32 lmn = 0xffffffffu, lmx = 0u, rmn = 0xffffffffu, rmx = 0u;
  u64 pred = 0ull, succ = ~0ull;
  for (int k = ln; k < bps; k += 64) {
    const PartPartial q = partials[s * bps + k];
    lmn = min(lmn, q.lmn);
    lmx = max(lmx, q.lmx);
    rmn = min(rmn, q.rmn);
    rmx = max(rmx, q.rmx);
    pred = q.lmax > pred ? q.lmax : pred;
    succ = q.rmin < succ ? q.rmin : succ;
  }
  const bool in = ln < int(M);
  const u32 p = r.lo + L + (in ? u32(ln) : 0u);
  float v[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) v[c] = dst.at(c, p);
  float kf = v[0], nf = v[0];
#pragma unroll
  for (int c = 1; c < D; ++c) {
    kf = c == axis ? v[c] : kf;
    nf = c == naxis ? v[c] : nf;
  }
  const u32 row = __float_as_uint(v[D]);
  const u64 ck = in ? comp(orderable(kf), row) : ~0ull;
  u32 rk = 0;
  for (u32 j = 0; j < M; ++j) rk += dev::shfl_u64(ck, int(j)) < ck ? 1u : 0u;
  // rank among the middle rows: < m - 1 - L left of c1, == m - 1 - L c1, == m - L the median
  const u32 r1 = m - 1 - L, r2 = m - L;
  const u32 nk = orderable(nf);
  if (in) {
    if (rk == r2) {
      const u32 slot = r.lo + m;
#pragma unroll
      for (int c = 0; c < D; ++c) out_pts[i64(slot) * D + c] = v[c];
      out_ids[slot] = ids ? ids[row] : id_base + row;
    } else {
      const u32 pos = rk < r1 ? r.lo + L + rk : (rk == r1 ? r.lo + m - 1 : r.lo + m + 1 + (rk - r2 - 1));
#pragma unroll
      for (int c = 0; c < NC; ++c) dst.at(c, pos) = v[c];
    }
    if (rk <= r1) {
      lmn = min(lmn, nk);
      lmx = max(lmx, nk);
    } else if (rk > r2) {
      rmn = min(rmn, nk);
      rmx = max(rmx, nk);
    }
    if (rk < r1) pred = ck > pred ? ck : pred;
    if (rk > r2) succ = ck < succ ? ck : succ;
  }
  const u64 c1 = dev::shfl_u64(ck, __ffsll((long long)__ballot(in && rk == r1)) - 1);
  const u64 c2 = dev::shfl_u64(ck, __ffsll((long long)__ballot(in && rk == r2)) - 1);
  lmn = dev::wave_min_u32(lmn);
  lmx = dev::wave_max_u32(lmx);
  rmn = dev::wave_min_u32(rmn);
  rmx = dev::wave_max_u32(rmx);
  pred = dev::wave_max_u64(pred);
  succ = dev::wave_min_u64(succ);
  if (ln == 0) {
    if (nseg) {
      nseg[2 * s].kmin = lmn;
      nseg[2 * s].kmax = lmx;
      nseg[2 * s + 1].kmin = rmn;
      nseg[2 * s + 1].kmax = rmx;
    }
    const u32 k1 = u32(c1 >> 32), k2 = u32(c2 >> 32);
    bool tie = k1 == k2;
    if (m >= 2 && pred != 0ull && u32(pred >> 32) == k1) tie = true;
    if (m + 1 <= r.n - 2 && succ != ~0ull && u32(succ >> 32) == k2) tie = true;
    if (tie) note_tie(ties, r.lo + m);
  }
}

// Blocks [0, gsm): four segments each, one wave per segment whose middle zone holds <= 64 rows;
// blocks [gsm, gsm + S): one segment each, the larger middle zones.
template <int NC>
__global__ __launch_bounds__(kBlock) void k_rr_refine(RowCols src, RowCols dst, int dim, int axis, int naxis,
                                                      const RefSeg* __restrict__ seg, RefSeg* __restrict__ nseg,
                                                      const PartPartial* __restrict__ partials, int bps,
                                                      const u32* __restrict__ ids, u32 id_base,
                                                      float* __restrict__ out_pts, u32* __restrict__ out_ids,
                                                      u32* __restrict__ ties, int S, int gsm) {
  if (int(blockIdx.x) < gsm) {
    const i64 sw = i64(blockIdx.x) * (kBlock / 64) + threadIdx.x / 64;
    if (sw >= S) return;
    const RefSeg r = seg[sw];
    if (r.n < 3 || r.M > 64u) return;
    rr_refine_wave<NC>(r, sw, dst, axis, naxis, nseg, partials, bps, ids, id_base, out_pts, out_ids, ties);
    return;
  }
  __shared__ u64 buf[kRefineCap];
  __shared__ u32 cl, cr;
  __shared__ u64 r64[kBlock / 64][3];
  __shared__ u32 red2[kBlock / 64][2];
  __shared__ u64 sc1, sc2;
  const i64 sb = i64(blockIdx.x) - gsm;
  const RefSeg r = seg[sb];
  if (r.n < 3 || r.M <= 64u) return;
  const u32 m = r.n / 2, L = r.L, M = r.M;
  const u32 base = r.lo + L;
  (void)dim;  // (NC = dim + 1)
  const int tid = threadIdx.x, w = tid / 64, ln = dev::lane();
  // the partition's partials
  u32 lmn = 0xffffffffu, lmx = 0u, rmn = 0xffffffffu, rmx = 0u;
  u64 pred = 0ull, succ = ~0ull;  // left zone max / right zone min so far
  for (int k = tid; k < bps; k += kBlock) {
    const PartPartial q = partials[sb * bps + k];
    lmn = min(lmn, q.lmn);
    lmx = max(lmx, q.lmx);
    rmn = min(rmn, q.rmn);
    rmx = max(rmx, q.rmx);
    pred = q.lmax > pred ? q.lmax : pred;
    succ = q.rmin < succ ? q.rmin : succ;
  }
  const bool in_lds = M <= u32(kRefineCap);
  for (u32 e = tid; e < M; e += kBlock) {
    const u32 p = base + e;
    float key = 0.0f;
    u32 row = 0;
    for (int c = 0; c < NC; ++c) {
      const float v = dst.at(c, p);
      src.at(c, p) = v;
      if (c == axis) key = v;
      if (c == dim) row = __float_as_uint(v);
    }
    if (in_lds) buf[e] = comp(orderable(key), row);
  }
  if (tid == 0) {
    cl = 0;
    cr = 0;
  }
  __syncthreads();
  auto val = [&](u32 e) -> u64 {
    return in_lds ? buf[e] : comp(orderable(src.at(axis, base + e)), __float_as_uint(src.at(dim, base + e)));
  };
  u64 c1, c2;
  if (M <= 64) {  // one wave: ranks by comparison, no barrier
    if (w == 0) {
      const u64 v = ln < int(M) ? buf[ln] : ~0ull;
      u32 rk = 0;
      for (u32 j = 0; j < M; ++j) rk += dev::shfl_u64(v, int(j)) < v ? 1u : 0u;
      const u64 m1 = __ballot(ln < int(M) && rk == m - 1 - L), m2 = __ballot(ln < int(M) && rk == m - L);
      const u64 a1 = dev::shfl_u64(v, __ffsll((long long)m1) - 1), a2 = dev::shfl_u64(v, __ffsll((long long)m2) - 1);
      if (ln == 0) {
        sc1 = a1;
        sc2 = a2;
      }
    }
    __syncthreads();
    c1 = sc1;
    c2 = sc2;
  } else {
    auto each = [&](auto f) {
      for (u32 e = tid; e < M; e += kBlock) f(val(e));
    };
    c1 = block_select(each, m - 1 - L);
    u64 nx = ~0ull;  // rank m is the successor of rank m - 1
    each([&](u64 v) {
      if (v > c1) nx = v < nx ? v : nx;
    });
    nx = dev::wave_min_u64(nx);
    if (ln == 0) r64[w][0] = nx;
    __syncthreads();
    c2 = r64[0][0];
    for (int k = 1; k < kBlock / 64; ++k) c2 = r64[k][0] < c2 ? r64[k][0] : c2;
  }
  for (u32 e = tid; e < M; e += kBlock) {
    const u32 p = base + e;
    const u64 v = val(e);
    const u32 nk = orderable(src.at(naxis, p));
    if (v < c1) pred = v > pred ? v : pred;
    if (v > c2) succ = v < succ ? v : succ;
    if (v == c2) {  // the median: its slot is final
      const u32 slot = r.lo + m, row = u32(v);
      for (int c = 0; c < dim; ++c) out_pts[i64(slot) * dim + c] = src.at(c, p);
      out_ids[slot] = ids ? ids[row] : id_base + row;
      continue;
    }
    u32 pos;
    if (v < c1) pos = base + atomicAdd(&cl, 1u);
    else if (v == c1) pos = r.lo + m - 1;
    else pos = r.lo + m + 1 + atomicAdd(&cr, 1u);
    for (int c = 0; c < NC; ++c) dst.at(c, pos) = src.at(c, p);
    if (v <= c1) {
      lmn = min(lmn, nk);
      lmx = max(lmx, nk);
    } else {
      rmn = min(rmn, nk);
      rmx = max(rmx, nk);
    }
  }
  block_minmax(&lmn, &lmx, red2);
  block_minmax(&rmn, &rmx, red2);
  pred = dev::wave_max_u64(pred);
  succ = dev::wave_min_u64(succ);
  if (ln == 0) {
    r64[w][1] = pred;
    r64[w][2] = succ;
  }
  __syncthreads();
  if (tid == 0) {
    for (int k = 0; k < kBlock / 64; ++k) {
      pred = r64[k][1] > pred ? r64[k][1] : pred;
      succ = r64[k][2] < succ ? r64[k][2] : succ;
    }
    if (nseg) {
      nseg[2 * sb].kmin = lmn;
      nseg[2 * sb].kmax = lmx;
      nseg[2 * sb + 1].kmin = rmn;
      nseg[2 * sb + 1].kmax = rmx;
    }
    const u32 k1 = u32(c1 >> 32), k2 = u32(c2 >> 32);
    bool tie = k1 == k2;
    if (m >= 2 && pred != 0ull && u32(pred >> 32) == k1) tie = true;
    if (m + 1 <= r.n - 2 && succ != ~0ull && u32(succ >> 32) == k2) tie = true;
    if (tie) note_tie(ties, r.lo + m);
  }
}

// Row-path LDS finish: the segment's columns are loaded once (X[c][local row]); slots hold
// local row indices, keys are read through them, and every slot's row is written to the
// output at the end. Thread t owns the kFinItems consecutive slots from t * kFinItems; a
// sub-segment's key range is combined per wave before its LDS atomics (seg_minmax).
__global__ __launch_bounds__(kFinThreads) void k_rr_finish(RowCols src, int dim, int depth0, i64 n_total, int lf,
                                                           int levels, const u32* __restrict__ ids, u32 id_base,
                                                           float* __restrict__ out_pts, u32* __restrict__ out_ids,
                                                           u32* __restrict__ ties) {
  extern __shared__ float X[];  // [dim + 1][kFinCap]
  __shared__ unsigned short P[2][kFinCap];
  __shared__ u32 H[kFinCap + 1];
  __shared__ u32 smin[kFinCap], smax[kFinCap];
  __shared__ unsigned short tp[kFinCap], SL[kFinCap], SN[kFinCap];
  __shared__ u32 wsum[kFinThreads / 64];
  u32* tk = smin;  // bucket-ordered keys (smin / smax are dead once the buckets are known)
  u32* K = smax;   // sorted keys of the level, for the tie checks
  i64 lo64 = 0, m64 = 0;
  seg_geometry(n_total, lf, blockIdx.x, &lo64, &m64);
  if (m64 <= 0) return;
  const int M = int(m64);
  const u32 lo = u32(lo64);
  const int tid = threadIdx.x, p0 = tid * kFinItems;
  for (int c = 0; c <= dim; ++c)
    for (int p = tid; p < M; p += kFinThreads) X[c * kFinCap + p] = src.at(c, lo + u32(p));
  for (int p = tid; p < M; p += kFinThreads) {
    P[0][p] = (unsigned short)p;
    SL[p] = 0;
    SN[p] = (unsigned short)M;
    smin[p] = 0xffffffffu;
    smax[p] = 0u;
  }
  int cur = 0;
  __syncthreads();
  for (int l = lf; l < levels; ++l) {
    const int axis = (depth0 + l) % dim;
    const float* xk = X + axis * kFinCap;
    for (int p = tid; p <= M; p += kFinThreads) H[p] = 0u;
    u32 key[kFinItems], slot[kFinItems], bk[kFinItems];
    bool srt[kFinItems];
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = p0 + i;
      srt[i] = false;
      key[i] = 0;
      int sl = 0;
      if (p < M) {
        const int sn = SN[p];
        sl = SL[p];
        srt[i] = sn >= 3 && p != sl + sn - 1;
        if (srt[i]) key[i] = orderable(xk[P[cur][p]]);
      }
      seg_minmax(smin, smax, sl, srt[i], key[i]);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = p0 + i;
      bk[i] = 0;
      slot[i] = 0;
      if (srt[i]) {
        const int sl = SL[p], sn = SN[p];
        const u32 kmn = smin[sl];
        bk[i] = u32(sl) + ref_bucket_s(key[i], ref_scale(kmn, smax[sl], u32(sn - 1)), u32(sn - 1));
        slot[i] = atomicAdd(&H[bk[i]], 1u);
      }
    }
    __syncthreads();
    {  // exclusive scan of H[0, M): thread t owns H[t * kFinItems, + kFinItems); H[M] = total
      u32 x[kFinItems], sum = 0;
#pragma unroll
      for (int j = 0; j < kFinItems; ++j) {
        x[j] = p0 + j < M ? H[p0 + j] : 0u;
        sum += x[j];
      }
      const u32 incl = dev::wave_incl_scan(sum);
      if (dev::lane() == 63) wsum[tid / 64] = incl;
      __syncthreads();
      u32 run = incl - sum;
      for (int w = 0; w < tid / 64; ++w) run += wsum[w];
#pragma unroll
      for (int j = 0; j < kFinItems; ++j) {
        if (p0 + j < M) H[p0 + j] = run;
        run += x[j];
      }
      if (tid == kFinThreads - 1) H[M] = run;
    }
    __syncthreads();
    u32 rank[kFinItems], st[kFinItems], cnt[kFinItems];
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = p0 + i;
      rank[i] = 0;
      st[i] = 0;
      cnt[i] = 0;
      if (srt[i]) {
        st[i] = H[bk[i]];
        cnt[i] = H[bk[i] + 1] - st[i];
        rank[i] = st[i] - H[SL[p]];
        tk[st[i] + slot[i]] = key[i];
        tp[st[i] + slot[i]] = (unsigned short)p;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = p0 + i;
      for (u32 j = 0; j < cnt[i]; ++j) {
        const u32 q = st[i] + j;
        const u32 kq = tk[q];
        rank[i] += (kq < key[i] || (kq == key[i] && int(tp[q]) < p)) ? 1u : 0u;
      }
    }
    __syncthreads();  // tk (= smin) is read above; K (= smax) is written below
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = p0 + i;
      if (p >= M) continue;
      const int np = srt[i] ? int(SL[p]) + int(rank[i]) : p;
      P[cur ^ 1][np] = P[cur][p];
      K[np] = key[i];
    }
    __syncthreads();
    cur ^= 1;
    // ties on the deciding pairs of every sub-segment (checked by its first slot's thread),
    // then the next level's sub-segments; their key-range words are reset at their heads
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = p0 + i;
      if (p >= M) continue;
      const int sl = SL[p], sn = SN[p];
      if (p == sl && sn >= 3) {
        const int m = sn / 2;
        const u32* kk = K + sl;
        bool tie = kk[m - 1] == kk[m];
        if (m >= 2 && kk[m - 2] == kk[m - 1]) tie = true;
        if (m + 1 <= sn - 2 && kk[m] == kk[m + 1]) tie = true;
        if (tie) note_tie(ties, lo + u32(sl) + u32(m));
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kFinItems; ++i) {
      const int p = p0 + i;
      if (p >= M) continue;
      smin[p] = 0xffffffffu;
      smax[p] = 0u;
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
  for (int e = tid; e < M * dim; e += kFinThreads) {  // rows out: consecutive threads, consecutive floats
    const int p = e / dim, c = e - p * dim;
    out_pts[i64(lo + u32(p)) * dim + c] = X[c * kFinCap + P[cur][p]];
  }
  for (int p = tid; p < M; p += kFinThreads) {
    const u32 row = __float_as_uint(X[dim * kFinCap + P[cur][p]]);
    out_ids[lo + u32(p)] = ids ? ids[row] : id_base + row;
  }
}

// Row-path LDS finish by rank propagation (the default; k_rr_finish above moves rows instead):
// rows never move. Every level ranks each live row among its sub-segment's sortable rows on
// the level's axis, and the rank alone decides median / left / right, as in the exact builder's
// subtree kernel (build_subtree.hip), with the reference's rules (kdtree_sequential.cpp:46-56):
// a sub-segment's DESIGNATED row (the one in its last slot: the input's last row, or the left
// maximum the parent put there) is not ranked and passes to the right child, which keeps it in
// its last slot; the rank m - 1 row becomes the left child's designated row. A designated row
// stays designated, so every row that is ranked again was ranked at the axis's previous use too.
//   * first use of an axis in the finish: value-linear buckets over the segment's range on
//     the axis, one block scan, bucket-ordered keys, exact (key, row) comparisons in a bucket;
//   * later uses: every ranked row keeps its rank relative to the child it went to (cr, in
//     registers); the ranks of a sub-segment's sortable rows are then distinct and ordered
//     like their keys, so the rank is a popcount prefix over one bitmap per sub-segment
//     (one atomicOr, a wave scan of word popcounts, one read) -- 3 barriers instead of 6.
// Deciding ties: the rows of ranks m - 2 .. m + 1 leave their keys at their sorted slots; the
// median row compares them after the level's closing barrier (the checks k_rr_finish makes).
template <int D>
__global__ __launch_bounds__(kFinThreads) void k_rr_finish_rank(RowCols src, int depth0, i64 n_total, int lf,
                                                                int levels, const u32* __restrict__ ids, u32 id_base,
                                                                float* __restrict__ out_pts, u32* __restrict__ out_ids,
                                                                u32* __restrict__ words) {
  constexpr int T = kFinThreads, I = kFinItems, CAP = kFinCap, NC = D + 1;
  constexpr int kBm = 1024;  // bitmap words of a compressed level (S * Wt above: first-use path)
  extern __shared__ float X[];  // [NC][CAP]
  __shared__ u32 H[CAP + 1 + 64];
  __shared__ u32 bm[2][kBm + 64];
  __shared__ u32 tk[CAP + 64], K[CAP + 64];
  __shared__ unsigned short tp[CAP + 64], fin[CAP + 64];
  __shared__ u32 wsum[T / 64];
  __shared__ u32 rng[D][2];
  u32* ties = words;
  i64 lo64 = 0, m64 = 0;
  seg_geometry(n_total, lf, blockIdx.x, &lo64, &m64);
  if (m64 <= 0) return;
  const int M = int(m64);
  const u32 glo = u32(lo64);
  const int tid = threadIdx.x, ln = dev::lane();
  const u32 dmy = u32(CAP) + u32(ln);  // per-lane dummy word of the H / tk / K / fin arrays
  for (int c = 0; c < NC; ++c)
    for (int p = tid; p < M; p += T) X[c * CAP + p] = src.at(c, glo + u32(p));
  if (tid < D) {
    rng[tid][0] = 0xffffffffu;
    rng[tid][1] = 0u;
  }
  for (int w = tid; w < CAP + 1 + 64; w += T) H[w] = 0u;
  for (int w = tid; w < 2 * (kBm + 64); w += T) (&bm[0][0])[w] = 0u;
  __syncthreads();
  {  // the segment's key range per axis: the first-use buckets' range
    u32 mn[D], mx[D];
#pragma unroll
    for (int c = 0; c < D; ++c) {
      mn[c] = 0xffffffffu;
      mx[c] = 0u;
    }
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int p = tid + i * T;
      if (p < M)
#pragma unroll
        for (int c = 0; c < D; ++c) {
          const u32 k = orderable(X[c * CAP + p]);
          mn[c] = min(mn[c], k);
          mx[c] = max(mx[c], k);
        }
    }
#pragma unroll
    for (int c = 0; c < D; ++c) {
      const u32 a = dev::wave_min_u32(mn[c]), b = dev::wave_max_u32(mx[c]);
      if (ln == 0 && a <= b) {
        atomicMin(&rng[c][0], a);
        atomicMax(&rng[c][1], b);
      }
    }
  }
  u32 lo[I], nn[I], sg[I], cr[I][D];
  bool des[I], live[I], tchk[I];
  u32 tlo[I], tn[I];
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const int p = tid + i * T;
    live[i] = p < M;
    des[i] = p == M - 1;
    lo[i] = 0u;
    nn[i] = u32(M);
    sg[i] = 0u;
    tchk[i] = false;
    tlo[i] = tn[i] = 0u;
#pragma unroll
    for (int c = 0; c < D; ++c) cr[i][c] = 0u;
  }
  __syncthreads();
  int cb = 0;
  for (int l = lf; l < levels; ++l) {
    const int t = l - lf, a = (depth0 + l) % D, S = 1 << t;
    // the previous level's deciding-tie checks (its keys were written before its closing barrier)
#pragma unroll
    for (int i = 0; i < I; ++i) {
      if (!tchk[i]) continue;
      tchk[i] = false;
      const u32 m = tn[i] / 2;
      const u32* kk = K + tlo[i];
      bool tie = kk[m - 1] == kk[m];
      if (m >= 2 && kk[m - 2] == kk[m - 1]) tie = true;
      if (m + 1 <= tn[i] - 2 && kk[m] == kk[m + 1]) tie = true;
      if (tie) note_tie(ties, glo + tlo[i] + m);
    }
    // rows of sub-segments of <= 2 rows are final (2: the designated row keeps the last slot)
    bool srt[I];
    u32 key[I], rank[I];
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int p = tid + i * T;
      if (live[i] && nn[i] <= 2u) {
        fin[lo[i] + ((nn[i] == 2u && des[i]) ? 1u : 0u)] = (unsigned short)p;
        live[i] = false;
      }
      srt[i] = live[i] && !des[i];
      key[i] = srt[i] ? orderable(X[a * CAP + (srt[i] ? p : 0)]) : 0u;
      rank[i] = 0u;
    }
    int Wt = 0;
    if (t >= D) {  // the axis was ranked at level t - D: child-relative ranks < M >> (t - D + 1)
      const u32 bits = u32(M) >> (t - D + 1);
      u32 w = (bits + 31u) / 32u;
      w = w <= 1u ? 1u : 1u << (32 - __clz(w - 1u));
      if (w <= 64u && u32(S) * w <= u32(kBm)) Wt = int(w);
    }
    if (Wt > 0) {
      // ---- compressed: one bitmap of Wt words per sub-segment ----
      u32* b = bm[cb];
      u32 wi[I], c[I];
#pragma unroll
      for (int i = 0; i < I; ++i) {
        u32 v = 0u;
#pragma unroll
        for (int q = 0; q < D; ++q) v = q == a ? cr[i][q] : v;
        c[i] = v;
        wi[i] = srt[i] ? sg[i] * u32(Wt) + (v >> 5) : u32(kBm) + u32(ln);
        if (srt[i]) atomicOr(&b[wi[i]], 1u << (v & 31u));
      }
      __syncthreads();
      for (int w = tid; w < kBm; w += T) bm[cb ^ 1][w] = 0u;  // the next compressed level's bitmaps
      const int nw = S * Wt;
      if (Wt > 1) {  // exclusive popcount prefix inside each group of Wt words (one wave holds a group)
        const u32 g = u32(ln) & u32(Wt - 1);
        for (int w0 = 0; w0 < nw; w0 += T) {
          const int w = w0 + tid;
          const bool in = w < nw;
          const u32 v = in ? u32(__popc(b[w])) : 0u;
          u32 incl = v;
          for (int o = 1; o < Wt; o <<= 1) {
            const u32 tt = __shfl_up(incl, o, 64);
            incl += g >= u32(o) ? tt : 0u;
          }
          tk[in ? u32(w) : dmy] = incl - v;
        }
        __syncthreads();
      }
#pragma unroll
      for (int i = 0; i < I; ++i)
        if (srt[i]) rank[i] = (Wt > 1 ? tk[wi[i]] : 0u) + u32(__popc(b[wi[i]] & ((1u << (c[i] & 31u)) - 1u)));
      cb ^= 1;
    } else {
      // ---- first use: value-linear buckets over the segment's range ----
      const int maxsz = M >> t;
      const int B = maxsz > 16 ? max(1, min(int(1u << (32 - __clz(u32(maxsz) - 1u))), CAP >> t)) : 1;
      const int nb = S * B;  // <= CAP; H[nb] = total after the scan
      const RefBk sc = ref_scale(rng[a][0], rng[a][1], u32(B));
      u32 bk[I], wi[I];
#pragma unroll
      for (int i = 0; i < I; ++i) {
        bk[i] = srt[i] ? sg[i] * u32(B) + (B > 1 ? ref_bucket_s(key[i], sc, u32(B)) : 0u) : dmy + 1u;
        wi[i] = atomicAdd(&H[bk[i]], 1u);
      }
      __syncthreads();
      {  // exclusive scan of H[0, nb): thread t owns H[t * I, + I)
        const int b0 = tid * I;
        u32 x[I], sum = 0;
#pragma unroll
        for (int j = 0; j < I; ++j) {
          x[j] = b0 + j < nb ? H[b0 + j] : 0u;
          sum += x[j];
        }
        const u32 incl = dev::wave_incl_scan(sum);
        if (ln == 63) wsum[tid / 64] = incl;
        __syncthreads();
        const u32 ws = wsum[ln & (T / 64 - 1)];
        const u32 pin = dev::wave_incl_scan(ln < T / 64 ? ws : 0u);
        const int wu = __builtin_amdgcn_readfirstlane(tid / 64);
        const u32 pl = u32(__builtin_amdgcn_readlane(int(pin), wu > 0 ? wu - 1 : 0));
        u32 run = (wu > 0 ? pl : 0u) + incl - sum;
#pragma unroll
        for (int j = 0; j < I; ++j) {
          if (b0 + j < nb) H[b0 + j] = run;
          run += x[j];
        }
        if (tid == T - 1) H[nb] = run;
      }
      __syncthreads();
      u32 st[I], cnt[I];
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int p = tid + i * T;
        st[i] = cnt[i] = 0u;
        if (srt[i]) {
          st[i] = H[bk[i]];
          cnt[i] = H[bk[i] + 1] - st[i];
          rank[i] = st[i] - H[sg[i] * u32(B)];
          tk[st[i] + wi[i]] = key[i];
          tp[st[i] + wi[i]] = (unsigned short)p;
        }
      }
      __syncthreads();
      for (int w = tid; w <= nb; w += T) H[w] = 0u;  // (every read of H is behind the barrier)
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int p = tid + i * T;
        for (u32 j = 0; j < cnt[i]; ++j) {
          const u32 q = st[i] + j;
          const u32 kq = tk[q];
          rank[i] += (kq < key[i] || (kq == key[i] && int(tp[q]) < p)) ? 1u : 0u;
        }
      }
      // tk is read above and rewritten only after the closing barrier (next level)
    }
    // ---- median / left / right ----
#pragma unroll
    for (int i = 0; i < I; ++i) {
      if (!live[i]) continue;
      const int p = tid + i * T;
      const u32 m = nn[i] / 2;
      if (des[i]) {  // to the right child's last slot
        lo[i] += m + 1;
        nn[i] -= m + 1;
        sg[i] = 2 * sg[i] + 1;
        continue;
      }
      const u32 r = rank[i];
      if (r + 2 >= m && r <= m + 1 && r + 2 <= nn[i]) K[lo[i] + r] = key[i];
      if (r == m) {
        fin[lo[i] + m] = (unsigned short)p;
        live[i] = false;
        tchk[i] = true;
        tlo[i] = lo[i];
        tn[i] = nn[i];
      } else {
        const bool right = r > m;
        const u32 v = right ? r - m - 1 : r;
#pragma unroll
        for (int q = 0; q < D; ++q) cr[i][q] = q == a ? v : cr[i][q];
        des[i] = r + 1 == m;
        lo[i] += right ? m + 1 : 0u;
        nn[i] = right ? nn[i] - m - 1 : m;
        sg[i] = 2 * sg[i] + (right ? 1u : 0u);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const int p = tid + i * T;
    if (tchk[i]) {
      const u32 m = tn[i] / 2;
      const u32* kk = K + tlo[i];
      bool tie = kk[m - 1] == kk[m];
      if (m >= 2 && kk[m - 2] == kk[m - 1]) tie = true;
      if (m + 1 <= tn[i] - 2 && kk[m] == kk[m + 1]) tie = true;
      if (tie) note_tie(ties, glo + tlo[i] + m);
    }
    if (live[i]) {
      if (nn[i] <= 2u) fin[lo[i] + ((nn[i] == 2u && des[i]) ? 1u : 0u)] = (unsigned short)p;
      else atomicOr(words + 1, 2u);  // (levels too few for the segment: never with the host's plan)
    }
  }
  __syncthreads();
  for (int e = tid; e < M * D; e += T) {  // rows out: consecutive threads, consecutive floats
    const int p = e / D, c = e - p * D;
    out_pts[i64(glo + u32(p)) * D + c] = X[c * CAP + fin[p]];
  }
  for (int p = tid; p < M; p += T) {
    const u32 row = __float_as_uint(X[D * CAP + fin[p]]);
    out_ids[glo + u32(p)] = ids ? ids[row] : id_base + row;
  }
}

size_t align_up(size_t v) { return (v + 255) / 256 * 256; }
int grid_for(i64 n) { return int(std::min<i64>(8192, std::max<i64>(1, (n + kBlock - 1) / kBlock))); }
int pow2_floor(i64 v) {
  int p = 1;
  while (i64(p) * 2 <= v) p *= 2;
  return p;
}

}  // namespace

ReferenceBuilder::ReferenceBuilder(i64 n, int dim, int depth0) : n_(n), dim_(dim), depth0_(depth0) {
  if (dim <= 0) throw std::invalid_argument("pkdtree: dim must be > 0");
  if (n < 0 || n >= (i64(1) << 32)) throw std::invalid_argument("pkdtree: n must be in [0, 2^32)");
  if (const char* e = std::getenv("PKD_REF_FIN")) fin_rank_ = std::string(e) != "0";  // A/B: 0 = k_rr_finish
  if (const char* e = std::getenv("PKD_REF_BLOCKS")) part_blocks_ = std::max(64, std::min(16384, std::atoi(e)));
  rows_ = dim <= 8;  // rows move as SoA columns; above, only a permutation (keys gathered per level)
  levels_ = 0;
  while ((n_ >> levels_) >= 2) ++levels_;  // the largest segment of level l has n >> l rows
  lfin_ = 0;  // global levels: while the largest segment exceeds the LDS finish
  while (lfin_ < levels_ && (n_ >> lfin_) > kFinCap) ++lfin_;
  i64 max_segs = 1, max_hist = 1, max_parts = 1;
  for (int l = 0; l < lfin_; ++l) {
    RefLevel p;
    p.segs = i64(1) << l;
    // about 8 rows per bucket, so the middle zone (the buckets of ranks m - 1 and m) fits the
    // refine's LDS; the histogram pass runs on 1/8 of the partition's blocks (fewer flushes)
    p.bins = std::max(64, std::min(rows_ ? 16384 : 2048, pow2_floor(std::max<i64>(1, (n_ >> l) / 8))));
    p.bps = int(std::max<i64>(1, std::min<i64>(part_blocks_ / p.segs, ((n_ >> l) + kChunk - 1) / kChunk)));
    p.hbps = int(std::max<i64>(1, std::min<i64>(p.bps, 256 / p.segs)));
    plan_.push_back(p);
    max_segs = std::max(max_segs, p.segs);
    max_hist = std::max(max_hist, p.segs * p.bins);
    max_parts = std::max(max_parts, p.segs * p.bps);  // partition blocks: one PartPartial each
  }
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + std::max<size_t>(bytes, 1));
    return o;
  };
  const size_t nn = size_t(std::max<i64>(n_, 1));
  ncol_ = i64(std::max<size_t>(64, (nn + 63) / 64 * 64));
  if (rows_) {
    off_perm_[0] = take(size_t(dim + 1) * size_t(ncol_) * 4);  // SoA columns (ping)
    off_perm_[1] = take(size_t(dim + 1) * size_t(ncol_) * 4);  // (pong)
    off_keys_ = take(size_t(std::max<i64>(max_parts, max_segs)) * sizeof(PartPartial));  // partition partials
  } else {
    off_perm_[0] = take(nn * 4);
    off_perm_[1] = take(nn * 4);
    off_keys_ = take(nn * 4);
    off_midc_ = take(lfin_ > 0 ? nn * 8 : 8);
  }
  off_hist_ = take(size_t(max_hist) * 4);
  {  // the row path's per-block histogram partials
    i64 hp = 1;
    if (rows_)
      for (const RefLevel& p : plan_)
        if (p.hbps > 1) hp = std::max(hp, p.segs * p.hbps * p.bins);
    off_hpart_ = take(size_t(hp) * 4);
  }
  off_segs_ = take(2 * size_t(max_segs) * sizeof(RefSeg));
  off_words_ = take(size_t(kTieOff + kTieSlots) * 4);  // [0] ties, [1] error, [kTieOff..] tied median slots
  ws_bytes_ = off;
}

std::vector<u32> ReferenceBuilder::read_tie_slots(const void* workspace, hipStream_t stream) const {
  const u32 t = read_ties(workspace, stream);
  std::vector<u32> v(std::min<u32>(t, kTieSlots));
  if (!v.empty()) {
    PKD_HIP_CHECK(hipMemcpyAsync(v.data(), static_cast<const char*>(workspace) + off_words_ + kTieOff * 4,
                                 v.size() * 4, hipMemcpyDeviceToHost, stream));
    PKD_HIP_CHECK(hipStreamSynchronize(stream));
  }
  return v;
}

u32 ReferenceBuilder::read_ties(const void* workspace, hipStream_t stream) const {
  u32 w[4] = {0, 0, 0, 0};
  if (n_ == 0) return 0;
  PKD_HIP_CHECK(hipMemcpyAsync(w, static_cast<const char*>(workspace) + off_words_, 16, hipMemcpyDeviceToHost, stream));
  PKD_HIP_CHECK(hipStreamSynchronize(stream));
  if (w[1]) throw std::runtime_error("pkdtree: reference build inconsistency (histogram select)");
  return w[0];
}

void ReferenceBuilder::build(const float* pts, const u32* ids, u32 id_base, float* out_pts, u32* out_ids,
                             void* workspace, hipStream_t stream) const {
  if (n_ == 0) return;
  char* ws = static_cast<char*>(workspace);
  u32* hist = reinterpret_cast<u32*>(ws + off_hist_);
  i64 max_segs = 1;
  for (const RefLevel& p : plan_) max_segs = std::max(max_segs, p.segs);
  RefSeg* segs[2] = {reinterpret_cast<RefSeg*>(ws + off_segs_), reinterpret_cast<RefSeg*>(ws + off_segs_) + max_segs};
  u32* words = reinterpret_cast<u32*>(ws + off_words_);
  PKD_HIP_CHECK(hipMemsetAsync(words, 0, 16, stream));
  const int g = grid_for(n_);
  auto seg_init = [&](RefSeg* sg, const RefLevel& p, int l, i64 hw) {
    k_ref_seg_init<<<int(std::min<i64>(1024, (std::max<i64>(hw, p.segs) + kBlock - 1) / kBlock)), kBlock, 0, stream>>>(
        sg, p.segs, n_, l, hist, hw);
    PKD_LAUNCH_CHECK();
  };
  if (rows_) {
    auto* partials = reinterpret_cast<PartPartial*>(ws + off_keys_);
    RowCols cols[2] = {{reinterpret_cast<float*>(ws + off_perm_[0]), ncol_},
                       {reinterpret_cast<float*>(ws + off_perm_[1]), ncol_}};
    const int NC = dim_ + 1;
    if (lfin_ > 0) seg_init(segs[0], plan_[0], 0, 0);
    k_rr_prep<<<std::min(g, 1024), kBlock, 0, stream>>>(pts, n_, dim_, depth0_ % dim_, cols[0],
                                                        lfin_ > 0 ? segs[0] : nullptr);
    PKD_LAUNCH_CHECK();
    int cur = 0;
    for (int l = 0; l < lfin_; ++l) {
      const RefLevel& p = plan_[size_t(l)];
      const int axis = (depth0_ + l) % dim_, naxis = (depth0_ + l + 1) % dim_;
      const int S = int(p.segs);
      RefSeg* sg = segs[l & 1];
      RefSeg* nsg = l + 1 < lfin_ ? segs[(l + 1) & 1] : nullptr;
      // this level's histogram (stored whole: no zeroing), the buckets of ranks m - 1 and m, and
      // the next level's descriptors (their key ranges are filled in by this level's refine)
      ensure_dynamic_lds(reinterpret_cast<const void*>(&k_rr_hist), p.bins * 4);
      if (p.hbps == 1) {  // one block per segment: the select runs in the histogram block
        k_rr_hist<<<S, kBlock, size_t(p.bins) * 4, stream>>>(cols[cur], axis, sg, 1, p.bins, hist, words + 1, nsg, 1);
        PKD_LAUNCH_CHECK();
      } else {
        u32* hpart = reinterpret_cast<u32*>(ws + off_hpart_);
        k_rr_hist<<<S * p.hbps, kBlock, size_t(p.bins) * 4, stream>>>(cols[cur], axis, sg, p.hbps, p.bins, hpart,
                                                                      words + 1, nsg, 0);
        PKD_LAUNCH_CHECK();
        const i64 tot = p.segs * p.bins;
        k_rr_hred<<<int((tot + kBlock - 1) / kBlock), kBlock, 0, stream>>>(hpart, p.hbps, p.bins, tot, hist);
        PKD_LAUNCH_CHECK();
        k_ref_select<<<S, kBlock, 0, stream>>>(sg, p.bins, hist, words + 1, nsg);
        PKD_LAUNCH_CHECK();
      }
      switch (NC) {
#define PKD_RR(N) \
  case N: k_rr_part<N><<<S * p.bps, kBlock, 0, stream>>>(cols[cur], cols[cur ^ 1], axis, naxis, sg, p.bps, p.bins, partials); break;
        PKD_RR(2) PKD_RR(3) PKD_RR(4) PKD_RR(5) PKD_RR(6) PKD_RR(7) PKD_RR(8) default: PKD_RR(9)
#undef PKD_RR
      }
      PKD_LAUNCH_CHECK();
      {  // middle zones of <= 64 rows by one wave each (4 per block), the rest by a block each
        const int gsm = (S + kBlock / 64 - 1) / (kBlock / 64);
        switch (NC) {
#define PKD_RF(N)                                                                                                      \
  case N:                                                                                                              \
    k_rr_refine<N><<<gsm + S, kBlock, 0, stream>>>(cols[cur], cols[cur ^ 1], dim_, axis, naxis, sg, nsg, partials,     \
                                                   p.bps, ids, id_base, out_pts, out_ids, words, S, gsm);              \
    break;
          PKD_RF(2) PKD_RF(3) PKD_RF(4) PKD_RF(5) PKD_RF(6) PKD_RF(7) PKD_RF(8) default: PKD_RF(9)
#undef PKD_RF
        }
      }
      PKD_LAUNCH_CHECK();
      cur ^= 1;
    }
    const i64 segs_f = i64(1) << lfin_;
    const size_t lds = size_t(NC) * kFinCap * 4;
    if (fin_rank_) {
      switch (NC) {
#define PKD_RFR(N)                                                                                                    \
  case N:                                                                                                             \
    ensure_dynamic_lds(reinterpret_cast<const void*>(&k_rr_finish_rank<N - 1>), int(lds));                           \
    k_rr_finish_rank<N - 1><<<int(segs_f), kFinThreads, lds, stream>>>(cols[cur], depth0_, n_, lfin_, levels_, ids,  \
                                                                       id_base, out_pts, out_ids, words);            \
    break;
        PKD_RFR(2) PKD_RFR(3) PKD_RFR(4) PKD_RFR(5) PKD_RFR(6) PKD_RFR(7) PKD_RFR(8) default: PKD_RFR(9)
#undef PKD_RFR
      }
    } else {
      ensure_dynamic_lds(reinterpret_cast<const void*>(&k_rr_finish), int(lds));
      k_rr_finish<<<int(segs_f), kFinThreads, lds, stream>>>(cols[cur], dim_, depth0_, n_, lfin_, levels_, ids,
                                                             id_base, out_pts, out_ids, words);
    }
    PKD_LAUNCH_CHECK();
    return;
  }
  u32* perm[2] = {reinterpret_cast<u32*>(ws + off_perm_[0]), reinterpret_cast<u32*>(ws + off_perm_[1])};
  u32* keys = reinterpret_cast<u32*>(ws + off_keys_);
  u64* midc = reinterpret_cast<u64*>(ws + off_midc_);
  k_ref_init<<<g, kBlock, 0, stream>>>(perm[0], n_);
  PKD_LAUNCH_CHECK();
  int cur = 0;
  for (int l = 0; l < lfin_; ++l) {
    const RefLevel& p = plan_[size_t(l)];
    const int axis = (depth0_ + l) % dim_;
    const int S = int(p.segs), grid = S * p.bps;
    seg_init(segs[0], p, l, p.segs * p.bins);
    k_ref_keys<<<grid, kBlock, 0, stream>>>(pts, dim_, axis, perm[cur], segs[0], p.bps, keys);
    PKD_LAUNCH_CHECK();
    k_ref_hist<<<grid, kBlock, size_t(p.bins) * 4, stream>>>(keys, segs[0], p.bps, p.bins, hist);
    PKD_LAUNCH_CHECK();
    k_ref_select<<<S, kBlock, 0, stream>>>(segs[0], p.bins, hist, words + 1, nullptr);
    PKD_LAUNCH_CHECK();
    k_ref_part<<<grid, kBlock, 0, stream>>>(keys, perm[cur], perm[cur ^ 1], midc, segs[0], p.bps, p.bins);
    PKD_LAUNCH_CHECK();
    k_ref_refine<<<S, kBlock, 0, stream>>>(segs[0], midc, perm[cur ^ 1], perm[cur], words);
    PKD_LAUNCH_CHECK();
    cur ^= 1;
  }
  if (lfin_ < levels_) {
    const i64 segs_f = i64(1) << lfin_;
    k_ref_finish<<<int(segs_f), kFinThreads, 0, stream>>>(pts, dim_, depth0_, perm[cur], n_, lfin_, levels_, words);
    PKD_LAUNCH_CHECK();
  }
  k_ref_gather<<<int(std::min<i64>(4096, std::max<i64>(1, (n_ * dim_ + 4 * kBlock - 1) / (4 * kBlock)))), kBlock, 0,
                 stream>>>(pts, ids, id_base, dim_, perm[cur], n_, out_pts, out_ids);
  PKD_LAUNCH_CHECK();
}

namespace {
// Host-decided slots of a repaired reference tree: slot slots[k] takes input row rows[k].
__global__ __launch_bounds__(kBlock) void k_ref_patch(const float* __restrict__ pts, const u32* __restrict__ ids,
                                                      u32 id_base, int dim, const u32* __restrict__ slots,
                                                      const u32* __restrict__ rows, i64 count,
                                                      float* __restrict__ out_pts, u32* __restrict__ out_ids) {
  const i64 total = count * i64(dim);
  for (i64 e = i64(blockIdx.x) * kBlock + threadIdx.x; e < total; e += i64(gridDim.x) * kBlock) {
    const i64 k = e / dim;
    const int c = int(e - k * dim);
    const u32 r = rows[k], sl = slots[k];
    out_pts[i64(sl) * dim + c] = pts[i64(r) * dim + c];
    if (c == 0) out_ids[sl] = ids ? ids[r] : id_base + r;
  }
}
}  // namespace

void reference_patch(const float* pts, const u32* ids, u32 id_base, int dim, const u32* slots, const u32* rows,
                     i64 count, float* out_pts, u32* out_ids, hipStream_t stream) {
  if (count <= 0) return;
  const int g = int(std::min<i64>(4096, (count * dim + kBlock - 1) / kBlock));
  k_ref_patch<<<g, kBlock, 0, stream>>>(pts, ids, id_base, dim, slots, rows, count, out_pts, out_ids);
  PKD_LAUNCH_CHECK();
}

namespace {
__global__ __launch_bounds__(kBlock) void k_ref_keys_of_levels(const float* __restrict__ pts, i64 n, int dim,
                                                               int depth0, int levels, float* __restrict__ out) {
  const i64 total = n * i64(levels);
  for (i64 e = i64(blockIdx.x) * kBlock + threadIdx.x; e < total; e += i64(gridDim.x) * kBlock) {
    const i64 r = e / levels;
    const int d = int(e - r * levels);
    out[e] = pts[r * dim + (depth0 + d) % dim];
  }
}
}  // namespace

void reference_level_keys(const float* pts, i64 n, int dim, int depth0, int levels, float* out, hipStream_t stream) {
  if (n <= 0 || levels <= 0) return;
  const int g = int(std::min<i64>(8192, (n * levels + kBlock - 1) / kBlock));
  k_ref_keys_of_levels<<<g, kBlock, 0, stream>>>(pts, n, dim, depth0, levels, out);
  PKD_LAUNCH_CHECK();
}

}  // namespace pkdtree
