// Sampled top levels (levels 0..3 in one row-moving pass): see top4.hpp for the scheme.
//
// Kernel sequence of one build (all on the caller's stream, no host round trip, graph-safe):
//   k_samp_gather   2^sample_log2 stratified random rows: the keys of the four level axes, and
//                   per-block key ranges; zeroes the state and histograms
//   k_samp_hist/sel per level: histogram of the node's sample keys (kSampBins >> j bins per node,
//                   linear in the key value over the node's sample range), then per node the
//                   bins of the sample ranks c/2 - h, c/2, c/2 + h (h = z sqrt(c) / 2): band
//                   [a, b] and the estimated pivot that routes the sample to the children
//   k_scatter       every input row once: certain rows into their level-4 segment, band rows
//                   into the staging arena (tag = node), SoA columns + ids, bounding box
//   per level j:    k_res_classify (route the staged rows by level j-1's exact pivot, classify
//                   the level-j ones against the band, kResBins >> j-bin histogram of the band
//                   rows' keys), k_res_sel1 (exact rank of the median in the band from the
//                   counts; its bin), k_res_collect (the bin's rows), k_res_sel2 (radix select
//                   on the (key, id) composites: the exact pivot)
//   k_res_insert    staged rows into the free slots of their level-4 segments
//   k_finish        bounding box, the 15 medians to the output, cells of nodes 0..30, the
//                   level-4 histogram parameters, consistency checks
//
// Histograms are built in LDS per workgroup and flushed with lane-contiguous atomics (one
// 256-B wave-instruction per 64 bins): scattered one-lane-per-bin global atomics run an order
// of magnitude below that rate on MI355X (they execute at the memory side), and were what
// bounded the first version of these kernels. Row moves (scatter, insert) rank rows per zone
// with wave ballots (no same-address LDS atomics) and reorder each tile through LDS, so every
// zone's rows leave the workgroup as contiguous runs instead of 16-B fragments.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <stdexcept>

#include "device_utils.hpp"
#include "pkdtree/hip_check.hpp"
#include "top4.hpp"

namespace pkdtree {
namespace top4 {
namespace {

constexpr int kBlock = 256;
constexpr int kSampBins = 1 << 14;   // sample histogram entries per level: kSampBins >> j per node
constexpr int kResBins = 1 << 13;    // resolution histogram entries per level
constexpr int kHistThreads = 1024;   // workgroup of the LDS histogram kernels
constexpr int kSampBlocks = 64;
constexpr int kResBlocks = 256;
constexpr int kSmallCap = 4096;      // rows of a median's bin selected in LDS
constexpr i64 kStreamCap = i64(1) << 20;  // staged rows a one-workgroup select over the arena may stream
constexpr u32 kMed = 0x80000000u;    // tag of a median row: kMed | node
constexpr int kMaxParts = 2048;      // scatter blocks (one bounding-box partial each)
constexpr int kMaxSampleLog2 = 21;
constexpr int kGatherRows = 4;       // sample rows per gather thread
constexpr int kMaxGather = (1 << kMaxSampleLog2) / (kBlock * kGatherRows);

__host__ __device__ constexpr int samp_bins(int j) { return kSampBins >> j; }
__host__ __device__ constexpr int res_bins(int j) { return kResBins >> j; }

struct State {
  u32 nbox_lo[8];  // ~(min sample key) per axis (0: none)
  u32 box_hi[8];   // max sample key per axis
  u32 rlo[kNodes], rhi[kNodes];             // sample range of the node on its axis (bins: sample_params)
  u32 scount[kNodes];
  u32 a[kNodes], b[kNodes], phat[kNodes];  // band (inclusive, orderable keys), estimated pivot
  dev::BucketParams bparam[kNodes];         // bin of a band row: bucket_of(key) over the band
  u32 staged_orig[kNodes];                  // rows the scatter staged at the node
  u32 late[kNodes][3];                      // staged rows of the node: left of / in / right of the band
  u32 sel[kNodes], sel_rank[kNodes], sel_cnt[kNodes], small_cnt[kNodes];
  u32 med_idx1[kNodes];                     // staging row + 1 of the median (0: not found)
  u32 cursor[kCells + 1];                   // rows the scatter put in each level-4 segment; [16]: staged
  u32 ins[kCells];                          // staged rows inserted per segment
  u32 pad[2];
  u64 pivot[kNodes];                        // exact (key, id) composite of the node's median
};

struct Layout {
  size_t state, fine_s, fine_r, zero_end, skey, gpart, small, part, total;
};

inline size_t al(size_t x) { return (x + 255) / 256 * 256; }

Layout layout() {
  Layout L{};
  size_t o = 0;
  L.state = o;
  o = al(o + sizeof(State));
  L.fine_s = o;
  o = al(o + size_t(kLevels) * kSampBins * 4);
  L.fine_r = o;
  o = al(o + size_t(kLevels) * kResBins * 4);
  L.zero_end = o;
  L.skey = o;
  o = al(o + size_t(kLevels) * (size_t(1) << kMaxSampleLog2) * 4);
  L.gpart = o;
  o = al(o + size_t(kMaxGather) * 2 * kLevels * 4);
  L.small = o;
  o = al(o + size_t(8) * kSmallCap * 8);
  L.part = o;
  o = al(o + size_t(kMaxParts) * 16 * 4);
  L.total = o;
  return L;
}

__device__ __forceinline__ int heap_level(u32 h) { return 31 - __builtin_clz(h + 1u); }

// Histogram bins linear in the key's VALUE over [lo, hi] (orderable keys): occupancy follows
// the data, not the float exponent.
__device__ __forceinline__ dev::BucketParams sample_params(u32 lo, u32 hi, int bins) {
  return dev::make_params(from_orderable(lo), from_orderable(hi), bins);
}
// A key below every value of bins >= b (b > 0) and one above every value of bins <= b: the
// float edge of the bin widened by a margin that covers the bucketing's rounding.
__device__ __forceinline__ u32 key_below_bin(dev::BucketParams p, u32 b, float span) {
  const float e = p.lo + float(b) / p.scale;
  return orderable(e - (fabsf(e) * 1e-5f + span * 1e-6f));
}
__device__ __forceinline__ u32 key_above_bin(dev::BucketParams p, u32 b, float span) {
  const float e = p.lo + float(b + 1) / p.scale;
  return orderable(e + (fabsf(e) * 1e-5f + span * 1e-6f));
}

__device__ __forceinline__ u32 mix32(u32 x) {  // murmur3 finaliser
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// Bin of the rank-th element (0-based) of a 256-bin histogram h (16-B aligned, global or
// LDS); every lane of the wave calls it. *below = elements in the bins before it, *total = all
// elements; returns 256 when rank >= total.
__device__ __forceinline__ u32 wave_find256(const u32* h, u32 rank, u32* below, u32* total) {
  const int ln = dev::lane();
  const uint4 v = reinterpret_cast<const uint4*>(h)[ln];
  const u32 s = v.x + v.y + v.z + v.w;
  const u32 incl = dev::wave_incl_scan(s);
  const u32 excl = incl - s;
  const u32 tot = __shfl(incl, 63, 64);
  const bool mine = rank >= excl && rank < incl;
  const u64 m = __ballot(mine);
  u32 bin = 256, bel = tot;
  if (m) {
    const int src = __ffsll((long long)m) - 1;
    u32 lb = 0, c = excl;
    if (mine) {
      if (rank >= c + v.x) {
        c += v.x;
        lb = 1;
        if (rank >= c + v.y) {
          c += v.y;
          lb = 2;
          if (rank >= c + v.z) {
            c += v.z;
            lb = 3;
          }
        }
      }
    }
    bin = u32(__shfl(int(4 * ln + lb), src, 64));
    bel = u32(__shfl(int(c), src, 64));
  }
  *below = bel;
  *total = tot;
  return bin;
}

// Entry of h[0, n) (n <= 64) holding the rank-th element; *below = elements before it.
__device__ __forceinline__ u32 wave_find_small(const u32* h, int n, u32 rank, u32* below) {
  const int ln = dev::lane();
  const u32 v = ln < n ? h[ln] : 0u;
  const u32 incl = dev::wave_incl_scan(v);
  const u32 excl = incl - v;
  const u64 m = __ballot(rank >= excl && rank < incl);
  if (!m) {
    *below = __shfl(incl, 63, 64);
    return u32(n);
  }
  const int src = __ffsll((long long)m) - 1;
  *below = u32(__shfl(int(excl), src, 64));
  return u32(src);
}

// Coarse sums of a node's F = 256 * gs bin histogram into co[256] (LDS): every thread of a
// kBlock workgroup calls it; the caller synchronises before reading co.
__device__ __forceinline__ void coarse_of(const u32* fine, int gs, u32* co) {
  const int t = threadIdx.x;
  u32 s = 0;
  static_assert(kSampBins / 256 <= 64 && kResBins / 256 <= 64, "coarse_of: at most 16 16-B loads per thread");
  if (gs % 4 == 0) {  // 16-B loads, all in flight (gs <= 64: at most 16 per thread)
    const uint4* f4 = reinterpret_cast<const uint4*>(fine + t * gs);
    uint4 v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = e < gs / 4 ? f4[e] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int e = 0; e < 16; ++e) s += v[e].x + v[e].y + v[e].z + v[e].w;
  } else {
    for (int e = 0; e < gs; ++e) s += fine[t * gs + e];
  }
  co[t] = s;
}

// Bin (of 256 * gs) holding the rank-th element, from the coarse sums and the fine bins (wave).
__device__ __forceinline__ u32 wave_find_fine(const u32* co, const u32* fine, int gs, u32 rank, u32* below,
                                              u32* total) {
  u32 b1 = 0, b2 = 0;
  const u32 cb = wave_find256(co, rank, &b1, total);
  if (cb >= 256) {
    *below = *total;
    return u32(256 * gs);
  }
  const u32 fb = wave_find_small(fine + size_t(cb) * gs, gs, rank - b1, &b2);
  *below = b1 + b2;
  return cb * u32(gs) + min(fb, u32(gs - 1));
}

__device__ __forceinline__ u32 wave_sum(u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += u32(__shfl_xor(int(v), o, 64));
  return v;
}

// Lanes of the wave in the same zone as this one (valid lanes only; zones < 2^BITS).
template <int BITS>
__device__ __forceinline__ u64 match_zone(u32 z, bool valid) {
  u64 m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const bool bit = (z >> b) & 1u;
    const u64 bb = __ballot(bit);
    m &= bit ? bb : ~bb;
  }
  return m;
}

// Rank of this lane's row among the wave's rows of its zone so far; wc = the wave's own zone
// counters in LDS (no other wave touches them until the next barrier).
template <int BITS>
__device__ __forceinline__ u32 wave_rank(u32 z, bool valid, u32* wc) {
  const u64 m = match_zone<BITS>(z, valid);
  const u32 below = dev::mbcnt(m);
  u32 r = 0;
  if (valid) {
    const u32 before = wc[z];
    r = before + below;
    if (below == 0) wc[z] = before + u32(__popcll(m));
  }
  return r;
}

// Per-tile zone bookkeeping of an LDS reorder (NH parts of a tile, NZ zones, 4 waves).
template <int NZ, int NH>
struct Reorder {
  u32 wc[NH][4][NZ];  // per-wave zone counts; offsets of the wave's rows after scan()
  u32 hoff[NH][NZ];   // LDS position of zone z's first row in part h
  u32 hcnt[NH];       // rows of part h
  u32 gbase[NH][NZ];  // destination index of zone z's first row of part h
};

// Wave 0: per-wave offsets, LDS zone offsets, and one reservation per zone for the whole tile
// (base = reserve(z, rows)); the caller brackets it with barriers.
template <int NZ, int NH, class Reserve>
__device__ __forceinline__ void reorder_scan(Reorder<NZ, NH>& s, Reserve reserve) {
  static_assert(NZ <= 32 && NH <= 2, "reorder: 32 zones, 2 parts");
  if (threadIdx.x >= 64) return;
  const int l = threadIdx.x, h = l >> 5, z = l & 31;
  const bool ok = h < NH && z < NZ;
  u32 c = 0;
  if (ok) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const u32 t = s.wc[h][w][z];
      s.wc[h][w][z] = c;
      c += t;
    }
  }
  const u32 incl = dev::wave_incl_scan(c);
  const u32 tot0 = __shfl(incl, 31, 64);
  const u32 excl = incl - c - (h ? tot0 : 0u);
  const u32 c1 = u32(__shfl(int(c), (l + 32) & 63, 64));
  if (ok) {
    s.hoff[h][z] = excl;
    if (z == NZ - 1) s.hcnt[h] = excl + c;
  }
  if (h == 0 && z < NZ) {
    const u32 base = reserve(z, c + c1);
    s.gbase[0][z] = base;
    if (NH > 1) s.gbase[NH - 1][z] = base + c;
  }
}

__device__ __forceinline__ void report(u32* err, u32 code, u32 t, u32 v) {
  atomicOr(err, kErrBit);
  if (atomicCAS(err + 1, 0u, code) == 0u) {
    err[2] = t;
    err[3] = v;
  }
}

// ---- sample -----------------------------------------------------------------------------
struct SampArgs {
  const float* pts;      // AoS input, or nullptr: columns
  const float* in_cols;  // SoA input columns (stride in_ncol) when pts is null
  i64 in_ncol;
  int dim;
  i64 n;
  int S;
  int ax[kLevels];
  u32* skey;   // [kLevels][S]
  u32* gpart;  // [gather blocks][2 kLevels]: per-block min / max key of each level's axis
  u32* zero;   // the state and histograms, zeroed here as well (no kernel of their own)
  i64 zwords;
  u32 salt;    // per-build: the sample positions (and so a band miss) are never fixed by the input
};

__global__ __launch_bounds__(kBlock) void k_samp_gather(SampArgs a) {
  for (i64 i = i64(blockIdx.x) * kBlock + threadIdx.x; i < a.zwords; i += i64(gridDim.x) * kBlock) a.zero[i] = 0u;
  __shared__ u32 red[kBlock / 64][2 * kLevels];
  u32 mn[kLevels], mx[kLevels];
#pragma unroll
  for (int j = 0; j < kLevels; ++j) {
    mn[j] = 0xffffffffu;
    mx[j] = 0u;
  }
  float v[kGatherRows][kLevels];
  int kk[kGatherRows];
#pragma unroll
  for (int u = 0; u < kGatherRows; ++u) {  // all loads first: the rows are independent
    const int k = (blockIdx.x * kGatherRows + u) * kBlock + threadIdx.x;
    kk[u] = k;
    const int kc = k < a.S ? k : a.S - 1;
    const i64 w0 = (i64(kc) * a.n) / a.S, w1 = (i64(kc + 1) * a.n) / a.S;
    const u32 win = u32(max<i64>(1, w1 - w0));
    const i64 r = w0 + i64(mix32(u32(kc) * 0x9e3779b9u + 0x7f4a7c15u + mix32(a.salt)) % win);
#pragma unroll
    for (int j = 0; j < kLevels; ++j) v[u][j] = a.pts ? a.pts[r * a.dim + a.ax[j]] : a.in_cols[a.ax[j] * a.in_ncol + r];
  }
#pragma unroll
  for (int u = 0; u < kGatherRows; ++u) {
    if (kk[u] >= a.S) continue;
#pragma unroll
    for (int j = 0; j < kLevels; ++j) {
      const u32 key = orderable(v[u][j]);
      a.skey[size_t(j) * a.S + kk[u]] = key;
      mn[j] = min(mn[j], key);
      mx[j] = max(mx[j], key);
    }
  }
  const int w = threadIdx.x / 64;
#pragma unroll
  for (int j = 0; j < kLevels; ++j) {
    const u32 lo = dev::wave_min_u32(mn[j]), hi = dev::wave_max_u32(mx[j]);
    if (dev::lane() == 0) {
      red[w][j] = lo;
      red[w][kLevels + j] = hi;
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * kLevels) {
    const int c = threadIdx.x;
    u32 r = red[0][c];
    for (int k = 1; k < kBlock / 64; ++k) r = c < kLevels ? min(r, red[k][c]) : max(r, red[k][c]);
    a.gpart[size_t(blockIdx.x) * 2 * kLevels + c] = r;
  }
}

struct SampLevelArgs {
  const u32* skey;
  const u32* gpart;
  int gblocks;
  int S;
  int j;
  int ax[kLevels + 1];
  State* st;
  u32* fine;  // [kLevels][kSampBins]: level j, node x at j * kSampBins + x * samp_bins(j)
  float z;
};

// LDS histogram of a contiguous share of the sample (every key routed to its level-j node by
// the estimated pivots), flushed with lane-contiguous atomics.
__global__ __launch_bounds__(kHistThreads) void k_samp_hist(SampLevelArgs a) {
  __shared__ u32 h[kSampBins];
  __shared__ u32 ph[kNodes], rl[8], rh[8];
  __shared__ dev::BucketParams bp[8];
  __shared__ u32 red[kHistThreads / 64][2 * kLevels];
  __shared__ u32 sbl[2 * kLevels];
  const int j = a.j, nodes = 1 << j, first = nodes - 1, F = samp_bins(j);
  const int tid = threadIdx.x;
  for (int i = tid; i < kSampBins; i += kHistThreads) h[i] = 0u;
  if (j == 0) {  // the sample's key range per level axis, from the gather blocks' partials
#pragma unroll
    for (int c = 0; c < 2 * kLevels; ++c) {
      u32 r = c < kLevels ? 0xffffffffu : 0u;
      for (int p = tid; p < a.gblocks; p += kHistThreads) {
        const u32 v = a.gpart[size_t(p) * 2 * kLevels + c];
        r = c < kLevels ? min(r, v) : max(r, v);
      }
      r = c < kLevels ? dev::wave_min_u32(r) : dev::wave_max_u32(r);
      if (dev::lane() == 0) red[tid / 64][c] = r;
    }
    __syncthreads();
    if (tid < 2 * kLevels) {
      u32 r = red[0][tid];
      for (int k = 1; k < kHistThreads / 64; ++k) r = tid < kLevels ? min(r, red[k][tid]) : max(r, red[k][tid]);
      sbl[tid] = r;
    }
  }
  if (tid < first) ph[tid] = a.st->phat[tid];
  __syncthreads();
  if (j == 0 && blockIdx.x == 0 && tid < 8) {  // per axis over the levels that split on it
    u32 mn = 0xffffffffu, mx = 0u;
    bool any = false;
    for (int l = 0; l < kLevels; ++l)
      if (a.ax[l] == tid) {
        mn = min(mn, sbl[l]);
        mx = max(mx, sbl[kLevels + l]);
        any = true;
      }
    if (any) {
      a.st->nbox_lo[tid] = ~mn;
      a.st->box_hi[tid] = mx;
    }
  }
  if (tid < nodes) {
    const int X = first + tid;
    u32 lo, hi;
    if (j == 0) {
      lo = sbl[0];
      hi = sbl[kLevels];
      if (hi < lo) hi = lo;
      if (blockIdx.x == 0) {
        a.st->rlo[0] = lo;
        a.st->rhi[0] = hi;
      }
    } else {
      lo = a.st->rlo[X];
      hi = a.st->rhi[X];
    }
    rl[tid] = lo;
    rh[tid] = hi;
    bp[tid] = sample_params(lo, hi, F);
  }
  __syncthreads();
  const int per = (a.S + int(gridDim.x) - 1) / int(gridDim.x);
  const int k0 = int(blockIdx.x) * per, k1 = min(a.S, k0 + per);
  for (int k = k0 + tid; k < k1; k += kHistThreads) {
    int X = 0;
    for (int i = 0; i < j; ++i) X = 2 * X + 1 + (a.skey[size_t(i) * a.S + k] >= ph[X] ? 1 : 0);
    const int x = X - first;
    u32 key = a.skey[size_t(j) * a.S + k];
    key = min(max(key, rl[x]), rh[x]);
    atomicAdd(&h[x * F + int(dev::bucket_of(from_orderable(key), bp[x], F))], 1u);
  }
  __syncthreads();
  u32* out = a.fine + size_t(j) * kSampBins;
  for (int i = tid; i < kSampBins; i += kHistThreads) {
    const u32 v = h[i];
    if (v) atomicAdd(&out[i], v);
  }
}

// One workgroup per node of level j: the band and estimated pivot from the sample ranks, then
// the children's sample ranges (the root box on their axis, clipped by every ancestor pivot on it).
__global__ __launch_bounds__(kBlock) void k_samp_sel(SampLevelArgs a) {
  __shared__ __align__(16) u32 co[256];
  const int j = a.j, first = (1 << j) - 1, F = samp_bins(j), gs = F / 256;
  const int X = first + blockIdx.x;
  const u32* fi = a.fine + size_t(j) * kSampBins + size_t(blockIdx.x) * F;
  coarse_of(fi, gs, co);
  __syncthreads();
  if (threadIdx.x >= 64) return;
  State* st = a.st;
  const u32 lo = st->rlo[X], hi = st->rhi[X];
  const dev::BucketParams bp = sample_params(lo, hi, F);
  const float span = from_orderable(hi) - from_orderable(lo);
  u32 below = 0, c = 0;
  (void)wave_find256(co, 0, &below, &c);
  u32 A = 0, B = 0xffffffffu, P = lo;
  if (c > 0) {
    const u32 half = u32(ceilf(a.z * sqrtf(float(c)) * 0.5f)) + 2u;
    const u32 rm = c / 2, rlo = rm > half ? rm - half : 0u, rhi = min(c - 1, rm + half);
    u32 t = 0;
    const u32 bl = wave_find_fine(co, fi, gs, rlo, &below, &t);
    const u32 bm = wave_find_fine(co, fi, gs, rm, &below, &t);
    const u32 bh = wave_find_fine(co, fi, gs, rhi, &below, &t);
    // the band: from below every sample of bin bl to above every sample of bin bh (open
    // ended where the sample rank range reaches the node's first / last sample, or the edge bins)
    const bool zero_span = !(bp.scale > 0.0f);
    A = (rlo == 0 || bl == 0 || zero_span) ? 0u : min(key_below_bin(bp, bl, span), hi);
    B = (rhi >= c - 1 || bh >= u32(F - 1) || zero_span) ? 0xffffffffu : max(key_above_bin(bp, bh, span), lo);
    P = zero_span ? lo : min(max(orderable(bp.lo + (float(bm) + 0.5f) / bp.scale), lo), hi);
  }
  if (dev::lane() == 0) {
    st->scount[X] = c;
    st->a[X] = A;
    st->b[X] = B;
    st->phat[X] = P;
    // bin of a band row: its key's value bin over the band (open ends: the node's sample
    // range; keys beyond it fall into the edge bins)
    st->bparam[X] = dev::make_params(from_orderable(A == 0 ? lo : A), from_orderable(B == 0xffffffffu ? hi : B),
                                     res_bins(j));
    if (j + 1 < kLevels) {
      const int ac = a.ax[j + 1];
      for (int s = 0; s < 2; ++s) {
        const int C = 2 * X + 1 + s;
        u32 clo2 = ~st->nbox_lo[ac], chi2 = st->box_hi[ac];
        int child = C, Y = X;
        for (;;) {
          if (a.ax[heap_level(u32(Y))] == ac) {
            const u32 pY = Y == X ? P : st->phat[Y];
            if (child == 2 * Y + 1) chi2 = min(chi2, pY > 0 ? pY - 1 : 0u);
            else clo2 = max(clo2, pY);
          }
          if (Y == 0) break;
          child = Y;
          Y = (Y - 1) / 2;
        }
        if (chi2 < clo2) chi2 = clo2;
        st->rlo[C] = clo2;
        st->rhi[C] = chi2;
      }
    }
  }
}

// ---- scatter ----------------------------------------------------------------------------
struct ScatArgs {
  const float* pts;      // AoS input, or nullptr: the SoA columns below (ids in column dim)
  const float* in_cols;
  i64 in_ncol;
  const u32* ids;
  u32 id_base;
  i64 n;
  float* cols;
  float* stage;
  u32* tags;
  i64 ncol;
  State* st;
  u32* part;
  u32* err;
  i64 tiles;
  i64 cell_lo[kCells];
  u32 cell_n[kCells];
  int ax[kLevels];
  int diag;  // timing diagnostics (output garbage): 2 no reservation atomics, 3 no stores
};

// Rows of one scatter tile held by a thread: v[u][c], id[u]; VEC (dim 3, 16-B aligned input):
// 4 consecutive rows per quad from three 16-B loads (rows 4 q .. 4 q + 3, q = tile quad base +
// u4 * kBlock + tid); otherwise row t0 + u * kBlock + tid.
template <int D, int R, bool VEC>
__device__ __forceinline__ u32 load_tile(const ScatArgs& a, i64 t0, float (&v)[R][D], u32 (&id)[R]) {
  u32 valid = 0;  // bit u: row u of this thread exists
  const int tid = threadIdx.x;
  if constexpr (VEC) {
    static_assert(D == 3 && R % 4 == 0, "vector tile: dim 3");
    const i64 q0 = t0 / 4;
    const float4* in = reinterpret_cast<const float4*>(a.pts);
#pragma unroll
    for (int u4 = 0; u4 < R / 4; ++u4) {
      const i64 q = q0 + i64(u4) * kBlock + tid;
      const i64 r0 = 4 * q;
      if (r0 + 3 < a.n) {
        const float4 x = in[3 * q], y = in[3 * q + 1], z = in[3 * q + 2];
        v[4 * u4][0] = x.x; v[4 * u4][1] = x.y; v[4 * u4][2] = x.z;
        v[4 * u4 + 1][0] = x.w; v[4 * u4 + 1][1] = y.x; v[4 * u4 + 1][2] = y.y;
        v[4 * u4 + 2][0] = y.z; v[4 * u4 + 2][1] = y.w; v[4 * u4 + 2][2] = z.x;
        v[4 * u4 + 3][0] = z.y; v[4 * u4 + 3][1] = z.z; v[4 * u4 + 3][2] = z.w;
        if (a.ids) {
          const uint4 iv = reinterpret_cast<const uint4*>(a.ids)[q];
          id[4 * u4] = iv.x; id[4 * u4 + 1] = iv.y; id[4 * u4 + 2] = iv.z; id[4 * u4 + 3] = iv.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) id[4 * u4 + e] = a.id_base + u32(r0 + e);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const i64 r = r0 + e;
          const i64 rr = r < a.n ? r : 0;
#pragma unroll
          for (int c = 0; c < 3; ++c) v[4 * u4 + e][c] = a.pts[rr * 3 + c];
          id[4 * u4 + e] = a.ids ? a.ids[rr] : a.id_base + u32(r);
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) valid |= (r0 + e < a.n ? 1u : 0u) << (4 * u4 + e);
    }
  } else if (a.pts) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const i64 r = t0 + i64(u) * kBlock + tid;
      const i64 rr = r < a.n ? r : 0;
#pragma unroll
      for (int c = 0; c < D; ++c) v[u][c] = a.pts[rr * D + c];
      id[u] = a.ids ? a.ids[rr] : a.id_base + u32(r);
      valid |= (r < a.n ? 1u : 0u) << u;
    }
  } else {  // SoA columns: every load coalesced
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const i64 r = t0 + i64(u) * kBlock + tid;
      const i64 rr = r < a.n ? r : 0;
#pragma unroll
      for (int c = 0; c < D; ++c) v[u][c] = a.in_cols[i64(c) * a.in_ncol + rr];
      id[u] = __float_as_uint(a.in_cols[i64(D) * a.in_ncol + rr]);
      valid |= (r < a.n ? 1u : 0u) << u;
    }
  }
  return valid;
}

// Zone code of a scatter row: 0..15 its level-4 segment, 16 + T staged at node T, 31 none.
// (Loading the next tile while this one is reordered and stored measured no faster: the
// registers it takes cost more occupancy than the overlap gains.)
// (Staging each tile's 48 KB of 3-D rows through LDS with lane-linear 16-B loads measured slower:
// 1.02 vs 0.91 ms to the end of the scatter at 100 M, profiles/r4_top_sizes_diag.txt.)
template <int D, int R, int NH, bool VEC>
__global__ __launch_bounds__(kBlock) void k_scatter(ScatArgs a) {
  constexpr int HR = R / NH, HALF = kBlock * HR, NZ = kCells + 1;
  constexpr int TILE = kBlock * R;
  constexpr int kBufWords = (D + 1) * HALF + HALF / 4;
  __shared__ uint2 sab[16];           // band [a, b] of heap node X
  __shared__ u32 zlo[NZ], zcap[NZ];   // first row and capacity of each zone's destination
  __shared__ Reorder<NZ, NH> ro;
  __shared__ __align__(16) float lds_rows[kBufWords];
  float(&buf)[D + 1][HALF] = *reinterpret_cast<float(*)[D + 1][HALF]>(lds_rows);
  unsigned char* bz = reinterpret_cast<unsigned char*>(lds_rows + (D + 1) * HALF);
  __shared__ u32 red[kBlock / 64][2 * D];
  const int tid = threadIdx.x, w = tid >> 6, ln = tid & 63;
  if (tid < kNodes) sab[tid] = make_uint2(a.st->a[tid], a.st->b[tid]);
  if (tid < NZ) {
    zlo[tid] = tid < kCells ? u32(a.cell_lo[tid]) : 0u;
    zcap[tid] = tid < kCells ? a.cell_n[tid] : 0xffffffffu;
  }
  if (tid < NH * 4 * NZ) (&ro.wc[0][0][0])[tid] = 0u;
  u32 mn[D], mx[D];
#pragma unroll
  for (int c = 0; c < D; ++c) {
    mn[c] = 0xffffffffu;
    mx[c] = 0u;
  }
  __syncthreads();
  for (i64 tile = blockIdx.x; tile < a.tiles; tile += gridDim.x) {
    float v[R][D];
    u32 id[R];
    const u32 vmask = load_tile<D, R, VEC>(a, tile * TILE, v, id);
    u32 code[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const bool valid = (vmask >> u) & 1u;
      u32 ok[D];
#pragma unroll
      for (int c = 0; c < D; ++c) ok[c] = orderable(v[u][c]);
      u32 X = 0, T = 0;
      bool staged = false;
#pragma unroll
      for (int j = 0; j < kLevels; ++j) {
        u32 k = ok[0];
#pragma unroll
        for (int c = 1; c < D; ++c) k = c == a.ax[j] ? ok[c] : k;
        const uint2 ab = sab[X];
        const bool lt = k < ab.x, gt = k > ab.y, in = !lt && !gt;
        T = (!staged && in) ? X : T;
        X = (staged || in) ? X : 2 * X + 1 + (gt ? 1u : 0u);
        staged = staged || in;
      }
      const u32 zc = !valid ? 31u : (staged ? u32(kCells) + T : X - u32(kNodes));
      const u32 r = wave_rank<5>(min(zc, u32(kCells)), valid, ro.wc[u / HR][w]);
      if (valid) {
#pragma unroll
        for (int c = 0; c < D; ++c) {
          mn[c] = min(mn[c], ok[c]);
          mx[c] = max(mx[c], ok[c]);
        }
      }
      code[u] = zc | (r << 8);
    }
    __syncthreads();
    reorder_scan(ro, [&](int z, u32 tot) -> u32 {
      u32 base = 0;
      if (a.diag == 2) {  // timing diagnostic: an in-range offset instead of the reservation
        const u32 cap = z < kCells ? a.cell_n[z] : u32(a.n);
        base = cap > u32(TILE) ? u32((u64(tile) * 977u) % u64(cap - u32(TILE))) : 0u;
      } else {
        base = tot ? atomicAdd(&a.st->cursor[z], tot) : 0u;
      }
      if (z < kCells && base + tot > a.cell_n[z]) report(a.err, 0x2001u, u32(z), base + tot);
      return base;
    });
    __syncthreads();
#pragma unroll
    for (int h = 0; h < NH; ++h) {
#pragma unroll
      for (int uu = 0; uu < HR; ++uu) {
        const int u = h * HR + uu;
        const u32 zc = code[u] & 255u;
        if (zc == 31u) continue;
        const u32 z = min(zc, u32(kCells));
        const u32 p = ro.hoff[h][z] + ro.wc[h][w][z] + (code[u] >> 8);
#pragma unroll
        for (int c = 0; c < D; ++c) buf[c][p] = v[u][c];
        buf[D][p] = __uint_as_float(id[u]);
        bz[p] = (unsigned char)zc;
      }
      if (ln < NZ) ro.wc[h][w][ln] = 0u;  // this wave's counters for the next tile
      __syncthreads();
      const u32 tot = a.diag == 3 ? 0u : ro.hcnt[h];  // diag 3: no global stores
      for (u32 i = tid; i < tot; i += kBlock) {
        const u32 zc = bz[i];
        const u32 z = min(zc, u32(kCells));
        const u32 q = ro.gbase[h][z] + (i - ro.hoff[h][z]);
        if (q < zcap[z]) {
          float* dst = (z < u32(kCells) ? a.cols : a.stage) + (zlo[z] + q);
#pragma unroll
          for (int c = 0; c <= D; ++c) dst[i64(c) * a.ncol] = buf[c][i];
          if (z == u32(kCells)) a.tags[q] = zc - u32(kCells);
        }
      }
      if (h + 1 < NH) __syncthreads();
    }
  }
#pragma unroll
  for (int c = 0; c < D; ++c) {
    const u32 lo = dev::wave_min_u32(mn[c]), hi = dev::wave_max_u32(mx[c]);
    if (dev::lane() == 0) {
      red[w][c] = lo;
      red[w][D + c] = hi;
    }
  }
  __syncthreads();
  if (tid < 2 * D) {
    u32 r = red[0][tid];
    for (int k = 1; k < kBlock / 64; ++k) r = tid < D ? min(r, red[k][tid]) : max(r, red[k][tid]);
    a.part[size_t(blockIdx.x) * 2 * D + tid] = r;
  }
}

// ---- resolution ---------------------------------------------------------------------------
struct ResArgs {
  const float* stage;
  u32* tags;
  i64 ncol;
  int dim;
  int j;
  int ax[kLevels];
  State* st;
  u32* fine;    // resolution histograms [kLevels][kResBins]
  u64* small;   // [8][kSmallCap]
  u32* err;
};

// J = level: the per-node counts live in registers (3 << J of them, plus the scatter's 15 tag
// counts at level 0), summed over the wave and the block once at the end.
template <int J>
__global__ __launch_bounds__(kHistThreads) void k_res_classify(ResArgs a) {
  if (dev::build_failed(a.err)) return;  // an earlier kernel reported a miss: the build is redone
  constexpr int NC = 3 << J, NO = J == 0 ? kNodes : 0;
  __shared__ u32 h[kResBins];
  __shared__ u32 cnt[8 * 3 + 16];  // [x][left / band / right], then the scatter's tags (j = 0)
  __shared__ u32 sa[8], sb[8];
  __shared__ dev::BucketParams sbp[8];
  __shared__ u64 spv[4];
  const int j = J, nodes = 1 << j, first = nodes - 1, firstp = nodes / 2 - 1, F = res_bins(j);
  u32 rc[NC + NO];
#pragma unroll
  for (int c = 0; c < NC + NO; ++c) rc[c] = 0u;
  const int tid = threadIdx.x;
  for (int i = tid; i < kResBins; i += kHistThreads) h[i] = 0u;
  if (tid < 8 * 3 + 16) cnt[tid] = 0u;
  if (tid < nodes) {
    sa[tid] = a.st->a[first + tid];
    sb[tid] = a.st->b[first + tid];
    sbp[tid] = a.st->bparam[first + tid];
  }
  if (j > 0 && tid < nodes / 2) spv[tid] = a.st->pivot[firstp + tid];
  __syncthreads();
  const i64 staged = a.st->cursor[kCells];
  const i64 per = ((staged + gridDim.x - 1) / gridDim.x + 63) / 64 * 64;
  const i64 i0 = i64(blockIdx.x) * per, i1 = min(staged, i0 + per);
  const int axj = a.ax[j], axp = j > 0 ? a.ax[j - 1] : 0;
  constexpr int U = 4;  // rows per thread per round: their loads are in flight together
  for (i64 ib = i0; ib < i1; ib += U * kHistThreads) {  // uniform trip count: the counts are wave ops
    u32 T[U];
    float kp[U], kj[U];
    u32 idp[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 i = ib + u * kHistThreads + tid;
      T[u] = i < i1 ? a.tags[i] : kMed;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 i = ib + u * kHistThreads + tid;
      const int lvl = (T[u] & kMed) ? -1 : heap_level(T[u]);
      kp[u] = kj[u] = 0.0f;
      idp[u] = 0;
      if (j > 0 && lvl == j - 1) {
        kp[u] = a.stage[i64(axp) * a.ncol + i];
        idp[u] = __float_as_uint(a.stage[i64(a.dim) * a.ncol + i]);
      }
      if (lvl == j || (j > 0 && lvl == j - 1)) kj[u] = a.stage[i64(axj) * a.ncol + i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 i = ib + u * kHistThreads + tid;
      u32 t = T[u];
      bool live = !(t & kMed);
      const bool live0 = live;
      int lvl = live ? heap_level(t) : -1;
      if (j > 0 && live && lvl == j - 1) {
        const u64 comp = (u64(orderable(kp[u])) << 32) | idp[u];
        const u64 P = spv[t - u32(firstp)];
        t = comp < P ? 2 * t + 1 : (comp > P ? 2 * t + 2 : (kMed | t));
        a.tags[i] = t;
        if (t & kMed) {
          a.st->med_idx1[t & 0xffu] = u32(i) + 1u;
          live = false;
        }
        lvl = j;
      }
      const bool at = live && lvl == j;
      u32 idx = 0;
      if (at) {
        const u32 x = t - u32(first);
        const u32 k = orderable(kj[u]);
        const u32 cls = k < sa[x] ? 0u : (k > sb[x] ? 2u : 1u);
        idx = 3 * x + cls;
        if (cls == 1u) atomicAdd(&h[int(x) * F + int(dev::bucket_of(kj[u], sbp[x], F))], 1u);
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) rc[c] += (at && idx == u32(c)) ? 1u : 0u;
#pragma unroll
      for (int c = 0; c < NO; ++c) rc[NC + c] += (live0 && (T[u] & 15u) == u32(c)) ? 1u : 0u;
    }
  }
#pragma unroll
  for (int c = 0; c < NC + NO; ++c) {
    const u32 v = wave_sum(rc[c]);
    if (dev::lane() == 0 && v) atomicAdd(&cnt[c < NC ? c : 24 + (c - NC)], v);
  }
  __syncthreads();
  u32* out = a.fine + size_t(j) * kResBins;
  for (int i = tid; i < kResBins; i += kHistThreads) {
    const u32 v = h[i];
    if (v) atomicAdd(&out[i], v);
  }
  if (tid < nodes * 3) {
    const u32 v = cnt[tid];
    if (v) atomicAdd(&a.st->late[first + tid / 3][tid % 3], v);
  }
  if (j == 0 && tid < kNodes && cnt[24 + tid]) atomicAdd(&a.st->staged_orig[tid], cnt[24 + tid]);
}

// One workgroup per node of level j: the median's rank inside the band from the exact counts
// (rows certain left / right from the scatter, staged rows classified by k_res_classify),
// then the bin holding it.
__global__ __launch_bounds__(kBlock) void k_res_sel1(ResArgs a, Geom g) {
  if (dev::build_failed(a.err)) return;  // an earlier kernel reported a miss: the build is redone
  __shared__ __align__(16) u32 co[256];
  const int j = a.j, first = (1 << j) - 1, F = res_bins(j), gs = F / 256;
  const int X = first + blockIdx.x;
  const u32* fi = a.fine + size_t(j) * kResBins + size_t(blockIdx.x) * F;
  coarse_of(fi, gs, co);
  __syncthreads();
  if (threadIdx.x >= 64) return;
  State* st = a.st;
  const int ln = dev::lane();
  u32 cl = 0, cr = 0;
  if (ln < kHeap) {
    const int Y = ln, ly = heap_level(u32(Y));
    if (ly > j) {
      const int anc = ((Y + 1) >> (ly - j - 1)) - 1;  // Y's ancestor at level j + 1
      if (anc == 2 * X + 1 || anc == 2 * X + 2) {
        const u32 c = Y >= kNodes ? st->cursor[Y - kNodes] : st->staged_orig[Y];
        if (anc == 2 * X + 1) cl = c;
        else cr = c;
      }
    }
  }
  cl = wave_sum(cl);
  cr = wave_sum(cr);
  const i64 L = i64(cl) + st->late[X][0], B = st->late[X][1], R = i64(cr) + st->late[X][2];
  const i64 nX = g.n[X], t = nX / 2 - L;
  const bool ok = L + B + R == nX && t >= 0 && t < B;
  if (!ok) {
    if (ln == 0) {
      report(a.err, L + B + R != nX ? 0x2002u : 0x2003u, u32(X), u32(t < 0 ? 0 : (t >= B ? 1 : 2)));
      st->sel[X] = 0xffffffffu;
    }
    return;
  }
  u32 below = 0, tot = 0;
  const u32 bin = wave_find_fine(co, fi, gs, u32(t), &below, &tot);
  if (ln == 0) {
    if (bin >= u32(F) || tot != u32(B)) {
      report(a.err, 0x2004u, u32(X), tot);
      st->sel[X] = 0xffffffffu;
      return;
    }
    st->sel[X] = bin;
    st->sel_rank[X] = u32(t) - below;
    st->sel_cnt[X] = fi[bin];
  }
}

__global__ __launch_bounds__(kBlock) void k_res_collect(ResArgs a) {
  if (dev::build_failed(a.err)) return;  // an earlier kernel reported a miss: the build is redone
  __shared__ u32 sa[8], sb[8], ssel[8];
  __shared__ dev::BucketParams sbp[8];
  const int j = a.j, nodes = 1 << j, first = nodes - 1, F = res_bins(j);
  const int tid = threadIdx.x;
  if (tid < nodes) {
    sa[tid] = a.st->a[first + tid];
    sb[tid] = a.st->b[first + tid];
    sbp[tid] = a.st->bparam[first + tid];
    ssel[tid] = a.st->sel[first + tid];
  }
  __syncthreads();
  const i64 staged = a.st->cursor[kCells];
  const int axj = a.ax[j];
  const i64 stride = i64(gridDim.x) * kBlock;
  constexpr int U = 4;  // rows per thread per round: their loads are in flight together
  for (i64 ib = i64(blockIdx.x) * (U * kBlock); ib < staged; ib += U * stride) {  // uniform per wave
    u32 T[U];
    float kf[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 i = ib + u * kBlock + tid;
      T[u] = i < staged ? a.tags[i] : kMed;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 i = ib + u * kBlock + tid;
      kf[u] = (!(T[u] & kMed) && heap_level(T[u]) == j) ? a.stage[i64(axj) * a.ncol + i] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 i = ib + u * kBlock + tid;
      bool want = false;
      u32 x = 0;
      u32 k = 0;
      if (!(T[u] & kMed) && heap_level(T[u]) == j) {
        x = T[u] - u32(first);
        k = orderable(kf[u]);
        want = k >= sa[x] && k <= sb[x] && dev::bucket_of(kf[u], sbp[x], F) == ssel[x];
      }
      // one reservation per (wave, node)
      u64 act = __ballot(want);
      while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const u32 key = u32(__shfl(int(x), leader, 64));
        const u64 m = __ballot(want && x == key);
        u32 base = 0;
        if (dev::lane() == leader) base = atomicAdd(&a.st->small_cnt[first + key], u32(__popcll(m)));
        base = u32(__shfl(int(base), leader, 64));
        if (want && x == key) {
          const u32 p = base + dev::mbcnt(m);
          const u64 comp = (u64(k) << 32) | __float_as_uint(a.stage[i64(a.dim) * a.ncol + i]);
          if (p < u32(kSmallCap)) a.small[size_t(x) * kSmallCap + p] = comp;
        }
        act &= ~m;
      }
    }
  }
}

// rank-th smallest (0-based) of the candidate composites visited by each(f) (f(u64) per
// candidate; every thread of the block calls it, visiting its share): MSD radix select with
// 8-bit digits below the highest bit in which the candidates differ.
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
      u32 below = 0, tot = 0;
      const u32 b = wave_find256(hist, rank, &below, &tot);
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

__global__ __launch_bounds__(kBlock) void k_res_sel2(ResArgs a) {
  if (dev::build_failed(a.err)) return;  // an earlier kernel reported a miss: the build is redone
  __shared__ u64 buf[kSmallCap];
  const int j = a.j, first = (1 << j) - 1, F = res_bins(j);
  const int X = first + blockIdx.x, x = blockIdx.x;
  State* st = a.st;
  const u32 sel = st->sel[X];
  if (sel == 0xffffffffu) return;
  const u32 cnt = st->sel_cnt[X], rank = st->sel_rank[X];
  u64 pivot;
  if (cnt <= u32(kSmallCap)) {
    if (st->small_cnt[X] != cnt) {
      if (threadIdx.x == 0) report(a.err, 0x2005u, u32(X), st->small_cnt[X]);
      return;
    }
    for (u32 e = threadIdx.x; e < cnt; e += kBlock) buf[e] = a.small[size_t(x) * kSmallCap + e];
    __syncthreads();
    pivot = block_select(
        [&](auto f) {
          for (u32 e = threadIdx.x; e < cnt; e += kBlock) f(buf[e]);
        },
        rank);
  } else {
    // heavy duplicates: the bin holds more rows than LDS takes; select over the staging arena
    // (every pass streams the staged rows: exact, but one workgroup per node streaming a large
    // arena up to 8 times would take longer than the unsampled build; above kStreamCap staged
    // rows the miss bit is reported instead, and the build is redone without sampling)
    const i64 staged = st->cursor[kCells];
    if (staged > kStreamCap) {
      if (threadIdx.x == 0) report(a.err, 0x200au, u32(X), cnt);
      return;
    }
    const u32 A = st->a[X], B = st->b[X];
    const dev::BucketParams bp = st->bparam[X];
    const int axj = a.ax[j];
    pivot = block_select(
        [&](auto f) {
          for (i64 i = threadIdx.x; i < staged; i += kBlock) {
            if (a.tags[i] != u32(X)) continue;
            const float kf = a.stage[i64(axj) * a.ncol + i];
            const u32 k = orderable(kf);
            if (k < A || k > B) continue;
            if (dev::bucket_of(kf, bp, F) != sel) continue;
            f((u64(k) << 32) | __float_as_uint(a.stage[i64(a.dim) * a.ncol + i]));
          }
        },
        rank);
  }
  if (threadIdx.x == 0) st->pivot[X] = pivot;
}

struct InsArgs {
  const float* stage;
  const u32* tags;
  float* cols;
  i64 ncol;
  int dim;
  int ax3;
  State* st;
  u32* err;
  i64 cell_lo[kCells];
  u32 cell_n[kCells];
};

// Staged rows routed by the level-3 pivots into the free tails of their level-4 segments
// (after the scatter's certain rows), reordered through LDS per tile like the scatter.
template <int D>
__global__ __launch_bounds__(kBlock) void k_res_insert(InsArgs a) {
  if (dev::build_failed(a.err)) return;  // an earlier kernel reported a miss: the build is redone
  constexpr int R = D <= 4 ? 16 : 8, NH = 2, HR = R / NH, HALF = kBlock * HR, NZ = kCells;
  constexpr int TILE = kBlock * R;
  __shared__ Reorder<NZ, NH> ro;
  __shared__ float buf[D + 1][HALF];
  __shared__ unsigned char bz[HALF];
  __shared__ u32 cert[kCells], zlo[kCells], zcap[kCells];
  __shared__ u64 spv[8];
  const int tid = threadIdx.x, w = tid >> 6, ln = tid & 63;
  if (tid < 8) spv[tid] = a.st->pivot[7 + tid];
  if (tid < kCells) {
    cert[tid] = a.st->cursor[tid];
    zlo[tid] = u32(a.cell_lo[tid]);
    zcap[tid] = a.cell_n[tid];
  }
  if (tid < NH * 4 * NZ) (&ro.wc[0][0][0])[tid] = 0u;
  __syncthreads();
  const i64 staged = a.st->cursor[kCells];
  const i64 tiles = (staged + TILE - 1) / TILE;
  for (i64 tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const i64 t0 = tile * TILE;
    float v[R][D + 1];
    u32 code[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const i64 i = t0 + i64(u) * kBlock + tid;
      const i64 ic = i < staged ? i : 0;
#pragma unroll
      for (int c = 0; c <= D; ++c) v[u][c] = a.stage[i64(c) * a.ncol + ic];
      const u32 T = i < staged ? a.tags[i] : kMed;
      u32 z = 31u;
      if (!(T & kMed)) {
        if (heap_level(T) != kLevels - 1) {
          report(a.err, 0x2006u, T, u32(i));
        } else {
          float kv = v[u][0];
#pragma unroll
          for (int c = 1; c < D; ++c) kv = c == a.ax3 ? v[u][c] : kv;  // no dynamic register index
          const u64 comp = (u64(orderable(kv)) << 32) | __float_as_uint(v[u][D]);
          const u64 P = spv[T - 7u];
          if (comp == P) a.st->med_idx1[T] = u32(i) + 1u;
          else z = (comp < P ? 2 * T + 1 : 2 * T + 2) - u32(kNodes);
        }
      }
      const bool valid = z != 31u;
      const u32 r = wave_rank<4>(z & 15u, valid, ro.wc[u / HR][w]);
      code[u] = z | (r << 8);
    }
    __syncthreads();
    reorder_scan(ro, [&](int z, u32 tot) -> u32 {
      const u32 base = (tot ? atomicAdd(&a.st->ins[z], tot) : 0u) + cert[z];
      if (base + tot > zcap[z]) report(a.err, 0x2007u, u32(z), base + tot);
      return base;
    });
    __syncthreads();
#pragma unroll
    for (int h = 0; h < NH; ++h) {
#pragma unroll
      for (int uu = 0; uu < HR; ++uu) {
        const int u = h * HR + uu;
        const u32 z = code[u] & 255u;
        if (z == 31u) continue;
        const u32 p = ro.hoff[h][z] + ro.wc[h][w][z] + (code[u] >> 8);
#pragma unroll
        for (int c = 0; c <= D; ++c) buf[c][p] = v[u][c];
        bz[p] = (unsigned char)z;
      }
      if (ln < NZ) ro.wc[h][w][ln] = 0u;
      __syncthreads();
      const u32 tot = ro.hcnt[h];
      for (u32 i = tid; i < tot; i += kBlock) {
        const u32 z = bz[i];
        const u32 q = ro.gbase[h][z] + (i - ro.hoff[h][z]);
        if (q < zcap[z]) {
          float* dst = a.cols + (zlo[z] + q);
#pragma unroll
          for (int c = 0; c <= D; ++c) dst[i64(c) * a.ncol] = buf[c][i];
        }
      }
      if (h + 1 < NH) __syncthreads();
    }
  }
}

struct FinArgs {
  const float* stage;
  i64 ncol;
  int dim;
  State* st;
  const u32* part;
  int nparts;
  float* out_pts;
  u32* out_ids;
  float* cells;
  dev::BucketParams* params;
  int bins4;
  u32* err;
};

__global__ __launch_bounds__(kBlock) void k_finish(FinArgs a, Geom g) {
  if (dev::build_failed(a.err)) return;  // an earlier kernel reported a miss: the build is redone
  __shared__ u32 box[16];
  __shared__ float split[kNodes];
  __shared__ u32 have[kNodes];
  __shared__ u32 red[kBlock / 64][16];
  __shared__ float scell[kHeap][16];
  const int D = a.dim, tid = threadIdx.x;
  {  // bounding box from the scatter blocks' partials: every value in one pass
    u32 r[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) r[c] = c < D ? 0xffffffffu : 0u;
    for (int p = tid; p < a.nparts; p += kBlock) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (c < 2 * D) {
          const u32 x = a.part[size_t(p) * 2 * D + c];
          r[c] = c < D ? min(r[c], x) : max(r[c], x);
        }
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const u32 v = c < D ? dev::wave_min_u32(r[c]) : dev::wave_max_u32(r[c]);
      if (dev::lane() == 0) red[tid / 64][c] = v;
    }
  }
  if (tid < kCells && a.st->cursor[tid] + a.st->ins[tid] != u32(g.n[kNodes + tid]))
    report(a.err, 0x2008u, u32(tid), a.st->cursor[tid] + a.st->ins[tid]);
  if (tid < kNodes) {
    const u32 i1 = a.st->med_idx1[tid];
    have[tid] = i1 != 0u;
    split[tid] = 0.0f;
    if (i1 == 0u) {
      if (!(*a.err & kErrBit)) report(a.err, 0x2009u, u32(tid), 0u);
    } else {
      const i64 i = i64(i1) - 1;
      const i64 mpos = g.lo[tid] + g.n[tid] / 2;
      for (int c = 0; c < D; ++c) a.out_pts[mpos * D + c] = a.stage[i64(c) * a.ncol + i];
      a.out_ids[mpos] = __float_as_uint(a.stage[i64(D) * a.ncol + i]);
      split[tid] = a.stage[i64(g.axis[heap_level(u32(tid))]) * a.ncol + i];
    }
  }
  __syncthreads();
  if (tid < 2 * D) {
    u32 r = red[0][tid];
    for (int k = 1; k < kBlock / 64; ++k) r = tid < D ? min(r, red[k][tid]) : max(r, red[k][tid]);
    box[tid] = r;
  }
  __syncthreads();
  // cells of nodes 0..30, one (node, bound) per thread: the root box narrowed by every
  // ancestor split on that axis
  for (int e = tid; e < kHeap * 2 * D; e += kBlock) {
    const int h = e / (2 * D), q = e - h * 2 * D, c = q / 2, side = q & 1;
    const int lh = heap_level(u32(h));
    float v = from_orderable(side ? box[D + c] : box[c]);
    for (int l = 0; l < lh; ++l) {
      const int Y = ((h + 1) >> (lh - l)) - 1, C = ((h + 1) >> (lh - l - 1)) - 1;
      if (g.axis[l] != c || !have[Y]) continue;
      const bool left = C == 2 * Y + 1;
      if (left && side == 1) v = split[Y];
      if (!left && side == 0) v = split[Y];
    }
    scell[h][q] = v;
    a.cells[size_t(h) * 2 * D + q] = v;
  }
  __syncthreads();
  if (tid < kCells) {
    const int h = kNodes + tid, ax = g.axis[kLevels];
    a.params[h] = dev::make_params(scell[h][2 * ax], scell[h][2 * ax + 1], a.bins4);
  }
}

template <int D, bool VEC>
void launch_scatter(int blocks, const ScatArgs& sc, hipStream_t stream) {
  constexpr int R = D <= 4 ? 16 : 8;
  k_scatter<D, R, 2, VEC><<<blocks, kBlock, 0, stream>>>(sc);
}

}  // namespace

size_t workspace_bytes() { return layout().total; }

void run(const Geom& g, const IO& io, const Tune& t, hipStream_t stream) {
  const Layout L = layout();
  char* ws = static_cast<char*>(io.ws);
  State* st = reinterpret_cast<State*>(ws + L.state);
  u32* fine_s = reinterpret_cast<u32*>(ws + L.fine_s);
  u32* fine_r = reinterpret_cast<u32*>(ws + L.fine_r);
  u32* skey = reinterpret_cast<u32*>(ws + L.skey);
  u32* gpart = reinterpret_cast<u32*>(ws + L.gpart);
  u64* small = reinterpret_cast<u64*>(ws + L.small);
  u32* part = reinterpret_cast<u32*>(ws + L.part);
  const int D = g.dim;
  if (D < 2 || D > 8) throw std::invalid_argument("top4: dim 2..8");
  const i64 n = io.n;
  // sample size: the sample costs ~S, the staged band rows ~n / sqrt(S), so the best S grows as
  // n^(2/3): 2^20 at 100 M points, 2^18 at 12.5 M (0 = by size)
  const int sl_auto = int(std::lround(20.0 + (2.0 / 3.0) * std::log2(double(std::max<i64>(io.n, 1)) / 1e8)));
  int sl = std::min(kMaxSampleLog2, std::max(10, t.sample_log2 > 0 ? t.sample_log2 : sl_auto));
  while (sl > 10 && (i64(1) << sl) > n / 4) --sl;
  const int S = 1 << sl;

  const i64 zwords = i64(L.zero_end - L.state) / 4;
  const int gblocks = (S + kBlock * kGatherRows - 1) / (kBlock * kGatherRows);
  SampArgs sa{io.pts, io.in_cols, io.in_ncol, D, n, S, {g.axis[0], g.axis[1], g.axis[2], g.axis[3]}, skey, gpart,
              reinterpret_cast<u32*>(ws + L.state), zwords, t.salt};
  k_samp_gather<<<gblocks, kBlock, 0, stream>>>(sa);
  PKD_LAUNCH_CHECK();
  const int hblocks = std::max(1, std::min(kSampBlocks, S / (kHistThreads * 4)));
  for (int j = 0; j < kLevels; ++j) {
    SampLevelArgs la{skey, gpart, gblocks, S, j, {g.axis[0], g.axis[1], g.axis[2], g.axis[3], g.axis[4]},
                     st, fine_s, t.z};
    k_samp_hist<<<hblocks, kHistThreads, 0, stream>>>(la);
    PKD_LAUNCH_CHECK();
    k_samp_sel<<<1 << j, kBlock, 0, stream>>>(la);
    PKD_LAUNCH_CHECK();
  }

  ScatArgs sc{};
  sc.pts = io.pts;
  sc.in_cols = io.in_cols;
  sc.in_ncol = io.in_ncol;
  sc.ids = io.ids;
  sc.id_base = io.id_base;
  sc.n = n;
  sc.cols = io.cols;
  sc.stage = io.stage;
  sc.tags = io.out_ids;
  sc.ncol = io.ncol;
  sc.st = st;
  sc.part = part;
  sc.err = io.err;
  for (int c = 0; c < kCells; ++c) {
    sc.cell_lo[c] = g.lo[kNodes + c];
    sc.cell_n[c] = u32(g.n[kNodes + c]);
  }
  for (int j = 0; j < kLevels; ++j) sc.ax[j] = g.axis[j];
  const int R = D <= 4 ? 16 : 8;
  const i64 tile = i64(kBlock) * R;
  sc.tiles = (n + tile - 1) / tile;
  sc.diag = t.diag;
  const int sblocks = int(std::max<i64>(1, std::min<i64>(t.scatter_blocks > 0 ? t.scatter_blocks : kMaxParts, sc.tiles)));
  const bool vec = D == 3 && io.pts && reinterpret_cast<uintptr_t>(io.pts) % 16 == 0 &&
                   (io.ids == nullptr || reinterpret_cast<uintptr_t>(io.ids) % 16 == 0);
  switch (D) {
    case 2: launch_scatter<2, false>(sblocks, sc, stream); break;
    case 3:
      if (vec) launch_scatter<3, true>(sblocks, sc, stream);
      else launch_scatter<3, false>(sblocks, sc, stream);
      break;
    case 4: launch_scatter<4, false>(sblocks, sc, stream); break;
    case 5: launch_scatter<5, false>(sblocks, sc, stream); break;
    case 6: launch_scatter<6, false>(sblocks, sc, stream); break;
    case 7: launch_scatter<7, false>(sblocks, sc, stream); break;
    default: launch_scatter<8, false>(sblocks, sc, stream); break;
  }
  PKD_LAUNCH_CHECK();
  if (t.diag) return;  // timing diagnostic: the rest is not run

  // staged rows are a few percent of n: grids sized for ~16 % of the rows, grid-stride beyond
  const int rgrid = int(std::max<i64>(64, std::min<i64>(2048, (n / 6 + kBlock * 4 - 1) / (kBlock * 4))));
  const int cgrid = int(std::max<i64>(1, std::min<i64>(kResBlocks, (n / 6 + kHistThreads * 16 - 1) / (kHistThreads * 16))));
  for (int j = 0; j < kLevels; ++j) {
    ResArgs ra{io.stage, io.out_ids, io.ncol, D, j, {g.axis[0], g.axis[1], g.axis[2], g.axis[3]}, st, fine_r, small,
               io.err};
    switch (j) {
      case 0: k_res_classify<0><<<cgrid, kHistThreads, 0, stream>>>(ra); break;
      case 1: k_res_classify<1><<<cgrid, kHistThreads, 0, stream>>>(ra); break;
      case 2: k_res_classify<2><<<cgrid, kHistThreads, 0, stream>>>(ra); break;
      default: k_res_classify<3><<<cgrid, kHistThreads, 0, stream>>>(ra); break;
    }
    PKD_LAUNCH_CHECK();
    k_res_sel1<<<1 << j, kBlock, 0, stream>>>(ra, g);
    PKD_LAUNCH_CHECK();
    k_res_collect<<<rgrid, kBlock, 0, stream>>>(ra);
    PKD_LAUNCH_CHECK();
    k_res_sel2<<<1 << j, kBlock, 0, stream>>>(ra);
    PKD_LAUNCH_CHECK();
  }
  InsArgs ia{};
  ia.stage = io.stage;
  ia.tags = io.out_ids;
  ia.cols = io.cols;
  ia.ncol = io.ncol;
  ia.dim = D;
  ia.ax3 = g.axis[3];
  ia.st = st;
  ia.err = io.err;
  for (int c = 0; c < kCells; ++c) {
    ia.cell_lo[c] = g.lo[kNodes + c];
    ia.cell_n[c] = u32(g.n[kNodes + c]);
  }
  const i64 itile = i64(kBlock) * R;
  const int igrid = int(std::max<i64>(16, std::min<i64>(1024, (n / 8 + itile - 1) / itile)));
  switch (D) {
    case 2: k_res_insert<2><<<igrid, kBlock, 0, stream>>>(ia); break;
    case 3: k_res_insert<3><<<igrid, kBlock, 0, stream>>>(ia); break;
    case 4: k_res_insert<4><<<igrid, kBlock, 0, stream>>>(ia); break;
    case 5: k_res_insert<5><<<igrid, kBlock, 0, stream>>>(ia); break;
    case 6: k_res_insert<6><<<igrid, kBlock, 0, stream>>>(ia); break;
    case 7: k_res_insert<7><<<igrid, kBlock, 0, stream>>>(ia); break;
    default: k_res_insert<8><<<igrid, kBlock, 0, stream>>>(ia); break;
  }
  PKD_LAUNCH_CHECK();
  FinArgs fa{io.stage, io.ncol, D, st, part, sblocks, io.out_pts, io.out_ids, io.cells, io.params, io.bins4, io.err};
  k_finish<<<1, kBlock, 0, stream>>>(fa, g);
  PKD_LAUNCH_CHECK();
}

void band_report(const void* ws, hipStream_t stream, u32 (*out)[3]) {
  const Layout L = layout();
  State h{};
  PKD_HIP_CHECK(hipMemcpyAsync(&h, static_cast<const char*>(ws) + L.state, sizeof(State), hipMemcpyDeviceToHost,
                               stream));
  PKD_HIP_CHECK(hipStreamSynchronize(stream));
  for (int X = 0; X < kNodes; ++X) {
    out[X][0] = h.late[X][1];
    out[X][1] = h.sel_rank[X];  // rank inside the median's bin (see sel for the bin)
    out[X][2] = h.staged_orig[X];
  }
}

}  // namespace top4
}  // namespace pkdtree
