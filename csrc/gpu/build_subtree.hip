// LDS subtree kernel: one workgroup builds a whole segment (<= NMAX points) in LDS.
//
// The rank-propagation kernel k_subtree_rank (below) is the one that ships: points never move
// inside LDS, every level computes each live point's exact (key, id) rank in its sub-segment.
// Each segment's subtree collapses the bottom ~12 levels of build_tree_rec
// (kdtree_sequential.cpp:30-66), where the reference spends millions of tiny sorts and
// `new Node`s. (Alternative kernels measured against it -- a histogram-partition kernel and a
// wave-level rank kernel -- were slower or within 1-2% and are no longer built; see
// profiles/r2_subtree_wave_ab.txt and README "Measured dead ends".)
#include <algorithm>
#include <cstdlib>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "device_utils.hpp"
#include "pkdtree/gpu_build.hpp"
#include "pkdtree/hip_check.hpp"
#include "subtree.hpp"
#include "subtree_common.hpp"

namespace pkdtree {

using dev::BucketParams;
using dev::bucket_of;
using dev::make_params;
using dev::mbcnt;

namespace {
using namespace subtree_detail;

constexpr size_t kLdsMax = 160 * 1024 - 1024;  // minus static LDS

// =====================================================================================
// Rank-based subtree kernel (default). Points never move inside LDS: every level only
// computes each live point's exact rank inside its current sub-segment on the level's axis,
// which decides left / median / right at once.
//   * The first `dim` levels (first use of each axis) rank with a per-sub-segment linear
//     bucket histogram (range from the sub-segment's LDS min/max), a block scan, a
//     bucket-ordered index list and exact (key, id) comparisons inside each bucket.
//   * Every rank is stored, relative to the child it sends the point to, as a 16-bit
//     "compressed rank" of that axis. When the axis comes round again d levels later the
//     ranks of the points of any sub-segment are distinct small integers in the (key, id)
//     order, so the rank inside the sub-segment is a prefix popcount over one LDS bitmap per
//     sub-segment: one ds_or, one scan of word popcounts, one read per point.
// The slot of a point is final when its rank is the median rank; the slot -> point table is
// written then and streamed out at the end with coalesced stores.
namespace rk {

// sub-segments up to this size rank by comparison in one bucket, placed by slot range (PKD_SUBTREE_SMALL;
// 100M 8D 16.62 -> 16.41 ms, 6D 13.37 -> 13.24 against 16; 32 is slower: profiles/r6_subtree_shapes.txt)
constexpr int kSmallSeg = 8;

__host__ __device__ inline int bitlen(u32 v) {
  int b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}
__device__ __forceinline__ u32 pow2_ceil(u32 v) { return v <= 1 ? 1u : 1u << (32 - __clz(v - 1)); }

// Axes whose compressed ranks are kept: only useful if an axis is used twice (dim < height).
__host__ __device__ inline int kept_axes(int dim, int nm) { return dim < bitlen(u32(nm)) ? dim : 0; }

// 32-bit words: rows (dim+1)*nm | crank u16 kept*nm | work nm+68 | aux nm+64 | fin u16 nm+64 |
//               tmpi u16 / bm1 nm/2+64 | root cell 2*dim. The 64 dummy entries at the end of work / aux /
//               fin / tmpi take the writes of finished points, one per lane, so those writes never share an
//               address. bm1 (the compressed levels' second bitmap buffer) aliases tmpi (first-use levels only).
size_t lds_words(int dim, int nm) {
  return size_t(dim + 1) * nm + (size_t(kept_axes(dim, nm)) * nm + 1) / 2 + size_t(nm) + 68 + size_t(nm) + 64 +
         (size_t(nm) + 64) / 2 + size_t(nm) / 2 + 64 + 2 * size_t(dim);
}
// narrow mode: ldim key slots + ids + input row indices, no compressed ranks (ldim <= dim)
size_t lds_words_narrow(int dim, int nm, int ldim) {
  return size_t(ldim + 2) * nm + size_t(nm) + 68 + size_t(nm) + 64 + (size_t(nm) + 64) / 2 + size_t(nm) / 2 + 64 +
         2 * size_t(dim);
}

// In-place exclusive scan of v[0, m) by the whole block; v[m] = total. Caller syncs after.
// m <= CMAX * THREADS. Fixed-trip predicated loops and a shuffle reduction of the wave
// totals: no per-lane loop bounds, so no exec-mask juggling on the (shared) scalar unit.
// Branch-free per lane: out-of-range entries are read from v[0] and written to v[dummy].
template <int THREADS, int CMAX>
__device__ __forceinline__ void block_excl_scan(u32* v, int m, u32* wsum, u32 dummy) {
  constexpr int W = THREADS / 64;
  const int tid = threadIdx.x, w = tid / 64, ln = dev::lane();
  const int C = (m + THREADS - 1) / THREADS;
  const int b0 = tid * C;
  u32 x[CMAX], s = 0;
#pragma unroll
  for (int j = 0; j < CMAX; ++j) {
    const bool in = (j < C) & (b0 + j < m);
    const u32 val = v[in ? b0 + j : 0];
    x[j] = in ? val : 0u;
    s += x[j];
  }
  const u32 incl = dev::wave_incl_scan(s);
  if (ln == 63) wsum[w] = incl;
  __syncthreads();
  // prefix of the wave totals: inclusive scan of wsum over lanes, read at lane w - 1
  const u32 ws = wsum[(W & (W - 1)) == 0 ? (ln & (W - 1)) : (ln < W ? ln : 0)];
  const u32 pin = dev::wave_incl_scan(ln < W ? ws : 0u);
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave-uniform: a scalar select, no exec juggling
  const u32 pl = u32(__builtin_amdgcn_readlane(int(pin), wu > 0 ? wu - 1 : 0));
  const u32 pw = wu > 0 ? pl : 0u;
  u32 run = pw + incl - s;
#pragma unroll
  for (int j = 0; j < CMAX; ++j) {
    const bool in = (j < C) & (b0 + j < m);
    v[in ? u32(b0 + j) : dummy] = run;
    run += x[j];
  }
  if (tid == THREADS - 1) v[m] = run;
}

}  // namespace rk

// NARROW is a template parameter so the classic (low-dim) instantiation carries none of the
// narrow path's registers: a runtime flag cost the 100M x 3D build's subtree kernel 3.7 -> 5.65 ms.
// DIMC > 0: the dimension as a compile-time constant (d = 3 headline shape), else a.dim.
// Two workgroups per CU are the design point below capacity 4096 (one block's barriers hide
// behind the other's work): the register budget is pinned to that many waves per SIMD, since one SGPR over the
// granule halves the resident blocks (82 SGPRs: 100M x 3D subtree 3.3 -> 4.9 ms, resident
// waves 63 -> 32 in profiles/r2_subtree_pmc.txt).
// NM = ITEMS * THREADS need not be a power of two (3 x 512 = 1536 holds the 1525-point segments
// of 100M / 2^16 and 12.5M / 2^13 without idle waves).
template <int ITEMS, int THREADS, bool NARROW, int DIMC>
__device__ __forceinline__ void subtree_rank_body(const SubArgs& a) {
  extern __shared__ __align__(16) u32 smem[];
  __shared__ u32 wsum[THREADS / 64];
  constexpr int NM = ITEMS * THREADS;
  constexpr bool kPow2 = (NM & (NM - 1)) == 0;
  const int dim = DIMC > 0 ? DIMC : a.dim;
  const i64 h = a.heap0 + blockIdx.x;
  const int n = int(a.seg_n[h]);
  if (n <= 0) return;
  const i64 glo = a.seg_lo[h];
  const int tid = threadIdx.x;
  __shared__ u32 failed;  // the build's error word (tested after the load barrier below)
  dev::build_failed_issue(a.err, &failed);
  const int lsub = rk::bitlen(u32(n));  // levels of the implicit subtree of n points
  const int kept_layout = rk::kept_axes(dim, NM);
  const bool keep = dim < lsub;
  // Narrow mode (high dim): LDS holds only the keys of the subtree's own levels (slot t = level
  // t's axis; a.ldim >= lsub and no axis repeats, so keep is false), the ids and the input row
  // indices; output rows are copied from the input. Classic: all dim coordinates + ids.
  constexpr bool narrow = NARROW;
  const int kslots = narrow ? a.ldim : dim;
  const int rcols = narrow ? a.ldim + 2 : dim + 1;
  float* rows = reinterpret_cast<float*>(smem);
  const u32* idrow = reinterpret_cast<const u32*>(rows + kslots * NM);
  u32* ridx = reinterpret_cast<u32*>(rows + (kslots + 1) * NM);  // narrow only
  // crank[axis][...]: a thread's compressed ranks are private to it; with 2 items per thread
  // they sit side by side (index 2 * tid + i), so one ds_read_b32 / ds_write_b32 moves both and
  // no two lanes share a dword
  u16* crank = reinterpret_cast<u16*>(smem + size_t(rcols) * NM);
  u32* work = smem + size_t(rcols) * NM + (size_t(kept_layout) * NM + 1) / 2;
  u32* aux = work + NM + 4 + 64;  // work: NM buckets, sentinel, 64 per-lane dummy words
  u16* fin = reinterpret_cast<u16*>(aux + NM + 64);  // aux / fin: NM entries + 64 per-lane dummies each
  u32* tmpw = aux + NM + 64 + (NM + 64) / 2;
  u16* tmpi = reinterpret_cast<u16*>(tmpw);  // NM + 64 entries (first-use levels)
  float* cellv = reinterpret_cast<float*>(tmpw + NM / 2 + 64);  // [dim][2] root cell of the segment
  // Compressed levels alternate their bitmaps between work and bm1 (NM/2 words + 64 dummies,
  // aliasing tmpi, which only first-use levels use): each level zeroes the buffer of the next
  // one after its first barrier, so a compressed level needs no zero phase of its own (2
  // barriers instead of 3-4); a first-use level zeroes work for whatever level follows it, so
  // the first compressed level after it ORs into work and zeroes bm1 once tmpi is dead.
  u32* bm1 = tmpw;
  const u32 lane_dummy = u32(dev::lane());
  const u32 dummy = u32(NM + 4) + lane_dummy;
  // Item i of a thread is point kid(i): wave w owns the contiguous points [w*64*ITEMS,
  // (w+1)*64*ITEMS), lanes consecutive within an item (conflict-free LDS reads). Waves whose
  // whole range lies beyond n (e.g. 4 of 16 at a 1526-point segment in 2048 slots) skip
  // the per-item phases of every level; they only join the block-wide scans and barriers.
  const int kbase = (tid & ~63) * ITEMS + (tid & 63);
  auto kid = [&](int i) { return kbase + i * 64; };
  const bool wlive = int(__builtin_amdgcn_readfirstlane((tid & ~63) * ITEMS)) < n;
  stamp(a, 0);

  if constexpr (NARROW) {  // ids and input row indices, then the subtree levels' keys from the input rows
    u32* idw = reinterpret_cast<u32*>(rows + kslots * NM);
    const u32* idc = reinterpret_cast<const u32*>(a.cols) + i64(a.narrow_k) * a.ncol + glo;
    for (int k = tid; k < n; k += THREADS) {
      idw[k] = idc[k];
      ridx[k] = idc[a.ncol + k];
    }
    for (int k = tid; k < 2 * dim; k += THREADS) cellv[k] = a.cells[h * dim * 2 + k];
    __syncthreads();
    constexpr int kG = 8;  // loads in flight per thread
    const int total = n * kslots;
    for (int e0 = tid; e0 < total; e0 += THREADS * kG) {
      float v[kG];
#pragma unroll
      for (int u = 0; u < kG; ++u) {
        const int e = e0 + u * THREADS, k = e / kslots, t = e - k * kslots;
        v[u] = e < total ? a.in_rows[i64(ridx[k]) * a.in_rs + (a.depth_base + t) % dim] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kG; ++u) {
        const int e = e0 + u * THREADS, k = e / kslots, t = e - k * kslots;
        if (e < total) rows[t * NM + k] = v[u];
      }
    }
  } else {  // rows -> LDS: every load of the first kLoadCols columns issued before any LDS store
    // (all 9 columns of an 8-D row in flight at once measured no faster: 100M x 8D 18.12 ms)
    constexpr int kLoadCols = 5;
    float v[kLoadCols][ITEMS];
#pragma unroll
    for (int c = 0; c < kLoadCols; ++c)
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int k = tid + i * THREADS;
        v[c][i] = (c <= dim && k < n) ? a.cols[i64(c) * a.ncol + glo + k] : 0.0f;
      }
    for (int k = tid; k < 2 * dim; k += THREADS) cellv[k] = a.cells[h * dim * 2 + k];
#pragma unroll
    for (int c = 0; c < kLoadCols; ++c)
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int k = tid + i * THREADS;
        if (c <= dim && k < n) rows[c * NM + k] = v[c][i];
      }
    for (int c = kLoadCols; c <= dim; ++c) {
      const float* col = a.cols + i64(c) * a.ncol + glo;
      float w[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int k = tid + i * THREADS;
        w[i] = k < n ? col[k] : 0.0f;
      }
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int k = tid + i * THREADS;
        if (k < n) rows[c * NM + k] = w[i];
      }
    }
  }
  // The per-item code of the levels is branch-free: finished or absent points compute on
  // harmless values, loads use clamped indices and stores of such points go to per-lane dummy
  // words. Per-item branches cost three scalar instructions each (exec save / branch /
  // restore) on the CU's one scalar unit, which bounded the kernel (SALU = 0.76 x VALU,
  // profiles/r2_subtree_pmc.txt).
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int k = tid + i * THREADS;
    fin[k < n ? u32(k) : u32(NM) + lane_dummy] = 0xffffu;
  }
#pragma unroll
  for (int j = 0; j <= ITEMS; ++j) {  // the first level's histogram (buckets + sentinel)
    const int w = tid + j * THREADS;
    work[w <= NM ? u32(w) : dummy] = 0;
  }
  u32 lo[ITEMS], nn[ITEMS], sg[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    lo[i] = 0;
    sg[i] = 0;
    nn[i] = kid(i) < n ? u32(n) : 0u;
  }
  __syncthreads();
  if (failed) return;  // the build already failed (a miss): it is redone
  stamp(a, 1);

  int cb = 0;          // bitmap buffer of the next compressed level: 1 = bm1, 0 = work
  bool synced = true;  // false after a compressed level (it ends without a barrier)
  bool wz = true;      // work holds zeros (a first-use level zeroes it for the next one)
  // Wt of level t: > 0 when its ranks come from the compressed ranks of the axis's last use
  auto words_of = [&](int t) -> int {
    if (narrow || !keep || t < dim) return 0;
    const u32 wbits = u32(n) >> (t - dim + 1);
    const u32 words = rk::pow2_ceil((wbits + 31) / 32);
    return (words <= 64 && u32(1u << t) * words <= u32(NM / 2)) ? int(words) : 0;
  };
  for (int t = 0; t < lsub; ++t) {
    const int axis = (a.depth_base + t) % dim;
    const float* kcol = rows + (narrow ? t : axis) * NM;
    u16* cr = crank + size_t(axis) * NM;
    const int S = 1 << t;
    const bool alone = (n >> t) <= 1;  // every sub-segment holds at most one point: it is the median
    const int Wt = alone ? 0 : words_of(t);
    u32 rank[ITEMS];
    if (alone) {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) rank[i] = 0;
    } else if (Wt > 0) {
      // ---- compressed ranks: one bitmap of Wt words per sub-segment ----
      // (already zeroed by the previous level; its readers finished before this level's barrier)
      u32* bmp = cb ? bm1 : work;
      u32* nxt = cb ? work : bm1;
      const u32 bdum = cb ? u32(NM / 2) + lane_dummy : dummy;
      const int nw = S * Wt;  // <= NM / 2
      u32 c[ITEMS], wi[ITEMS];
      if (wlive) {
        if (ITEMS == 2) {
          const u32 both = reinterpret_cast<const u32*>(cr)[tid];
          c[0] = both & 0xffffu;
          c[ITEMS - 1] = both >> 16;
        } else {
#pragma unroll
          for (int i = 0; i < ITEMS; ++i) c[i] = cr[tid + i * THREADS];
        }
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const u32 wv = sg[i] * u32(Wt) + (c[i] >> 5);
          const u32 bit = 1u << (c[i] & 31);
          wi[i] = nn[i] ? wv : bdum;
          atomicOr(&bmp[wi[i]], nn[i] ? bit : 0u);
        }
      }
      __syncthreads();
      // the next compressed level's buffer: last read by the level before this one
      for (int w = tid; w < NM / 2; w += THREADS) nxt[w] = 0;
      if (Wt > 1) {  // exclusive popcount prefix inside each group of Wt words (one wave holds a group)
        const u32 g = lane_dummy & u32(Wt - 1);
        for (int w0 = 0; w0 < nw; w0 += THREADS) {
          const int w = w0 + tid;
          const bool in = w < nw;
          const u32 pc = u32(__popc(bmp[in ? w : 0]));
          const u32 v = in ? pc : 0u;
          u32 incl = v;
          for (int o = 1; o < Wt; o <<= 1) {
            const u32 tt = __shfl_up(incl, o, 64);
            incl += g >= u32(o) ? tt : 0u;
          }
          aux[in ? u32(w) : u32(NM) + lane_dummy] = incl - v;
        }
        __syncthreads();
      }
      if (wlive) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const u32 below = Wt > 1 ? aux[kPow2 ? (wi[i] & (NM - 1)) : min(wi[i], u32(NM - 1))] : 0u;
          rank[i] = below + u32(__popc(bmp[wi[i]] & ((1u << (c[i] & 31)) - 1u)));
        }
      }
      cb ^= 1;
      wz = false;
    } else {
      // ---- exact ranks from bucket histograms (first use of the axis) ----
      // Bucket range: the block root's cell on this axis. On an axis's first use no split
      // inside the block has narrowed it, so it is the sub-segment's own range; otherwise it
      // is a valid (wider) range. Any monotone bucketing gives exact ranks.
      // About one point per bucket (S * B <= NM): most buckets need no comparison at all.
      const int maxsize = n >> t;
      const int B = maxsize > a.small_seg ? min(int(rk::pow2_ceil(u32(maxsize))), NM >> t) : 1;
      // B == 1 (sub-segments of <= kSmallSeg points): a sub-segment's points go to its own slot
      // range [lo, lo + nn) of the bucket order -- the layout the scan would give, up to gaps -- so
      // the level needs no scan (one barrier and a block scan fewer; 8-D's levels 6 and 7)
      const bool direct = B == 1;
      const int nb = S * B;  // <= NM; work[nb] is the scan's total (sentinel)
      u32* tmpk = aux;       // orderable keys in bucket order
      const BucketParams pr = make_params(cellv[2 * axis], cellv[2 * axis + 1], B);
      if (!wz) {  // (normally the previous level zeroed work before its closing barrier)
        if (!synced) __syncthreads();  // the previous (compressed) level's readers of work / aux
#pragma unroll
        for (int j = 0; j <= ITEMS; ++j) {
          const int w = tid + j * THREADS;
          work[w <= nb ? u32(w) : dummy] = 0;
        }
        __syncthreads();
      }
      if (t == 0) stamp(a, 20);
      u32 ok[ITEMS];
      u32 bk[ITEMS], wi[ITEMS];
      if (wlive) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {  // finished points count into a per-lane dummy word
          const float kf = kcol[kid(i)];
          ok[i] = orderable(kf);
          const u32 b = sg[i] * u32(B) + (B > 1 ? bucket_of(kf, pr, B) : 0u);
          bk[i] = nn[i] ? b : dummy;
          wi[i] = atomicAdd(&work[bk[i]], 1u);
        }
      }
      __syncthreads();
      if (t == 0) stamp(a, 21);
      if (!direct) {
        rk::block_excl_scan<THREADS, ITEMS>(work, nb, wsum, dummy);
        __syncthreads();
      }
      if (t == 0) stamp(a, 22);
      // scatter into bucket order; every read of the scanned histogram happens here, so the
      // histogram can be zeroed for the next level right after the barrier below
      u32 pos[ITEMS], st[ITEMS], cnt[ITEMS];
      if (wlive) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const u32 bi = nn[i] ? bk[i] : 0u;
          const u32 sb = nn[i] ? sg[i] * u32(B) : 0u;
          u32 s0 = lo[i], e0 = lo[i] + nn[i], b0 = lo[i];
          if (!direct) {
            s0 = work[bi];
            e0 = work[bi + 1];
            b0 = work[sb];
          }
          pos[i] = nn[i] ? s0 + wi[i] : u32(NM) + lane_dummy;
          tmpk[pos[i]] = ok[i];
          tmpi[pos[i]] = u16(kid(i));
          st[i] = s0;
          cnt[i] = nn[i] ? e0 - s0 : 0u;  // 0 for finished points
          rank[i] = s0 - b0;
        }
      }
      __syncthreads();
      if (t == 0) stamp(a, 23);
      // the next level's buckets + sentinel (first use) or bitmaps (compressed), zeroed now
      wz = t + 1 < lsub;
      cb = 0;
      if (wz) {
#pragma unroll
        for (int j = 0; j <= ITEMS; ++j) {
          const int w = tid + j * THREADS;
          work[w <= NM ? u32(w) : dummy] = 0;
        }
      }
      if (wlive) {
        // in-bucket comparisons, kU members per round: all items' reads of a round are issued
        // together; wave-uniform trip count = largest bucket among the wave's items / kU
        constexpr u32 kU = 2;
        for (u32 j0 = 0;; j0 += kU) {
          u32 any = 0;
#pragma unroll
          for (int i = 0; i < ITEMS; ++i) any |= u32(j0 < cnt[i]);
          if (!__ballot(any)) break;
          u32 qk[kU][ITEMS];
#pragma unroll
          for (u32 u = 0; u < kU; ++u)
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
              const u32 q = st[i] + j0 + u;
              qk[u][i] = tmpk[j0 + u < cnt[i] ? q : 0u];
            }
          u32 tany = 0;
#pragma unroll
          for (u32 u = 0; u < kU; ++u)
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
              const u32 act = u32(j0 + u < cnt[i]);
              rank[i] += act & u32(qk[u][i] < ok[i]);
              tany |= act & u32(qk[u][i] == ok[i]) & u32(st[i] + j0 + u != pos[i]);
            }
          if (__ballot(tany)) {  // equal keys: the id decides
#pragma unroll
            for (u32 u = 0; u < kU; ++u)
#pragma unroll
              for (int i = 0; i < ITEMS; ++i) {
                const u32 q = st[i] + j0 + u;
                const u32 tie = u32(j0 + u < cnt[i]) & u32(qk[u][i] == ok[i]) & u32(q != pos[i]);
                const u32 other = idrow[tmpi[tie ? q : 0u]];
                rank[i] += tie & u32(other < idrow[kid(i)]);
              }
          }
        }
      }
      if (t == 0) stamp(a, 24);
    }
    // ---- median / left / right (selects only; the median's slot write goes to a dummy
    // word for every other point) ----
    if (wlive) {
      u32 cn[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 n0 = nn[i], mid = n0 >> 1, r = rank[i];
        const u32 is_mid = u32(n0 != 0) & u32(r == mid);
        const u32 right = u32(r > mid);
        const u32 fslot = lo[i] + mid, rr = r - mid - 1, lr = lo[i] + mid + 1, nr = n0 - mid - 1;
        fin[is_mid ? fslot : u32(NM) + lane_dummy] = u16(kid(i));
        cn[i] = right ? rr : r;
        if (keep && ITEMS != 2) cr[tid + i * THREADS] = u16(cn[i]);
        lo[i] = right ? lr : lo[i];
        sg[i] = 2 * sg[i] + right;
        const u32 nc = right ? nr : mid;
        nn[i] = is_mid ? 0u : nc;  // n0 == 0 gives nc == 0 as well (mid 0, right only if r > 0 -> nr wraps)
        nn[i] = n0 ? nn[i] : 0u;
      }
      if (keep && ITEMS == 2) reinterpret_cast<u32*>(cr)[tid] = (cn[0] & 0xffffu) | (cn[ITEMS - 1] << 16);
    }
    // Closing barrier for first-use levels (the next level rewrites work) and for compressed
    // levels without a prefix phase (it orders their zeroing of the next buffer before the next
    // level's ORs); a compressed level with Wt > 1 already had its second barrier after that.
    synced = Wt <= 1;
    if (synced) __syncthreads();
    if (t < 18) stamp(a, 2 + t);
  }
  if (!synced) __syncthreads();  // fin: the last level's slot writes
  stamp(a, 30);
  // in-order rows out: thread per slot, the row's dim floats (consecutive threads cover
  // consecutive 4*dim-byte runs, merged in L2)
  float* outp = a.out_pts + glo * dim;
  if constexpr (NARROW) {  // slot -> input row index, then rows copied from the input (coalesced per row)
    for (int k = tid; k < n; k += THREADS) {
      u32 p = fin[k];
      if (p >= u32(NM)) {
        report(a.err, 0x800u, u32(k), p);
        p = 0;
      }
      a.out_ids[glo + k] = idrow[p];
      work[k] = ridx[p];
    }
    __syncthreads();
    constexpr int kG = 8;
    const int total = n * dim;
    for (int e0 = tid; e0 < total; e0 += THREADS * kG) {
      float v[kG];
#pragma unroll
      for (int u = 0; u < kG; ++u) {
        const int e = e0 + u * THREADS, k = e / dim, c = e - k * dim;
        v[u] = e < total ? a.in_rows[i64(work[k]) * a.in_rs + c] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kG; ++u) {
        const int e = e0 + u * THREADS;
        if (e < total) outp[e] = v[u];
      }
    }
  } else {
    for (int k = tid; k < n; k += THREADS) {
      u32 p = fin[k];
      if (p >= u32(NM)) {
        report(a.err, 0x800u, u32(k), p);
        p = 0;
      }
      for (int c = 0; c < dim; ++c) outp[i64(k) * dim + c] = rows[c * NM + p];
      a.out_ids[glo + k] = idrow[p];
    }
  }
  __syncthreads();
  stamp(a, 31);
}

// WPE: waves per SIMD the register budget is pinned to (0: two blocks per CU below capacity
// 4096, else one; a CU holds at most 8 waves per SIMD)
template <int ITEMS, int THREADS, bool NARROW, int DIMC = 0, int WPE = 0>
__global__ __launch_bounds__(THREADS)
__attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : (ITEMS * THREADS >= 4096 ? 1 : 2) * THREADS / 256)))
void k_subtree_rank(SubArgs a) {
  subtree_rank_body<ITEMS, THREADS, NARROW, DIMC>(a);
}

template <int ITEMS, int THREADS, int WPE3 = 0>
void launch_rank_cfg(const SubArgs& a0, i64 segs, hipStream_t stream) {
  SubArgs a = a0;
  if (a.ldim > 0) {  // a key slot for every level a segment of this capacity can have
    a.ldim = std::max(a.ldim, rk::bitlen(u32(ITEMS * THREADS)));
    if (a.ldim > a.dim) throw std::runtime_error("pkdtree: narrow subtree needs dim >= its levels");
  }
  const size_t lds = 4 * (a.ldim > 0 ? rk::lds_words_narrow(a.dim, ITEMS * THREADS, a.ldim)
                                     : rk::lds_words(a.dim, ITEMS * THREADS));
  const bool nar = a.ldim > 0;
  const void* fn = nar ? reinterpret_cast<const void*>(&k_subtree_rank<ITEMS, THREADS, true>)
                       : reinterpret_cast<const void*>(&k_subtree_rank<ITEMS, THREADS, false>);
  ensure_dynamic_lds(fn, int(kLdsMax));
  bool done = false;
  if (nar) {
    k_subtree_rank<ITEMS, THREADS, true><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
    done = true;
  }
  if constexpr (ITEMS == 2 || ITEMS * THREADS == 1536) {
    if (!done && a.dim == 3) {
      ensure_dynamic_lds(reinterpret_cast<const void*>(&k_subtree_rank<ITEMS, THREADS, false, 3, WPE3>), int(kLdsMax));
      k_subtree_rank<ITEMS, THREADS, false, 3, WPE3><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
      done = true;
    }
  }
  if constexpr ((ITEMS == 1 && THREADS == 1024) || ITEMS * THREADS == 768) {  // d = 8 (BASELINE's high-dim config)
    if (!done && a.dim == 8) {
      ensure_dynamic_lds(reinterpret_cast<const void*>(&k_subtree_rank<ITEMS, THREADS, false, 8>), int(kLdsMax));
      k_subtree_rank<ITEMS, THREADS, false, 8><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
      done = true;
    }
  }
  if (!done) k_subtree_rank<ITEMS, THREADS, false><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
  PKD_LAUNCH_CHECK();
}

size_t impl_lds_bytes(int dim, int nm) { return 4 * rk::lds_words(dim, nm); }

}  // namespace

unsigned long long*& subtree_stamp_buffer() {
  static unsigned long long* p = nullptr;
  return p;
}

std::string subtree_stamp_report() {
  unsigned long long* d = subtree_stamp_buffer();
  if (!d) return "stamps disabled (set PKD_SUBTREE_STAMPS=1)";
  std::vector<unsigned long long> h(size_t(kStampBlocks) * kStampSlots);
  PKD_HIP_CHECK(hipDeviceSynchronize());
  PKD_HIP_CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  // per block, the recorded slots in time order; each slot is charged the cycles since the
  // previous recorded one (mean over blocks that recorded start and end)
  double acc[kStampSlots] = {};
  int cnt[kStampSlots] = {};
  for (int b = 0; b < kStampBlocks; ++b) {
    const unsigned long long* s = &h[size_t(b) * kStampSlots];
    if (!s[0] || !s[31]) continue;
    std::vector<std::pair<unsigned long long, int>> ev;
    for (int i = 0; i < kStampSlots; ++i)
      if (s[i]) ev.emplace_back(s[i], i);
    std::sort(ev.begin(), ev.end());
    for (size_t k = 1; k < ev.size(); ++k) {
      acc[ev[k].second] += double(ev[k].first - ev[k - 1].first);
      ++cnt[ev[k].second];
    }
  }
  std::ostringstream os;
  os << "subtree stamps (mean cycles since the previous mark, in time order):";
  for (int i = 1; i < kStampSlots; ++i) {
    if (!cnt[i]) continue;
    os << " ";
    if (i == 1) os << "load";
    else if (i == 30) os << "levels-end";
    else if (i >= 20 && i <= 29) os << "s" << i;
    else if (i == 31) os << "store";
    else os << "L" << (i - 2);
    os << "=" << long(acc[i] / cnt[i]);
  }
  return os.str();
}

int subtree_capacity(int dim) {
  // Prefer two workgroups per CU (LDS <= ~78 KiB) so one block's barriers hide behind the
  // other's work; fall back to smaller capacities for high dimensions.
  for (int nm = 2048; nm >= 64; nm /= 2)
    if (impl_lds_bytes(dim, nm) <= kLdsMax / 2) return nm;
  for (int nm = 64; nm >= 32; nm /= 2)
    if (impl_lds_bytes(dim, nm) <= kLdsMax) return nm;
  throw std::invalid_argument("pkdtree: dimension too large for the LDS subtree kernel");
}

int subtree_capacity_narrow(int dim) {
  for (int nm = 2048; nm >= 64; nm /= 2) {
    const int ldim = rk::bitlen(u32(nm));
    if (ldim <= dim && 4 * rk::lds_words_narrow(dim, nm, ldim) <= kLdsMax / 2) return nm;
  }
  return 0;
}

int subtree_capacity_max(int dim) {
  for (int nm = 4096; nm >= 32; nm /= 2)
    if (impl_lds_bytes(dim, nm) <= kLdsMax) return nm;
  throw std::invalid_argument("pkdtree: dimension too large for the LDS subtree kernel");
}

void launch_subtree(const float* cols, i64 ncol, int dim, const i64* seg_lo, const i64* seg_n, const float* cells,
                    i64 heap0, i64 segs, int depth_base, int nmax, float* out_pts, u32* out_ids, u32* err,
                    hipStream_t stream, int narrow_idcol, const float* in_rows, i64 in_rs) {
  if (segs <= 0) return;
  static unsigned long long* stamps = nullptr;
  if (std::getenv("PKD_SUBTREE_STAMPS") && !stamps) {
    PKD_HIP_CHECK(hipMalloc(&stamps, size_t(kStampBlocks) * kStampSlots * sizeof(unsigned long long)));
    PKD_HIP_CHECK(hipMemset(stamps, 0, size_t(kStampBlocks) * kStampSlots * sizeof(unsigned long long)));
  }
  subtree_stamp_buffer() = stamps;
  // narrow: one key slot per subtree level (no axis repeats: the host enables narrow
  // columns only for dim >= the subtree's levels)
  const int ldim = narrow_idcol >= 0 ? rk::bitlen(u32(std::max(nmax, 1))) : 0;
  if (ldim > dim) throw std::runtime_error("pkdtree: narrow subtree needs dim >= its levels");
  const char* ess = ab_knob("PKD_SUBTREE_SMALL");
  SubArgs a{cols, ncol, dim, seg_lo, seg_n, cells, heap0, depth_base, out_pts, out_ids, err, stamps,
            std::max(narrow_idcol, 0), in_rows, in_rs, ldim, ess ? std::max(1, std::atoi(ess)) : rk::kSmallSeg};
  {
    // (read per launch, so tests can vary them within one process)
    const char* ew = ab_knob("PKD_SUBTREE_WIDE");
    const bool wide = !(ew && std::string(ew) == "0");
    const char* ec = ab_knob("PKD_SUBTREE_CFG");
    const std::string cfg = ec ? ec : "";
    const char* e15 = ab_knob("PKD_SUBTREE_1536");
    const bool c1536 = !(e15 && std::string(e15) == "0");
    if (nmax > 2048) launch_rank_cfg<4, 1024>(a, segs, stream);
    // 3-D segments of 1025..1536 points (100M / 2^16 and 12.5M / 2^13: 1525 points): capacity
    // 1536 = 3 items x 512 threads, 52 KiB of LDS, three workgroups (24 waves) per CU. Against
    // 2 x 1024 (4 idle waves of 16 at 1525 points, two workgroups per CU): 100M x 3D 11.64 ->
    // 11.14-11.43 ms, 12.5M 1.753 -> 1.680 ms; 2 x 768 (two workgroups of 12 waves) was in
    // between (profiles/r3_subtree_1536.txt)
    else if (nmax > 1024 && nmax <= 1536 && cfg == "6x256" && a.ldim == 0) launch_rank_cfg<6, 256>(a, segs, stream);
    else if (nmax > 1024 && nmax <= 1536 && cfg == "4x384" && a.ldim == 0) launch_rank_cfg<4, 384>(a, segs, stream);
    else if (nmax > 1024 && nmax <= 1536 && cfg == "2x768" && a.ldim == 0) launch_rank_cfg<2, 768>(a, segs, stream);
    else if (nmax > 1024 && nmax <= 1536 && wide && c1536 && dim == 3 && a.ldim == 0)
      launch_rank_cfg<3, 512, 6>(a, segs, stream);
    else if (nmax > 1024 && wide) launch_rank_cfg<2, 1024>(a, segs, stream);
    else if (nmax > 1024) launch_rank_cfg<4, 512>(a, segs, stream);
    // Segments of 513..1024 / 257..512 points (dims >= 4, whose rows fill the LDS sooner): the
    // higher the dim, the more levels are first uses of an axis (latency-bound histogram
    // ranking), so more waves per segment win: 100M x 8D 31.4 -> 28.1 ms with 1024 threads
    // instead of 256 (profiles/r1_subtree_config_sweep.txt). PKD_SUBTREE_CFG overrides.
    else if (nmax > 512 && (cfg == "4x256")) launch_rank_cfg<4, 256>(a, segs, stream);
    // Segments of 513..768 points (100M / 2^17 = 763 at dims 4..8): capacity 768 instead of 1024,
    // fewer threads per workgroup, three workgroups per CU. 100M build, ms (profiles/r6_subtree_shapes.txt):
    //            default (2x512 / 1x1024)  3x256   2x384
    //   4-D      11.2                      10.24   11.14
    //   5-D      12.46                     12.58   13.28
    //   6-D      15.46                     12.97   13.71
    //   7-D      17.53                     16.00   15.89
    //   8-D      17.83                     16.97   16.78
    else if (nmax > 512 && nmax <= 768 && cfg.empty() && a.ldim == 0 && (dim == 4 || dim == 6))
      launch_rank_cfg<3, 256>(a, segs, stream);
    else if (nmax > 512 && nmax <= 768 && cfg.empty() && a.ldim == 0 && (dim == 7 || dim == 8))
      launch_rank_cfg<2, 384>(a, segs, stream);
    else if (nmax > 512 && nmax <= 768 && cfg == "1x768") launch_rank_cfg<1, 768>(a, segs, stream);
    else if (nmax > 512 && nmax <= 768 && cfg == "3x256") launch_rank_cfg<3, 256>(a, segs, stream);
    else if (nmax > 512 && nmax <= 768 && cfg == "6x128") launch_rank_cfg<6, 128>(a, segs, stream);
    else if (nmax > 512 && nmax <= 768 && cfg == "2x384") launch_rank_cfg<2, 384>(a, segs, stream);
    // (2 x 512 up to 7-D: 100M x 6D 16.90 -> 16.79 ms, 7D 18.23 -> 18.18; 8D 18.42 -> 19.24 with it)
    else if (nmax > 512 && (cfg == "2x512" || (cfg.empty() && dim <= 7))) launch_rank_cfg<2, 512>(a, segs, stream);
    else if (nmax > 512) launch_rank_cfg<1, 1024>(a, segs, stream);
    else if (nmax > 256 && cfg == "2x256") launch_rank_cfg<2, 256>(a, segs, stream);
    else if (nmax > 256) launch_rank_cfg<1, 512>(a, segs, stream);
    else if (nmax > 128) launch_rank_cfg<1, 256>(a, segs, stream);
    else if (nmax > 64) launch_rank_cfg<1, 128>(a, segs, stream);
    else launch_rank_cfg<1, 64>(a, segs, stream);
  }
}

}  // namespace pkdtree
