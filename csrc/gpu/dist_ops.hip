// Device ops of the global (distributed) decomposition; see dist_ops.hpp.
#include <algorithm>
#include <stdexcept>

#include "device_utils.hpp"
#include "pkdtree/dist_ops.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {

using dev::BucketParams;
using dev::bucket_of;
using dev::make_params;
using dev::mbcnt;

namespace {

constexpr int kBlock = 256;
constexpr int kPivotThreads = 1024;
constexpr int kBboxBlocks = 512;      // grid of the bounding-box reduction
// keys of a node's middle rows in LDS (+ where each came from: 12 B per row, 156 KiB); larger
// middles stream from L2. (A 100 M-point build's middle holds ~12.2 K rows at every level.)
constexpr int kPivotLdsKeys = 13312;

__device__ __forceinline__ u32 point_id(const TopPoints& p, i64 i) { return p.ids ? p.ids[i] : p.id_base + u32(i); }

// Route one point one level down below the pivot of its node (heap order). The id is only
// read when the keys tie.
__device__ __forceinline__ u32 route_key(u32 h, float key, const TopPoints& p, i64 i, const u64* pivots) {
  if (h == kTopDone) return h;
  const u32 k = orderable(key);
  const u64 pv = pivots[h];
  const u32 pk = u32(pv >> 32);
  if (k != pk) return k < pk ? 2 * h + 1 : 2 * h + 2;
  const u32 id = point_id(p, i), pid = u32(pv);
  return id < pid ? 2 * h + 1 : (id > pid ? 2 * h + 2 : kTopDone);
}
__device__ __forceinline__ u32 route(u32 h, const TopPoints& p, i64 i, int axis, const u64* pivots) {
  if (h == kTopDone) return h;
  const u32 k = orderable(p.pts[i * p.dim + axis]);
  const u64 pv = pivots[h];
  const u32 pk = u32(pv >> 32);
  if (k != pk) return k < pk ? 2 * h + 1 : 2 * h + 2;
  const u32 id = point_id(p, i), pid = u32(pv);
  return id < pid ? 2 * h + 1 : (id > pid ? 2 * h + 2 : kTopDone);
}

// ---- bounding box --------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_top_bbox(TopPoints p, i64 T, i64* __restrict__ box) {
  extern __shared__ __align__(16) u32 sb[];  // [2 * dim]
  const int dim = p.dim;
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) sb[c] = 0xffffffffu;
  __syncthreads();
  const i64 t = i64(blockIdx.x) * kBlock + threadIdx.x;
  if (t < T) {  // T is a multiple of dim, so this thread always sees axis t % dim
    const int c = int(t % dim);
    u32 lo = 0xffffffffu, nhi = 0xffffffffu;
    const i64 total = p.n * dim;
    constexpr int U = 8;  // loads in flight per thread; past the end a thread re-reads its first value
    const float first = p.pts[t];  // t < T <= total, same axis
    for (i64 f0 = t; f0 < total; f0 += U * T) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const i64 f = f0 + i64(u) * T;
        v[u] = f < total ? p.pts[f] : first;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const u32 k = orderable(v[u]);
        lo = min(lo, k);
        nhi = min(nhi, ~k);
      }
    }
    atomicMin(&sb[c], lo);
    atomicMin(&sb[dim + c], nhi);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) {
    if (sb[c] != 0xffffffffu)
      atomicMin(reinterpret_cast<unsigned long long*>(box + c), (unsigned long long)sb[c]);
  }
}

// 16-B loads (rows 16-B aligned): thread t reads float4s t, t + T4, ...; 4 T4 is a multiple of
// dim, so element e of every float4 of a thread has axis (4 t + e) % dim. The < 4 floats past the
// last whole float4 are read by thread 0.
__global__ __launch_bounds__(kBlock) void k_top_bbox4(TopPoints p, i64 T4, i64* __restrict__ box) {
  extern __shared__ __align__(16) u32 sb[];  // [2 * dim]
  const int dim = p.dim;
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) sb[c] = 0xffffffffu;
  __syncthreads();
  const i64 t = i64(blockIdx.x) * kBlock + threadIdx.x;
  const i64 total = p.n * dim, total4 = total / 4;
  if (t < T4 && t < total4) {
    u32 lo[4], nhi[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) lo[e] = nhi[e] = 0xffffffffu;
    const float4* in = reinterpret_cast<const float4*>(p.pts);
    const float4 first = in[t];
    constexpr int U = 8;
    for (i64 q0 = t; q0 < total4; q0 += U * T4) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const i64 q = q0 + i64(u) * T4;
        v[u] = q < total4 ? in[q] : first;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const u32 k = orderable(x[e]);
          lo[e] = min(lo[e], k);
          nhi[e] = min(nhi[e], ~k);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = int((4 * t + e) % dim);
      atomicMin(&sb[c], lo[e]);
      atomicMin(&sb[dim + c], nhi[e]);
    }
  }
  if (t == 0) {
    for (i64 f = total4 * 4; f < total; ++f) {
      const u32 k = orderable(p.pts[f]);
      const int c = int(f % dim);
      atomicMin(&sb[c], k);
      atomicMin(&sb[dim + c], ~k);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * dim; c += kBlock) {
    if (sb[c] != 0xffffffffu)
      atomicMin(reinterpret_cast<unsigned long long*>(box + c), (unsigned long long)sb[c]);
  }
}

__global__ void k_top_root_cell(const i64* __restrict__ box, int dim, float* __restrict__ cells) {
  for (int c = threadIdx.x; c < dim; c += blockDim.x) {
    cells[2 * c] = from_orderable(u32(box[c]));
    cells[2 * c + 1] = from_orderable(~u32(box[dim + c]));
  }
}

// ---- route + histogram ---------------------------------------------------------------
__device__ __forceinline__ void load_params(BucketParams* prm, const float* cells, int first, int nodes, int dim,
                                            int axis, int bins) {
  for (int j = threadIdx.x; j < nodes; j += blockDim.x) {
    const float* c = cells + (size_t(first + j) * dim + axis) * 2;
    prm[j] = make_params(c[0], c[1], bins);
  }
}

__global__ __launch_bounds__(kBlock) void k_top_route_hist(TopPoints p, u32* __restrict__ node, int level,
                                                           const u64* __restrict__ pivots, int prev_axis, int axis,
                                                           const float* __restrict__ cells, int bins,
                                                           u32* __restrict__ hist) {
  extern __shared__ __align__(16) u32 sh[];
  __shared__ BucketParams prm[kTopMaxNodes];
  const int nodes = 1 << level;
  const u32 first = u32(nodes - 1);
  const int nb_total = nodes * bins;
  for (int b = threadIdx.x; b < nb_total; b += kBlock) sh[b] = 0;
  load_params(prm, cells, int(first), nodes, p.dim, axis, bins);
  __syncthreads();
  const i64 stride = i64(gridDim.x) * kBlock;
  // kU rows per thread per round, every load of a round issued before its atomics
  constexpr int kU = 4;
  for (i64 base = i64(blockIdx.x) * kBlock + threadIdx.x; base < p.n; base += kU * stride) {
    u32 hn[kU];
    float kp[kU], ka[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const i64 i = base + u * stride;
      const i64 ii = i < p.n ? i : 0;
      hn[u] = level > 1 ? node[ii] : 0u;
      kp[u] = p.pts[ii * p.dim + prev_axis];
      ka[u] = p.pts[ii * p.dim + axis];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const i64 i = base + u * stride;
      if (i >= p.n) continue;
      u32 h = 0;
      if (level > 0) {
        h = route_key(hn[u], kp[u], p, i, pivots);
        node[i] = h;
      }
      if (h == kTopDone) continue;
      const u32 j = h - first;
      atomicAdd(&sh[j * bins + bucket_of(ka[u], prm[j], bins)], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb_total; b += kBlock) {
    const u32 v = sh[b];
    if (v) atomicAdd(&hist[b], v);
  }
}

// ---- median bucket per node ----------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_top_select(const u32* __restrict__ hist, int level, int bins,
                                                       TopSizes sizes, u32* __restrict__ sel, u32* __restrict__ err,
                                                       u32* __restrict__ zero_hist, u32* __restrict__ zero_hdr) {
  __shared__ u32 part[kBlock];
  const int j = blockIdx.x;
  // the next level's histogram (kTopBins words, one slice per block) and the staging header:
  // zeroed here instead of by separate fill launches
  if (zero_hist) {
    const int per = kTopBins >> level;
    for (int b = threadIdx.x; b < per; b += kBlock) zero_hist[j * per + b] = 0u;
  }
  if (zero_hdr && j == 0 && threadIdx.x < 4) zero_hdr[threadIdx.x] = 0u;
  const u32* hs = hist + size_t(j) * bins;
  const i64 size = sizes.n[j];
  const int per = (bins + kBlock - 1) / kBlock;
  const int b0 = min(bins, int(threadIdx.x) * per), b1 = min(bins, b0 + per);
  u32 s = 0;
  for (int b = b0; b < b1; ++b) s += hs[b];
  // exclusive scan of the 256 partial sums: wave scans, then the wave totals
  __shared__ u32 wtot[kBlock / 64];
  const u32 incl = dev::wave_incl_scan(s);
  if (dev::lane() == 63) wtot[threadIdx.x / 64] = incl;
  __syncthreads();
  u32 wbase = 0, acc = 0;
  for (int w = 0; w < kBlock / 64; ++w) {
    wbase += w < int(threadIdx.x / 64) ? wtot[w] : 0u;
    acc += wtot[w];
  }
  part[threadIdx.x] = wbase + incl - s;
  if (threadIdx.x == 0) {
    if (i64(acc) != size) atomicOr(err, 2u);
    if (size == 0) {
      sel[4 * j + 0] = 0xffffffffu;
      sel[4 * j + 1] = 0;
      sel[4 * j + 2] = 0;
    }
  }
  __syncthreads();
  if (size == 0) return;
  const u32 r = u32(size / 2);
  const u32 ex = part[threadIdx.x];
  if (r >= ex && r < ex + s) {
    u32 c = ex;
    for (int b = b0; b < b1; ++b) {
      const u32 v = hs[b];
      if (r < c + v) {
        sel[4 * j + 0] = u32(b);
        sel[4 * j + 1] = c;
        sel[4 * j + 2] = v;
        break;
      }
      c += v;
    }
  }
}

// ---- middle-bucket compaction fused with the next level's routing and histogram ----------
// Per point of a level-l node h: its bucket b on the level's axis against the node's median
// bucket b*. b != b*: the side is already certain -> node[i] = child and (l + 1 < levels) the
// point counts into the child's histogram of the next axis, bucketed over h's cell (so a
// node's histogram is always bucketed over its PARENT's cell: the only cell known before the
// parent's pivot; for dim >= 2 it equals the node's own cell on that axis). b == b*: the row
// is staged for the exact pivot; top_fixup routes it once the pivot is known. One pass per
// level instead of a collect pass plus a route+histogram pass.
// Staged row: coordinates, id bits, node h, input row index (dim + 3 words).
__global__ __launch_bounds__(kBlock) void k_top_collect_route(TopPoints p, u32* __restrict__ node, int level,
                                                              int axis, int next_axis, const float* __restrict__ cells,
                                                              int bins, int next_bins, const u32* __restrict__ sel,
                                                              float* __restrict__ buf, i64 cap,
                                                              u32* __restrict__ hist_next, int radix) {
  extern __shared__ __align__(16) u32 nh[];  // next level's histogram (2 * nodes * next_bins words)
  __shared__ BucketParams prm[kTopMaxNodes], nprm[kTopMaxNodes];
  __shared__ u32 bs[kTopMaxNodes];
  const int nodes = 1 << level;
  const u32 first = u32(nodes - 1);
  const bool has_next = hist_next != nullptr;
  const int nb_next = has_next ? 2 * nodes * next_bins : 0;
  for (int b = threadIdx.x; b < nb_next; b += kBlock) nh[b] = 0;
  // level-l bucket ranges: the parent's cell (see k_top_select's histograms: at level l >= 1
  // they are built by the previous level's pass, which knows only the parent's cell)
  for (int j = threadIdx.x; j < nodes; j += kBlock) {
    const int hc = level == 0 ? 0 : (int(first) + j - 1) / 2;
    const float* c = cells + (size_t(hc) * p.dim + axis) * 2;
    prm[j] = make_params(c[0], c[1], bins);
  }
  if (has_next) load_params(nprm, cells, int(first), nodes, p.dim, next_axis, next_bins);
  for (int j = threadIdx.x; j < nodes; j += kBlock) bs[j] = sel[4 * j];
  __syncthreads();
  u32* count = reinterpret_cast<u32*>(buf);
  float* rows = buf + 4;
  const int rs = p.dim + 3;
  // A block notes its median-bucket rows in LDS and reserves them with ONE global atomic at
  // the end: the count word is shared by every block of every XCD, and per-wave atomics on it
  // serialise at the memory side (~1 us each). Rows beyond the staging take the direct path.
  constexpr int kStage = 1024;
  __shared__ u32 sidx[kStage];
  __shared__ u32 scount, sbase;
  if (threadIdx.x == 0) scount = 0;
  __syncthreads();
  auto write_row = [&](i64 slot, i64 i, u32 h) {
    if (slot >= cap) {
      // the median bucket overflowed its staging slots: the pivot kernel flags it and the
      // whole top-level pass is retried with larger slots; until then the row still gets a
      // valid child, so every later kernel indexes in range
      node[i] = 2 * h + 1;
      return;
    }
    float* o = rows + slot * rs;
    const float* r = p.pts + i * p.dim;
    for (int c = 0; c < p.dim; ++c) o[c] = r[c];
    o[p.dim] = __uint_as_float(point_id(p, i));
    o[p.dim + 1] = __uint_as_float(h);
    o[p.dim + 2] = __uint_as_float(u32(i));
  };
  const i64 stride = i64(gridDim.x) * kBlock;
  // the trip count is uniform across the wave (ballots below need every lane); kU rows per
  // thread per round with their loads issued together
  constexpr int kU = 4;
  for (i64 base0 = i64(blockIdx.x) * kBlock; base0 < p.n; base0 += kU * stride) {
    u32 hn[kU];
    float ka[kU], kn[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const i64 i = base0 + u * stride + threadIdx.x;
      const i64 ii = i < p.n ? i : 0;
      hn[u] = level > 0 ? node[ii] : 0u;
      ka[u] = p.pts[ii * p.dim + axis];
      kn[u] = has_next ? p.pts[ii * p.dim + next_axis] : 0.0f;  // the last top level has no next histogram
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const i64 i = base0 + u * stride + threadIdx.x;
      bool take = false;
      const u32 h = hn[u];
      if (i < p.n && h != kTopDone && h - first < u32(nodes)) {
        const u32 j = h - first;
        const u32 b = bucket_of(ka[u], prm[j], bins), bst = bs[j];
        take = b == bst;
        if (!take) {
          const u32 c = b < bst ? 0u : 1u;
          node[i] = 2 * h + 1 + c;
          if (has_next) atomicAdd(&nh[(2 * j + c) * next_bins + bucket_of(kn[u], nprm[j], next_bins)], 1u);
        } else if (radix) {
          node[i] = h;  // stays at its node: the distributed radix rounds find the pivot among these
          take = false;
        }
      }
      const u64 m = __ballot(take);
      if (!m) continue;
      const int leader = __ffsll((long long)m) - 1;
      u32 lbase = 0;
      if (dev::lane() == leader) lbase = atomicAdd(&scount, u32(__popcll(m)));
      lbase = __shfl(lbase, leader, 64);
      const u32 ls = lbase + mbcnt(m);
      if (take && ls < u32(kStage)) sidx[ls] = u32(i);
      const bool direct = take && ls >= u32(kStage);
      if (__ballot(direct)) {  // staging full (a very skewed block): reserve per wave
        const u64 md = __ballot(direct);
        const int ld = __ffsll((long long)md) - 1;
        u32 gb = 0;
        if (dev::lane() == ld) gb = atomicAdd(count, u32(__popcll(md)));
        gb = __shfl(gb, ld, 64);
        if (direct) write_row(i64(gb) + mbcnt(md), i, h);
      }
    }
  }
  __syncthreads();
  const u32 staged = min(scount, u32(kStage));
  if (threadIdx.x == 0) sbase = staged ? atomicAdd(count, staged) : 0u;
  __syncthreads();
  for (u32 k = threadIdx.x; k < staged; k += kBlock) {
    const i64 i = sidx[k];
    write_row(i64(sbase) + k, i, level > 0 ? node[i] : 0u);
  }
  for (int b = threadIdx.x; b < nb_next; b += kBlock) {
    const u32 v = nh[b];
    if (v) atomicAdd(&hist_next[b], v);
  }
}

// The staged (median-bucket) rows of this rank, once the level's pivots are known: route each
// below its node's pivot (the pivot itself -> kTopDone) and count it into the next histogram.
__global__ __launch_bounds__(kBlock) void k_top_fixup(const float* __restrict__ buf, i64 cap, int dim, int level,
                                                      int axis, int next_axis, const u64* __restrict__ pivots,
                                                      const float* __restrict__ cells, int next_bins,
                                                      u32* __restrict__ node, u32* __restrict__ hist_next) {
  const u32 cnt = min(u32(cap), reinterpret_cast<const u32*>(buf)[0]);
  const float* rows = buf + 4;
  const u32 first = u32((1 << level) - 1);
  for (u32 k = blockIdx.x * kBlock + threadIdx.x; k < cnt; k += gridDim.x * kBlock) {
    const float* r = rows + i64(k) * (dim + 3);
    const u32 h = __float_as_uint(r[dim + 1]);
    if (h - first >= u32(1 << level)) continue;  // never: staged rows carry their level's node
    const u64 ck = composite_key(r[axis], __float_as_uint(r[dim]));
    const u64 pv = pivots[h];
    const u32 child = ck < pv ? 2 * h + 1 : (ck > pv ? 2 * h + 2 : kTopDone);
    node[__float_as_uint(r[dim + 2])] = child;
    if (hist_next != nullptr && child != kTopDone) {
      const u32 j = h - first;
      const float* c = cells + (size_t(h) * dim + next_axis) * 2;
      const BucketParams np = make_params(c[0], c[1], next_bins);
      atomicAdd(&hist_next[(child - 2 * first - 1) * next_bins + bucket_of(r[next_axis], np, next_bins)], 1u);
      (void)j;
    }
  }
}

// ---- exact pivot per node (radix select over the gathered middles) ---------------------
struct MidView {
  const float* g;
  i64 stride;  // words per rank buffer
  i64 cap;
  int P, dim, axis;
  __device__ u32 count(int r) const { return min(u32(cap), reinterpret_cast<const u32*>(g + r * stride)[0]); }
  __device__ const float* row(int r, u32 k) const { return g + r * stride + 4 + i64(k) * (dim + 3); }
  __device__ u64 key(const float* row) const {
    return composite_key(row[axis], __float_as_uint(row[dim]));
  }
  __device__ u32 node(const float* row) const { return __float_as_uint(row[dim + 1]); }
};

__global__ __launch_bounds__(kPivotThreads) void k_top_pivot(MidView mv, int level, TopSizes sizes,
                                                             const u32* __restrict__ sel, u64* __restrict__ pivots,
                                                             float* __restrict__ top_rows, float* __restrict__ cells,
                                                             u32* __restrict__ err) {
  extern __shared__ __align__(16) u64 keys[];  // [kPivotLdsKeys], then u32 locs[kPivotLdsKeys]
  u32* locs = reinterpret_cast<u32*>(keys + kPivotLdsKeys);  // (rank << 26) | row of keys[i]
  __shared__ u32 hist[256];
  __shared__ u32 s_cnt, s_digit, s_rem, s_found, s_bincnt;
  __shared__ u64 s_mn[kPivotThreads / 64], s_mx[kPivotThreads / 64], s_one;
  const int j = blockIdx.x;
  const u32 h = u32((1 << level) - 1 + j);
  const int dim = mv.dim, axis = mv.axis;
  const int tid = threadIdx.x;
  const i64 size = sizes.n[j];
  float* cl = cells + size_t(2 * h + 1) * dim * 2;
  float* cr = cells + size_t(2 * h + 2) * dim * 2;
  const float* cp = cells + size_t(h) * dim * 2;
  for (int c = tid; c < 2 * dim; c += kPivotThreads) {
    cl[c] = cp[c];
    cr[c] = cp[c];
  }
  if (size == 0) {
    if (tid == 0) pivots[h] = ~0ull;
    for (int c = tid; c <= dim; c += kPivotThreads) top_rows[size_t(h) * (dim + 1) + c] = 0.0f;
    return;
  }
  __shared__ u32 s_pre[kTopMaxRanks + 1];  // rank r's middle rows: s_pre[r + 1] - s_pre[r]
  static_assert(kTopMaxRanks == 64, "one lane per rank");
  if (tid < 64) {  // lane r: rank r's row count (all loads in flight at once), a wave scan
    const int r = tid;
    const u32 raw = r < mv.P ? reinterpret_cast<const u32*>(mv.g + r * mv.stride)[0] : 0u;
    if (raw > u32(mv.cap)) atomicOr(err, 1u);
    const u32 c = min(raw, u32(mv.cap));
    const u32 incl = dev::wave_incl_scan(c);
    if (r < mv.P) s_pre[r] = incl - c;
    if (r == mv.P - 1) s_pre[mv.P] = incl;
    if (r == 0) {
      s_cnt = 0;
      s_found = 0;
    }
  }
  __syncthreads();
  // 1. this node's keys into LDS (one reservation per wave, not one same-address atomic per
  // row), with their range
  u64 mn = ~0ull, mx = 0ull;
  constexpr int U = 4;  // rows per thread per round: their loads in flight together (one block
                        // per node walks every rank's middle rows, so rounds are latency-bound)
  // (one flat index space over all ranks with 16 rows per thread, a binary search per row for its
  // rank, measured slower: P = 8 levels 1 / 2 48 -> 58 / 67 -> 74 us; U = 8 per rank: 36 -> 47 us at level 0)
  for (int r = 0; r < mv.P; ++r) {
    const u32 c = s_pre[r + 1] - s_pre[r];
    for (u32 k0 = 0; k0 < c; k0 += U * kPivotThreads) {  // uniform trip count: wave ballots below
      bool mine[U];
      u64 key[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const u32 k = k0 + u * kPivotThreads + tid;
        const float* row = mv.row(r, k < c ? k : 0u);
        const u32 nd = mv.node(row);  // loaded unconditionally: no wait per row
        key[u] = mv.key(row);
        mine[u] = (k < c) & (nd == h);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const u64 m = __ballot(mine[u]);
        if (!m) continue;
        const int leader = __ffsll((long long)m) - 1;
        u32 base = 0;
        if (dev::lane() == leader) base = atomicAdd(&s_cnt, u32(__popcll(m)));
        base = u32(__shfl(int(base), leader, 64));
        if (mine[u]) {
          const u32 sidx = base + mbcnt(m);
          if (sidx < u32(kPivotLdsKeys)) {
            keys[sidx] = key[u];
            locs[sidx] = (u32(r) << 26) | (k0 + u * kPivotThreads + tid);
          }
          mn = key[u] < mn ? key[u] : mn;
          mx = key[u] > mx ? key[u] : mx;
        }
      }
    }
  }
  mn = dev::wave_min_u64(mn);
  mx = dev::wave_max_u64(mx);
  if (dev::lane() == 0) {
    s_mn[tid / 64] = mn;
    s_mx[tid / 64] = mx;
  }
  __syncthreads();
  const u32 m = s_cnt;
  const u32 cmid = sel[4 * j + 2];
  const u32 target = u32(size / 2) - sel[4 * j + 1];
  if (m != cmid || target >= m) {
    if (tid == 0) {
      atomicOr(err, 1u);
      pivots[h] = ~0ull;
    }
    return;
  }
  mn = s_mn[0];
  mx = s_mx[0];
  for (int w = 1; w < kPivotThreads / 64; ++w) {
    mn = s_mn[w] < mn ? s_mn[w] : mn;
    mx = s_mx[w] > mx ? s_mx[w] : mx;
  }
  const bool in_lds = m <= u32(kPivotLdsKeys);
  // 2. radix select, 8 bits per pass from the highest bit in which the keys differ (the median
  // bucket's keys share their top bits: those passes are skipped). Histogram adds: one per
  // wave when all its lanes carry the same digit, else one per lane.
  u64 prefix = mn;
  u32 rem = target;
  const u64 diff = mn ^ mx;
  int hb = diff ? 63 - __builtin_clzll(diff) : -1;
  prefix = hb >= 63 ? 0ull : (hb < 0 ? mn : (mn & ~((2ull << hb) - 1ull)));
  while (hb >= 0) {
    const int shift = hb >= 7 ? hb - 7 : 0;
    const u32 dmask = (2u << (hb - shift)) - 1u;
    const u64 hmask = hb >= 63 ? 0ull : ~((2ull << hb) - 1ull);
    for (int b = tid; b < 256; b += kPivotThreads) hist[b] = 0;
    __syncthreads();
    auto add = [&](bool act, u32 d) {
      const u64 am = __ballot(act);
      if (!am) return;
      const int l0 = __ffsll((long long)am) - 1;
      const u32 d0 = u32(__shfl(int(d), l0, 64));
      if (__ballot(act && d == d0) == am) {
        if (dev::lane() == l0) atomicAdd(&hist[d0], u32(__popcll(am)));
      } else if (act) {
        atomicAdd(&hist[d], 1u);
      }
    };
    if (in_lds) {
      for (u32 k0 = 0; k0 < m; k0 += kPivotThreads) {
        const u32 k = k0 + tid;
        const u64 key = k < m ? keys[k] : 0ull;
        add(k < m && (key & hmask) == prefix, u32(key >> shift) & dmask);
      }
    } else {
      for (int r = 0; r < mv.P; ++r) {
        const u32 c = mv.count(r);
        for (u32 k0 = 0; k0 < c; k0 += kPivotThreads) {
          const u32 k = k0 + tid;
          bool act = false;
          u64 key = 0;
          if (k < c) {
            const float* row = mv.row(r, k);
            key = mv.key(row);
            act = mv.node(row) == h && (key & hmask) == prefix;
          }
          add(act, u32(key >> shift) & dmask);
        }
      }
    }
    __syncthreads();
    if (tid < 64) {
      const int l = tid;
      u32 v[4], s = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = hist[4 * l + q];
        s += v[q];
      }
      const u32 incl = dev::wave_incl_scan(s);
      u32 c = incl - s;
      if (rem >= c && rem < incl) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (rem >= c && rem < c + v[q]) {
            s_digit = u32(4 * l + q);
            s_rem = rem - c;
            s_bincnt = v[q];
          }
          c += v[q];
        }
      }
    }
    __syncthreads();
    prefix |= u64(s_digit & dmask) << shift;
    rem = s_rem;
    hb = shift - 1;
    if (s_bincnt == 1u && hb >= 0 && in_lds) {
      // one candidate left (its key digits are distinct from every other row's): it is the pivot
      const u64 hm = ~((2ull << hb) - 1ull);
      for (u32 k = tid; k < m; k += kPivotThreads)
        if ((keys[k] & hm) == prefix) s_one = keys[k];
      __syncthreads();
      prefix = s_one;
      hb = -1;
    }
    __syncthreads();
  }
  // 3. the pivot row (composite keys are unique): from its LDS location, else by walking the rows
  auto take = [&](const float* row) {
    s_found = 1;
    pivots[h] = prefix;
    float* tr = top_rows + size_t(h) * (dim + 1);
    for (int q = 0; q <= dim; ++q) tr[q] = row[q];
    cl[2 * axis + 1] = row[axis];
    cr[2 * axis] = row[axis];
  };
  // locations fit 26 bits of row index while every rank holds < 2^26 middle rows
  const bool by_loc = in_lds && s_pre[mv.P] < (1u << 26);
  if (by_loc) {
    for (u32 k = tid; k < m; k += kPivotThreads)
      if (keys[k] == prefix) take(mv.row(int(locs[k] >> 26), locs[k] & ((1u << 26) - 1u)));
  }
  for (int r = 0; r < (by_loc ? 0 : mv.P); ++r) {
    const u32 c = s_pre[r + 1] - s_pre[r];
    for (u32 k0 = 0; k0 < c; k0 += U * kPivotThreads) {
      bool hit[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const u32 k = k0 + u * kPivotThreads + tid;
        const float* row = mv.row(r, k < c ? k : 0u);
        const u32 nd = mv.node(row);
        const u64 kk = mv.key(row);
        hit[u] = (k < c) & (nd == h) & (kk == prefix);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!hit[u]) continue;
        take(mv.row(r, k0 + u * kPivotThreads + tid));
      }
    }
  }
  __syncthreads();
  if (tid == 0 && !s_found) atomicOr(err, 1u);
}

// ---- counting sort by destination leaf (T <= 64 leaves) --------------------------------
// Rows are grouped by top-level leaf; which rank receives a leaf in which exchange round is
// the host planner's business (global_plan::make_plan), so the kernels never see ranks.
__global__ __launch_bounds__(kBlock) void k_pack_count(const u32* __restrict__ node, i64 n, int levels, int T,
                                                       i64 per_block, u32* __restrict__ bcount) {
  __shared__ u32 cnt[64];
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const i64 b0 = i64(blockIdx.x) * per_block, b1 = min(n, b0 + per_block);
  const u32 first = u32(T - 1);
  for (i64 i = b0 + threadIdx.x; i < b1; i += kBlock) {
    // the top levels left every point at its leaf (or kTopDone for pivots); no top levels:
    // every point is at the root's single leaf and `node` was never written
    const u32 h = levels > 0 ? node[i] : 0u;
    // out-of-range nodes (a bug) are dropped: the leaf totals then fail the plan's geometry
    // check on every rank instead of indexing out of bounds here
    if (h != kTopDone && h - first < u32(T)) atomicAdd(&cnt[h - first], 1u);
  }
  __syncthreads();
  if (threadIdx.x < T) bcount[i64(blockIdx.x) * T + threadIdx.x] = cnt[threadIdx.x];
}

// offsets[block][d] = sum_{d' < d} total[d'] + sum_{b' < block} bcount[b'][d]: one workgroup per
// destination d, a block-wide scan of its column (blocks <= 2 * kScanThreads) plus a block-wide
// sum of the columns before it. (One thread per destination walking all blocks took 158 us
// at 1526 blocks: a chain of dependent loads.)
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void k_pack_scan(const u32* __restrict__ bcount, int blocks, int P,
                                                            u32* __restrict__ offsets, i64* __restrict__ counts,
                                                            const u32* __restrict__ err) {
  constexpr int W = kScanThreads / 64;
  __shared__ u32 wsum[W], wbef[W];
  const int d = blockIdx.x, tid = threadIdx.x, w = tid / 64, ln = tid & 63;
  u32 before = 0;
  for (int b = tid; b < blocks; b += kScanThreads)
    for (int e = 0; e < d; ++e) before += bcount[i64(b) * P + e];
  const int C = (blocks + kScanThreads - 1) / kScanThreads;  // 1 or 2
  const int b0 = tid * C;
  const bool in0 = b0 < blocks, in1 = C > 1 && b0 + 1 < blocks;
  const u32 x0 = in0 ? bcount[i64(b0) * P + d] : 0u;
  const u32 x1 = in1 ? bcount[i64(b0 + 1) * P + d] : 0u;
  const u32 sum = x0 + x1;
  const u32 incl = dev::wave_incl_scan(sum);
  u32 bw = before;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bw += __shfl_xor(bw, o, 64);
  if (ln == 63) wsum[w] = incl;
  if (ln == 0) wbef[w] = bw;
  __syncthreads();
  u32 pre = 0, tot = 0, base = 0;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const u32 v = wsum[k];
    pre += k < w ? v : 0u;
    tot += v;
    base += wbef[k];
  }
  u32 run = base + pre + incl - sum;
  if (in0) offsets[i64(b0) * P + d] = run;
  run += x0;
  if (in1) offsets[i64(b0 + 1) * P + d] = run;
  if (tid == 0) {
    counts[4 * d] = i64(tot);
    counts[4 * d + 1] = i64(*err);
  }
}

// cs == 0: rows of rs floats; cs > 0: SoA planes of stride cs (ids never travel in planes: the
// planar exchange is always the compact one). bm != nullptr: the leaf bitmaps of the compact
// exchange come from the same ballots (a block's rows start on a multiple of 256, so wave w's
// 64 rows of a chunk are exactly bitmap words 2 k and 2 k + 1 of every leaf).
// Four 256-row sub-chunks per round: their node loads, then their rows' loads, are in flight
// together; sub-chunks are ranked in order, so each leaf's rows stay in source-row order.
__global__ __launch_bounds__(kBlock) void k_pack_scatter(TopPoints p, const u32* __restrict__ node, int levels, int T,
                                                         i64 per_block, const u32* __restrict__ offsets,
                                                         float* __restrict__ out, int rs, i64 cs, u32* __restrict__ bm,
                                                         i64 bm_words) {
  constexpr int U = 4;
  __shared__ u32 cur[64];
  __shared__ u32 wcnt[U][kBlock / 64][64];
  const u32 first = u32(T - 1);
  if (threadIdx.x < T) cur[threadIdx.x] = offsets[i64(blockIdx.x) * T + threadIdx.x];
  __syncthreads();
  const i64 b0 = i64(blockIdx.x) * per_block, b1 = min(p.n, b0 + per_block);
  const int w = threadIdx.x / 64, ln = dev::lane();
  const int dim = p.dim;
  for (i64 c0 = b0; c0 < b1; c0 += U * kBlock) {
    int d[U];
    u32 my[U];
    float3 row3[U];  // dim 3: the rows are loaded with their nodes, before the ranking (the
                     // stores below would otherwise wait on each row's load in turn)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i64 i = c0 + u * kBlock + threadIdx.x;
      const u32 h = i < b1 ? (levels > 0 ? node[i] : 0u) : kTopDone;
      d[u] = (h == kTopDone || h - first >= u32(T)) ? -1 : int(h - first);
      if (dim == 3) row3[u] = *reinterpret_cast<const float3*>(p.pts + (i < b1 ? i : b0) * 3);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      my[u] = 0;
      const i64 word = (c0 + u * kBlock + 64 * w) / 32;  // this wave's first bitmap word
      for (int e = 0; e < T; ++e) {  // stable rank among same-destination points of the sub-chunk
        const u64 m = __ballot(d[u] == e);
        if (ln == 0) wcnt[u][w][e] = __popcll(m);
        if (d[u] == e) my[u] = mbcnt(m);
        if (bm && ln < 2 && word + ln < bm_words && c0 + u * kBlock < b1)
          bm[i64(e) * bm_words + word + ln] = ln == 0 ? u32(m) : u32(m >> 32);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (d[u] < 0) continue;
      const i64 i = c0 + u * kBlock + threadIdx.x;
      u32 off = cur[d[u]];
      for (int uu = 0; uu < u; ++uu)
        for (int v = 0; v < kBlock / 64; ++v) off += wcnt[uu][v][d[u]];
      for (int v = 0; v < w; ++v) off += wcnt[u][v][d[u]];
      const i64 k = i64(off + my[u]);
      const float* r = p.pts + i * dim;
      if (cs > 0) {
        if (dim == 3) {  // one 12-B row load, three coalesced plane stores
          const float3 v = row3[u];
          out[k] = v.x;
          out[cs + k] = v.y;
          out[2 * cs + k] = v.z;
        } else {
          for (int c = 0; c < dim; ++c) out[c * cs + k] = r[c];
        }
      } else {
        float* o = out + k * rs;
        if (dim == 3) {  // one 12-B load and store per row (dwordx3) instead of three dword pairs
          *reinterpret_cast<float3*>(o) = row3[u];
        } else {
          for (int c = 0; c < dim; ++c) o[c] = r[c];
        }
        if (rs > dim) o[dim] = __uint_as_float(point_id(p, i));
      }
    }
    __syncthreads();
    if (threadIdx.x < T) {
      u32 add = 0;
#pragma unroll
      for (int u = 0; u < U; ++u)
        for (int v = 0; v < kBlock / 64; ++v) add += wcnt[u][v][threadIdx.x];
      cur[threadIdx.x] += add;
    }
    __syncthreads();
  }
}

// Receiver side: popcount sums of kBmWords-word blocks of every source's bitmap.
constexpr int kBmWords = 2048;  // words per block (8 per thread)
__global__ __launch_bounds__(kBlock) void k_bm_block_sums(const u32* __restrict__ bm, BmSources srcs, int nblk,
                                                          u32* __restrict__ bsum) {
  const int s = blockIdx.y, b = blockIdx.x;
  const u32* src = bm + srcs.bm_off[s];
  const i64 ws = srcs.words[s];
  u32 c = 0;
  for (int k = threadIdx.x; k < kBmWords; k += kBlock) {
    const i64 w = i64(b) * kBmWords + k;
    c += w < ws ? u32(__popc(src[w])) : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ u32 part[kBlock / 64];
  if (dev::lane() == 0) part[threadIdx.x / 64] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 t = 0;
    for (int v = 0; v < kBlock / 64; ++v) t += part[v];
    bsum[i64(s) * nblk + b] = t;
  }
}

// ids[recv_off[s] + k] = id_base[s] + (position of the k-th set bit of source s's bitmap):
// the rows of a source arrive in its stable pack order, i.e. by increasing source row.
// Words are taken lane-consecutively (word w0 + j * kBlock + tid for round j), so every round's
// ids land in one contiguous run: each lane writes its ~4 set bits (at 1/8 density) next to
// its neighbours' instead of walking 256 bits of its own range alone.
__global__ __launch_bounds__(kBlock) void k_bm_ids(const u32* __restrict__ bm, int nblk, const u32* __restrict__ bsum,
                                                   BmSources src, u32* __restrict__ ids, u32* __restrict__ err) {
  constexpr int kPer = kBmWords / kBlock;
  const int s = blockIdx.y, b = blockIdx.x;
  const i64 ws = src.words[s];
  const i64 last = ws > 0 ? (ws - 1) / kBmWords : 0;  // this source's last block
  if (b > last) return;
  __shared__ u32 part[kBlock / 64];
  __shared__ u32 wtot[kPer][kBlock / 64];
  // set bits in blocks before b
  u32 pre = 0;
  for (int k = threadIdx.x; k < b; k += kBlock) pre += bsum[i64(s) * nblk + k];
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (dev::lane() == 0) part[threadIdx.x / 64] = pre;
  const u32* sb = bm + src.bm_off[s];
  const i64 wb = i64(b) * kBmWords;
  const int wv = threadIdx.x / 64;
  u32 words[kPer], incl[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const i64 w = wb + j * kBlock + threadIdx.x;
    words[j] = w < ws ? sb[w] : 0u;
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    incl[j] = dev::wave_incl_scan(u32(__popc(words[j])));
    if (dev::lane() == 63) wtot[j][wv] = incl[j];
  }
  __syncthreads();
  u32 run = 0;  // set bits of this block before round j
  for (int v = 0; v < kBlock / 64; ++v) run += part[v];
  const i64 off = src.off[s];
  const u32 idb = src.base[s];
  const i64 cap = src.cnt[s];
  u32 k = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    u32 before = 0, tot = 0;
    for (int v = 0; v < kBlock / 64; ++v) {
      if (v < wv) before += wtot[j][v];
      tot += wtot[j][v];
    }
    u32 x = words[j];
    k = run + before + incl[j] - u32(__popc(x));
    const i64 w = wb + j * kBlock + threadIdx.x;
    while (x) {
      const int t = __ffs(int(x)) - 1;
      x &= x - 1;
      if (i64(k) < cap) ids[off + k] = idb + u32(w * 32 + t);
      else atomicOr(err, 8u);
      ++k;
    }
    run += tot;
  }
  if (b == last && threadIdx.x == 0 && i64(run) != cap) atomicOr(err, 8u);
}

// pattern fill of 64-bit words; words j with (j % period) == slot get `alt` instead (the count
// matrix's id-base / n_local columns)
__global__ void k_fill64(u64* __restrict__ p, i64 n, u64 v, int period, int slot_a, u64 alt_a, int slot_b,
                         u64 alt_b) {
  for (i64 j = i64(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += i64(gridDim.x) * blockDim.x) {
    const int r = period > 0 ? int(j % period) : -1;
    p[j] = (period > 0 && r == slot_a) ? alt_a : ((period > 0 && r == slot_b) ? alt_b : v);
  }
}

// blockIdx.y: the segment
__global__ void k_fill64_multi(FillSegs f) {
  const int i = blockIdx.y;
  u64* p = f.p[i];
  const u64 v = f.v[i];
  for (i64 j = i64(blockIdx.x) * blockDim.x + threadIdx.x; j < f.n[i]; j += i64(gridDim.x) * blockDim.x) p[j] = v;
}

int pack_blocks(i64 n) { return int(std::max<i64>(1, std::min<i64>(2048, (n + 8191) / 8192))); }
int stream_grid(i64 n) { return int(std::max<i64>(1, std::min<i64>(512, (n + 16383) / 16384))); }

}  // namespace

void fill_u64_multi(const FillSegs& f, hipStream_t stream) {
  if (f.count <= 0) return;
  if (f.count > kFillSegs) throw std::invalid_argument("fill_u64_multi: too many segments");
  i64 nmax = 0;
  for (int i = 0; i < f.count; ++i) nmax = std::max(nmax, f.n[i]);
  const int gx = int(std::max<i64>(1, std::min<i64>(64, (nmax + 255) / 256)));
  k_fill64_multi<<<dim3(gx, f.count), 256, 0, stream>>>(f);
  PKD_LAUNCH_CHECK();
}

void fill_u64(void* p, i64 n, u64 v, hipStream_t stream) {
  if (n <= 0) return;
  k_fill64<<<int(std::min<i64>(1024, (n + 255) / 256)), 256, 0, stream>>>(static_cast<u64*>(p), n, v, 0, -1, 0, -1, 0);
  PKD_LAUNCH_CHECK();
}

namespace {
__global__ void k_fill32(u32* __restrict__ p, i64 n, u32 v) {
  for (i64 i = i64(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += i64(gridDim.x) * blockDim.x) p[i] = v;
}
}  // namespace

void fill_u32(void* p, i64 n, u32 v, hipStream_t stream) {
  if (n <= 0) return;
  k_fill32<<<int(std::min<i64>(1024, (n + 255) / 256)), 256, 0, stream>>>(static_cast<u32*>(p), n, v);
  PKD_LAUNCH_CHECK();
}

void top_counts_init(i64* counts, int slots, i64 id_base, i64 n_local, hipStream_t stream) {
  k_fill64<<<1, 256, 0, stream>>>(reinterpret_cast<u64*>(counts), i64(slots) * 4, 0, 4, 2, u64(id_base), 3,
                                  u64(n_local));
  PKD_LAUNCH_CHECK();
}

void top_bbox(const TopPoints& p, i64* box, hipStream_t stream) {
  if (p.n <= 0) return;
  const int dim = p.dim;
  if (reinterpret_cast<uintptr_t>(p.pts) % 16 == 0 && p.n * dim >= 4) {
    // 4 T4 a multiple of dim: T4 a multiple of dim / gcd(dim, 4)
    const i64 g = dim % 4 == 0 ? 4 : (dim % 2 == 0 ? 2 : 1), unit = dim / g;
    // 512 blocks x 8 float4 in flight per thread: the read still streams at full rate, and each
    // box word takes 512 same-address global atomics instead of 2048 (they serialise at the
    // memory side: 46 us for 12.5 M x 3D with 2048 blocks)
    const i64 want = std::min<i64>((p.n * dim) / 4, i64(kBboxBlocks) * kBlock);
    const i64 T4 = std::max<i64>(unit, (want / unit) * unit);
    k_top_bbox4<<<int((T4 + kBlock - 1) / kBlock), kBlock, size_t(2) * dim * 4, stream>>>(p, T4, box);
    PKD_LAUNCH_CHECK();
    return;
  }
  // up to kBboxBlocks blocks of 8 loads in flight per thread; one LDS-reduced atomic pair per block and axis
  const i64 want = std::min<i64>(p.n * dim, i64(kBboxBlocks) * kBlock);
  const i64 T = std::max<i64>(dim, (want / dim) * dim);
  const int grid = int((T + kBlock - 1) / kBlock);
  k_top_bbox<<<grid, kBlock, size_t(2) * dim * 4, stream>>>(p, T, box);
  PKD_LAUNCH_CHECK();
}

void top_root_cell(const i64* box, int dim, float* cells, hipStream_t stream) {
  k_top_root_cell<<<1, 256, 0, stream>>>(box, dim, cells);
  PKD_LAUNCH_CHECK();
}

void top_route_hist(const TopPoints& p, u32* node, int level, const u64* pivots, int prev_axis, int axis,
                    const float* cells, int bins, u32* hist, hipStream_t stream) {
  if ((1 << level) > kTopMaxNodes) throw std::invalid_argument("top_route_hist: too many nodes");
  const int nb_total = (1 << level) * bins;
  if (nb_total > kTopBins) throw std::invalid_argument("top_route_hist: nodes * bins exceeds 8192");
  if (p.n <= 0) return;
  k_top_route_hist<<<stream_grid(p.n), kBlock, size_t(nb_total) * 4, stream>>>(p, node, level, pivots, prev_axis,
                                                                               axis, cells, bins, hist);
  PKD_LAUNCH_CHECK();
}

void top_select(const u32* hist, int level, int bins, const TopSizes& sizes, u32* sel, u32* err, u32* zero_hist,
                u32* zero_hdr, hipStream_t stream) {
  k_top_select<<<1 << level, kBlock, 0, stream>>>(hist, level, bins, sizes, sel, err, zero_hist, zero_hdr);
  PKD_LAUNCH_CHECK();
}

size_t top_middle_words(int dim, i64 cap) { return 4 + size_t(cap) * size_t(dim + 3); }

void top_collect_route(const TopPoints& p, u32* node, int level, int axis, int next_axis, const float* cells,
                       int bins, int next_bins, const u32* sel, float* buf, i64 cap, u32* hist_next,
                       hipStream_t stream, bool radix) {
  if ((1 << level) > kTopMaxNodes) throw std::invalid_argument("top_collect_route: too many nodes");
  if (hist_next && 2 * (1 << level) * next_bins > kTopBins)
    throw std::invalid_argument("top_collect_route: next level's nodes * bins exceeds 8192");
  if (p.n <= 0) return;
  const size_t lds = hist_next ? size_t(2) * (1 << level) * next_bins * 4 : 0;
  k_top_collect_route<<<stream_grid(p.n), kBlock, lds, stream>>>(p, node, level, axis, next_axis, cells, bins,
                                                                  next_bins, sel, buf, cap, hist_next,
                                                                  radix ? 1 : 0);
  PKD_LAUNCH_CHECK();
}

void top_fixup(const float* buf, i64 cap, int dim, int level, int axis, int next_axis, const u64* pivots,
               const float* cells, int next_bins, u32* node, u32* hist_next, hipStream_t stream) {
  // the staged rows: at most cap, usually a few thousand; one small grid
  const int grid = int(std::max<i64>(1, std::min<i64>(256, (cap + kBlock - 1) / kBlock)));
  k_top_fixup<<<grid, kBlock, 0, stream>>>(buf, cap, dim, level, axis, next_axis, pivots, cells, next_bins, node,
                                           hist_next);
  PKD_LAUNCH_CHECK();
}

void top_pivot(const float* gathered, int P, i64 cap, int level, int axis, int dim, const TopSizes& sizes,
               const u32* sel, u64* pivots, float* top_rows, float* cells, u32* err, hipStream_t stream) {
  if (P < 1 || P > kTopMaxRanks) throw std::invalid_argument("top_pivot: 1 <= P <= 64 ranks");
  const size_t lds = size_t(kPivotLdsKeys) * 12;
  ensure_dynamic_lds(reinterpret_cast<const void*>(&k_top_pivot), int(lds));
  MidView mv{gathered, i64(top_middle_words(dim, cap)), cap, P, dim, axis};
  k_top_pivot<<<1 << level, kPivotThreads, lds, stream>>>(mv, level, sizes, sel, pivots, top_rows, cells, err);
  PKD_LAUNCH_CHECK();
}

// ---- median by distributed radix rounds (duplicate-heavy data) --------------------------
namespace {
// rows of level-l node h still at h after the radix-mode collect (its median bucket): 8-bit digit
// `pass` of the composite key among those matching the node's prefix above it
__global__ __launch_bounds__(kBlock) void k_top_radix_hist(TopPoints p, const u32* __restrict__ node, int level,
                                                           int axis, const TopRadix* __restrict__ rs, int pass,
                                                           u32* __restrict__ hist) {
  __shared__ u32 h[kTopMaxNodes * 256];
  __shared__ u64 pre[kTopMaxNodes];
  const int nodes = 1 << level;
  const u32 first = u32(nodes - 1);
  for (int b = threadIdx.x; b < nodes * 256; b += kBlock) h[b] = 0;
  for (int j = threadIdx.x; j < nodes; j += kBlock) pre[j] = rs[j].prefix;
  __syncthreads();
  const int shift = 8 * pass;
  const u64 hmask = pass == 7 ? 0ull : (~0ull << (shift + 8));
  const i64 stride = i64(gridDim.x) * kBlock;
  for (i64 i = i64(blockIdx.x) * kBlock + threadIdx.x; i < p.n; i += stride) {
    const u32 hn = node[i];
    if (hn - first >= u32(nodes)) continue;
    const u32 j = hn - first;
    const u64 k = composite_key(p.pts[i * p.dim + axis], point_id(p, i));
    if ((k & hmask) == (pre[j] & hmask)) atomicAdd(&h[j * 256 + (u32(k >> shift) & 255u)], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nodes * 256; b += kBlock) {
    const u32 v = h[b];
    if (v) atomicAdd(&hist[b], v);
  }
}

// one wave per node: the digit holding the node's remaining rank (all ranks' histograms summed)
__global__ __launch_bounds__(64) void k_top_radix_sel(u32* __restrict__ hist, int level, int pass,
                                                      TopRadix* __restrict__ rs, u32* __restrict__ err) {
  const int j = blockIdx.x, ln = dev::lane();
  u32* hs = hist + size_t(j) * 256;
  TopRadix r = rs[j];
  if (r.active) {
    u32 v[4], s = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = hs[4 * ln + q];
      s += v[q];
    }
    const u32 incl = dev::wave_incl_scan(s);
    const u32 excl = incl - s;
    const bool mine = r.rank >= excl && r.rank < incl;
    const u64 m = __ballot(mine);
    if (!m) {
      if (ln == 0) atomicOr(err, 1u);
    } else {
      const int src = __ffsll((long long)m) - 1;
      u32 c = excl, dg = 0;
      if (mine) {
        for (int q = 0; q < 4; ++q) {
          if (r.rank < c + v[q]) {
            dg = u32(4 * ln + q);
            break;
          }
          c += v[q];
        }
      }
      dg = u32(__shfl(int(dg), src, 64));
      c = u32(__shfl(int(c), src, 64));
      if (ln == 0) {
        r.prefix |= u64(dg) << (8 * pass);
        r.rank -= c;
        rs[j] = r;
      }
    }
  }
  for (int q = 0; q < 4; ++q) hs[4 * ln + q] = 0u;  // ready for the next round
}

__global__ void k_top_radix_init(const u32* __restrict__ sel, TopSizes sizes, int level, TopRadix* __restrict__ rs) {
  const int j = threadIdx.x;
  if (j >= (1 << level)) return;
  TopRadix r{};
  r.prefix = 0;
  r.active = sizes.n[j] > 0 ? 1u : 0u;
  r.rank = r.active ? u32(sizes.n[j] / 2) - sel[4 * j + 1] : 0u;
  rs[j] = r;
}

// the pivot's row (composite keys are unique: exactly one rank holds it) as i64 words for a
// MIN all-reduce (absent: INT64_MAX, prefilled by the caller)
__global__ __launch_bounds__(kBlock) void k_top_radix_row(TopPoints p, const u32* __restrict__ node, int level,
                                                          int axis, const TopRadix* __restrict__ rs,
                                                          i64* __restrict__ rowbuf) {
  const int nodes = 1 << level;
  const u32 first = u32(nodes - 1);
  const i64 stride = i64(gridDim.x) * kBlock;
  for (i64 i = i64(blockIdx.x) * kBlock + threadIdx.x; i < p.n; i += stride) {
    const u32 hn = node[i];
    if (hn - first >= u32(nodes)) continue;
    const u32 j = hn - first;
    const u32 id = point_id(p, i);
    if (composite_key(p.pts[i * p.dim + axis], id) != rs[j].prefix) continue;
    i64* o = rowbuf + size_t(j) * (p.dim + 1);
    for (int c = 0; c < p.dim; ++c) o[c] = i64(__float_as_uint(p.pts[i * p.dim + c]));
    o[p.dim] = i64(id);
  }
}

// pivots, top rows and children cells from the all-reduced rows
__global__ void k_top_radix_pivot(const i64* __restrict__ rowbuf, const TopRadix* __restrict__ rs, int level,
                                  int axis, int dim, u64* __restrict__ pivots, float* __restrict__ top_rows,
                                  float* __restrict__ cells, u32* __restrict__ err) {
  const int j = blockIdx.x;
  const u32 h = u32((1 << level) - 1 + j);
  float* cl = cells + size_t(2 * h + 1) * dim * 2;
  float* cr = cells + size_t(2 * h + 2) * dim * 2;
  const float* cp = cells + size_t(h) * dim * 2;
  for (int c = threadIdx.x; c < 2 * dim; c += blockDim.x) {
    cl[c] = cp[c];
    cr[c] = cp[c];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const TopRadix r = rs[j];
  float* tr = top_rows + size_t(h) * (dim + 1);
  if (!r.active) {
    pivots[h] = ~0ull;
    for (int c = 0; c <= dim; ++c) tr[c] = 0.0f;
    return;
  }
  const i64* o = rowbuf + size_t(j) * (dim + 1);
  if (o[dim] == INT64_MAX) {
    atomicOr(err, 1u);
    pivots[h] = ~0ull;
    return;
  }
  pivots[h] = r.prefix;
  for (int c = 0; c <= dim; ++c) tr[c] = __uint_as_float(u32(o[c]));
  const float split = __uint_as_float(u32(o[axis]));
  cl[2 * axis + 1] = split;
  cr[2 * axis] = split;
}

// rows left at their level-l node (its median bucket): below / above the pivot, or the pivot
__global__ __launch_bounds__(kBlock) void k_top_radix_fixup(TopPoints p, u32* __restrict__ node, int level, int axis,
                                                            int next_axis, const u64* __restrict__ pivots,
                                                            const float* __restrict__ cells, int next_bins,
                                                            u32* __restrict__ hist_next) {
  const int nodes = 1 << level;
  const u32 first = u32(nodes - 1);
  const i64 stride = i64(gridDim.x) * kBlock;
  for (i64 i = i64(blockIdx.x) * kBlock + threadIdx.x; i < p.n; i += stride) {
    const u32 h = node[i];
    if (h - first >= u32(nodes)) continue;
    const u64 ck = composite_key(p.pts[i * p.dim + axis], point_id(p, i));
    const u64 pv = pivots[h];
    const u32 child = ck < pv ? 2 * h + 1 : (ck > pv ? 2 * h + 2 : kTopDone);
    node[i] = child;
    if (hist_next != nullptr && child != kTopDone) {
      const float* c = cells + (size_t(h) * p.dim + next_axis) * 2;
      const BucketParams np = make_params(c[0], c[1], next_bins);
      atomicAdd(&hist_next[(child - 2 * first - 1) * next_bins + bucket_of(p.pts[i * p.dim + next_axis], np, next_bins)],
                1u);
    }
  }
}
}  // namespace

void top_radix_init(const u32* sel, const TopSizes& sizes, int level, TopRadix* rs, hipStream_t stream) {
  k_top_radix_init<<<1, kTopMaxNodes, 0, stream>>>(sel, sizes, level, rs);
  PKD_LAUNCH_CHECK();
}

void top_radix_hist(const TopPoints& p, const u32* node, int level, int axis, const TopRadix* rs, int pass,
                    u32* hist, hipStream_t stream) {
  if (p.n <= 0) return;
  k_top_radix_hist<<<stream_grid(p.n), kBlock, 0, stream>>>(p, node, level, axis, rs, pass, hist);
  PKD_LAUNCH_CHECK();
}

void top_radix_sel(u32* hist, int level, int pass, TopRadix* rs, u32* err, hipStream_t stream) {
  k_top_radix_sel<<<1 << level, 64, 0, stream>>>(hist, level, pass, rs, err);
  PKD_LAUNCH_CHECK();
}

void top_radix_row(const TopPoints& p, const u32* node, int level, int axis, const TopRadix* rs, i64* rowbuf,
                   hipStream_t stream) {
  if (p.n <= 0) return;
  k_top_radix_row<<<stream_grid(p.n), kBlock, 0, stream>>>(p, node, level, axis, rs, rowbuf);
  PKD_LAUNCH_CHECK();
}

void top_radix_pivot(const i64* rowbuf, const TopRadix* rs, int level, int axis, int dim, u64* pivots, float* top_rows,
                     float* cells, u32* err, hipStream_t stream) {
  k_top_radix_pivot<<<1 << level, 64, 0, stream>>>(rowbuf, rs, level, axis, dim, pivots, top_rows, cells, err);
  PKD_LAUNCH_CHECK();
}

void top_radix_fixup(const TopPoints& p, u32* node, int level, int axis, int next_axis, const u64* pivots,
                     const float* cells, int next_bins, u32* hist_next, hipStream_t stream) {
  if (p.n <= 0) return;
  k_top_radix_fixup<<<stream_grid(p.n), kBlock, 0, stream>>>(p, node, level, axis, next_axis, pivots, cells,
                                                              next_bins, hist_next);
  PKD_LAUNCH_CHECK();
}

size_t top_pack_scratch_bytes(i64 n, int T) { return size_t(2) * pack_blocks(n) * size_t(T) * 4; }

void top_pack(const TopPoints& p, const u32* node, int levels, float* out, int row_stride, i64 col_stride,
              u32* bitmaps, i64 bitmap_words, i64* counts, const u32* err, void* scratch, hipStream_t stream) {
  top_pack_count(p, node, levels, counts, err, scratch, stream);
  top_pack_scatter(p, node, levels, out, row_stride, col_stride, bitmaps, bitmap_words, scratch, stream);
}

void top_pack_count(const TopPoints& p, const u32* node, int levels, i64* counts, const u32* err, void* scratch,
                    hipStream_t stream) {
  if (levels < 0 || levels > 6) throw std::invalid_argument("top_pack: at most 6 top levels (64 leaves)");
  const int T = 1 << levels;
  const int blocks = pack_blocks(p.n);
  const i64 per_block = ((std::max<i64>(p.n, 1) + blocks - 1) / blocks + 255) / 256 * 256;
  u32* bcount = static_cast<u32*>(scratch);
  u32* offsets = bcount + size_t(blocks) * T;
  k_pack_count<<<blocks, kBlock, 0, stream>>>(node, p.n, levels, T, per_block, bcount);
  PKD_LAUNCH_CHECK();
  static_assert(2 * kScanThreads >= 2048, "k_pack_scan covers at most 2 * kScanThreads blocks");
  k_pack_scan<<<T, kScanThreads, 0, stream>>>(bcount, blocks, T, offsets, counts, err);
  PKD_LAUNCH_CHECK();
}

void top_pack_scatter(const TopPoints& p, const u32* node, int levels, float* out, int row_stride, i64 col_stride,
                      u32* bitmaps, i64 bitmap_words, const void* scratch, hipStream_t stream) {
  if (levels < 0 || levels > 6) throw std::invalid_argument("top_pack: at most 6 top levels (64 leaves)");
  const int T = 1 << levels;
  if (col_stride > 0 && (col_stride < p.n || p.ids != nullptr))
    throw std::invalid_argument("top_pack: planar output needs col_stride >= n and implicit ids");
  if (col_stride == 0 && row_stride != p.dim && row_stride != p.dim + 1)
    throw std::invalid_argument("top_pack: row stride dim or dim+1");
  if (bitmaps && bitmap_words * 32 < p.n) throw std::invalid_argument("top_pack: bitmap stride too small");
  const int blocks = pack_blocks(p.n);
  // rows per block a multiple of 256: every wave's 64 rows of a chunk are two whole bitmap words
  const i64 per_block = ((std::max<i64>(p.n, 1) + blocks - 1) / blocks + 255) / 256 * 256;
  const u32* offsets = static_cast<const u32*>(scratch) + size_t(blocks) * T;
  if (bitmaps && p.n == 0) {
    // no chunk runs, so no ballot writes the (one-word) bitmaps: zero them (the receiver pops
    // bitmap_words words per leaf even from an empty sender)
    fill_u32(bitmaps, i64(T) * bitmap_words, 0u, stream);
  }
  k_pack_scatter<<<blocks, kBlock, 0, stream>>>(p, node, levels, T, per_block, offsets, out, row_stride, col_stride,
                                                bitmaps, bitmap_words);
  PKD_LAUNCH_CHECK();
}

namespace {
__global__ void k_place_rows(const float* __restrict__ top_rows, int dim, TopPlacement pl, float* __restrict__ out_pts,
                             u32* __restrict__ out_ids) {
  const int i = blockIdx.x;
  const float* r = top_rows + size_t(pl.heap[i]) * (dim + 1);
  const i64 s = pl.slot[i];
  for (int c = threadIdx.x; c < dim; c += blockDim.x) out_pts[s * dim + c] = r[c];
  if (threadIdx.x == 0) out_ids[s] = __float_as_uint(r[dim]);
}
}  // namespace

namespace {
__global__ void k_or_word(const u32* __restrict__ src, u32* __restrict__ dst) {
  if (threadIdx.x == 0) *dst |= *src;
}
}  // namespace

void or_error_word(const u32* src, u32* dst, hipStream_t stream) {
  k_or_word<<<1, 64, 0, stream>>>(src, dst);
  PKD_LAUNCH_CHECK();
}

void top_place_rows(const float* top_rows, int dim, const TopPlacement& pl, float* out_pts, u32* out_ids,
                    hipStream_t stream) {
  if (pl.count <= 0) return;
  if (pl.count > 64) throw std::invalid_argument("top_place_rows: at most 64 rows");
  k_place_rows<<<pl.count, 64, 0, stream>>>(top_rows, dim, pl, out_pts, out_ids);
  PKD_LAUNCH_CHECK();
}

namespace {
// axis of heap node h (top tree rooted at depth depth0)
__device__ __forceinline__ int rq_axis(i64 h, int depth0, int dim) {
  int l = 0;
  while (((h + 1) >> (l + 1)) > 0) ++l;
  return (depth0 + l) % dim;
}

__global__ __launch_bounds__(kBlock) void k_rq_home(const float* __restrict__ q, i64 Q, int dim,
                                                    const float* __restrict__ top_rows, RqBlocks bl,
                                                    u32* __restrict__ lists, u32* __restrict__ counts,
                                                    int* __restrict__ home) {
  const i64 i = i64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= Q) return;
  i64 h = 0;
  for (int l = 0; l < bl.LL; ++l) {
    const int ax = (bl.depth0 + l) % dim;
    const float piv = top_rows[h * (dim + 1) + ax];
    h = 2 * h + 1 + (q[i * dim + ax] >= piv ? 1 : 0);
  }
  const int leaf = int(h - (bl.T - 1));
  const int b = bl.leaf_block[leaf];
  home[i] = b;
  if (b >= 0) {
    const u32 k = atomicAdd(&counts[b], 1u);
    lists[i64(b) * Q + k] = u32(i);
  }
}

__global__ __launch_bounds__(kBlock) void k_rq_reach(const float* __restrict__ q, i64 Q, int dim,
                                                     const float* __restrict__ top_rows, RqBlocks bl,
                                                     const u64* __restrict__ best, const int* __restrict__ home,
                                                     u32* __restrict__ lists, u32* __restrict__ counts) {
  const i64 i = i64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= Q) return;
  const double d2 = double(packed_dist(best[i]));
  const int hb = home[i];
  for (int b = 0; b < bl.nb; ++b) {
    if (b == hb) continue;
    // box distance: the pivots above the block root bound it (closed box)
    double g2 = 0.0;
    i64 child = bl.heap[b];
    // per axis the tightest bounds; dims <= 64 walked pivot by pivot (<= LL of them)
    for (int c = 0; c < dim; ++c) {
      double lo = -1e300, hi = 1e300;
      i64 ch = child;
      while (ch > 0) {
        const i64 h = (ch - 1) / 2;
        if (rq_axis(h, bl.depth0, dim) == c) {
          const double v = double(top_rows[h * (dim + 1) + c]);
          if (ch == 2 * h + 1) hi = v < hi ? v : hi;
          else lo = v > lo ? v : lo;
        }
        ch = h;
      }
      const double x = double(q[i * dim + c]);
      const double gap = (x < lo ? lo - x : 0.0) + (x > hi ? x - hi : 0.0);
      g2 += gap * gap;
    }
    if (g2 <= d2 * (1.0 + 1e-5)) {
      const u32 k = atomicAdd(&counts[b], 1u);
      lists[i64(b) * Q + k] = u32(i);
    }
  }
}
}  // namespace

void rq_home(const float* queries, i64 Q, int dim, const float* top_rows, const RqBlocks& bl, u32* lists,
             u32* counts, int* home, hipStream_t stream) {
  if (Q <= 0) return;
  if (bl.nb > kRqMaxBlocks || bl.T > 64) throw std::invalid_argument("rq_home: at most 64 blocks / leaves");
  k_rq_home<<<int((Q + kBlock - 1) / kBlock), kBlock, 0, stream>>>(queries, Q, dim, top_rows, bl, lists, counts, home);
  PKD_LAUNCH_CHECK();
}

void rq_reach(const float* queries, i64 Q, int dim, const float* top_rows, const RqBlocks& bl, const u64* best,
              const int* home, u32* lists, u32* counts, hipStream_t stream) {
  if (Q <= 0 || bl.nb == 0) return;
  k_rq_reach<<<int((Q + kBlock - 1) / kBlock), kBlock, 0, stream>>>(queries, Q, dim, top_rows, bl, best, home, lists,
                                                                    counts);
  PKD_LAUNCH_CHECK();
}

size_t ids_from_bitmaps_scratch_bytes(i64 max_words, int P) {
  return size_t(P) * size_t(std::max<i64>(1, (max_words + kBmWords - 1) / kBmWords)) * 4;
}

void ids_from_bitmaps(const u32* bitmaps, int P, const BmSources& src, u32* ids, void* scratch, u32* err,
                      hipStream_t stream) {
  if (P > kBmMaxSources) throw std::invalid_argument("ids_from_bitmaps: too many sources");
  i64 max_words = 0;
  for (int s = 0; s < P; ++s) max_words = std::max(max_words, src.words[s]);
  const int nblk = int(std::max<i64>(1, (max_words + kBmWords - 1) / kBmWords));
  u32* bsum = static_cast<u32*>(scratch);
  k_bm_block_sums<<<dim3(nblk, P), kBlock, 0, stream>>>(bitmaps, src, nblk, bsum);
  PKD_LAUNCH_CHECK();
  k_bm_ids<<<dim3(nblk, P), kBlock, 0, stream>>>(bitmaps, nblk, bsum, src, ids, err);
  PKD_LAUNCH_CHECK();
}

}  // namespace pkdtree
