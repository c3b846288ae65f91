// Device ops of the global (distributed) decomposition; see dist_ops.hpp.
#include <algorithm>

#include "device_utils.hpp"
#include "pkdtree/dist_ops.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {

using dev::BucketParams;
using dev::bucket_of;
using dev::mbcnt;

namespace {

constexpr int kBlock = 256;
constexpr int kMaxTopBins = 8192;  // nodes * bins per level (LDS histogram)

__device__ __forceinline__ u64 row_key(const float* r, int dim, int axis) {
  return composite_key(r[axis], __float_as_uint(r[dim]));
}

// Route one point one level down below the pivot of its node (heap order).
__device__ __forceinline__ u32 route(u32 h, const float* r, int dim, int axis, const u64* pivots) {
  if (h == kTopDone) return h;
  const u64 k = row_key(r, dim, axis);
  const u64 pv = pivots[h];
  return k < pv ? 2 * h + 1 : (k > pv ? 2 * h + 2 : kTopDone);
}

__global__ __launch_bounds__(kBlock) void k_top_route_hist(const float* __restrict__ rows, i64 n, int dim,
                                                           u32* __restrict__ node, int level,
                                                           const u64* __restrict__ pivots, int prev_axis, int axis,
                                                           const float* __restrict__ params, int bins,
                                                           u32* __restrict__ hist) {
  extern __shared__ __align__(16) u32 sh[];
  const u32 first = (1u << level) - 1;
  const int nb_total = (1 << level) * bins;
  for (int b = threadIdx.x; b < nb_total; b += kBlock) sh[b] = 0;
  __syncthreads();
  const i64 stride = i64(gridDim.x) * kBlock;
  const int rs = dim + 1;
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += stride) {
    const float* r = rows + p * rs;
    u32 h = node[p];
    if (level > 0) {
      h = route(h, r, dim, prev_axis, pivots);
      node[p] = h;
    }
    if (h == kTopDone) continue;
    const u32 j = h - first;
    BucketParams pr;
    pr.lo = params[2 * j];
    pr.scale = params[2 * j + 1];
    atomicAdd(&sh[j * bins + bucket_of(r[axis], pr, bins)], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb_total; b += kBlock) {
    const u32 v = sh[b];
    if (v) atomicAdd(&hist[b], v);
  }
}

__global__ __launch_bounds__(kBlock) void k_top_collect(const float* __restrict__ rows, i64 n, int dim,
                                                        const u32* __restrict__ node, int level, int axis,
                                                        const float* __restrict__ params, int bins,
                                                        const u32* __restrict__ bstar, float* __restrict__ out,
                                                        i64 cap, unsigned long long* __restrict__ count) {
  const u32 first = (1u << level) - 1;
  const i64 stride = i64(gridDim.x) * kBlock;
  const int rs = dim + 1;
  for (i64 p = i64(blockIdx.x) * kBlock + threadIdx.x; p < n; p += stride) {
    const u32 h = node[p];
    if (h == kTopDone) continue;
    const float* r = rows + p * rs;
    const u32 j = h - first;
    BucketParams pr;
    pr.lo = params[2 * j];
    pr.scale = params[2 * j + 1];
    if (bucket_of(r[axis], pr, bins) != bstar[j]) continue;
    const unsigned long long slot = atomicAdd(count, 1ull);
    if (i64(slot) < cap) {
      float* o = out + i64(slot) * (rs + 1);
      for (int c = 0; c < rs; ++c) o[c] = r[c];
      o[rs] = __uint_as_float(h);  // node of the middle point rides along
    }
  }
}

// --- counting sort by destination (P <= 64) -------------------------------------------
__global__ __launch_bounds__(kBlock) void k_pack_count(const float* __restrict__ rows, i64 n, int dim,
                                                       u32* __restrict__ node, const u64* __restrict__ pivots,
                                                       int last_axis, int P, i64 per_block,
                                                       u32* __restrict__ bcount) {
  __shared__ u32 cnt[64];
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const i64 b0 = i64(blockIdx.x) * per_block, b1 = min(n, b0 + per_block);
  const u32 first = u32(P - 1);
  for (i64 p = b0 + threadIdx.x; p < b1; p += kBlock) {
    const u32 h = route(node[p], rows + p * (dim + 1), dim, last_axis, pivots);
    node[p] = h;
    if (h != kTopDone) atomicAdd(&cnt[h - first], 1u);
  }
  __syncthreads();
  if (threadIdx.x < P) bcount[i64(blockIdx.x) * P + threadIdx.x] = cnt[threadIdx.x];
}

// offsets[block][d] = sum_{d' < d} total[d'] + sum_{b' < block} bcount[b'][d]; counts[d] = total[d]
__global__ void k_pack_scan(const u32* __restrict__ bcount, int blocks, int P, u32* __restrict__ offsets,
                            u32* __restrict__ counts) {
  __shared__ u32 tot[64];
  const int d = threadIdx.x;
  if (d < P) {
    u32 s = 0;
    for (int b = 0; b < blocks; ++b) s += bcount[i64(b) * P + d];
    tot[d] = s;
    counts[d] = s;
  }
  __syncthreads();
  if (d < P) {
    u32 base = 0;
    for (int e = 0; e < d; ++e) base += tot[e];
    for (int b = 0; b < blocks; ++b) {
      offsets[i64(b) * P + d] = base;
      base += bcount[i64(b) * P + d];
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_pack_scatter(const float* __restrict__ rows, i64 n, int dim,
                                                         const u32* __restrict__ node, int P, i64 per_block,
                                                         const u32* __restrict__ offsets, float* __restrict__ out) {
  __shared__ u32 cur[64];
  __shared__ u32 wcnt[4][64];
  const u32 first = u32(P - 1);
  if (threadIdx.x < P) cur[threadIdx.x] = offsets[i64(blockIdx.x) * P + threadIdx.x];
  __syncthreads();
  const i64 b0 = i64(blockIdx.x) * per_block, b1 = min(n, b0 + per_block);
  const int w = threadIdx.x / 64, ln = dev::lane();
  const int rs = dim + 1;
  for (i64 c0 = b0; c0 < b1; c0 += kBlock) {
    const i64 p = c0 + threadIdx.x;
    const u32 h = p < b1 ? node[p] : kTopDone;
    const int d = h == kTopDone ? -1 : int(h - first);
    u32 my = 0;
    for (int e = 0; e < P; ++e) {  // stable rank among same-destination points of the chunk
      const u64 m = __ballot(d == e);
      if (ln == 0) wcnt[w][e] = __popcll(m);
      if (d == e) my = mbcnt(m);
    }
    __syncthreads();
    if (d >= 0) {
      u32 off = cur[d];
      for (int v = 0; v < w; ++v) off += wcnt[v][d];
      float* o = out + i64(off + my) * rs;
      const float* r = rows + p * rs;
      for (int c = 0; c < rs; ++c) o[c] = r[c];
    }
    __syncthreads();
    if (threadIdx.x < P) {
      u32 add = 0;
      for (int v = 0; v < kBlock / 64; ++v) add += wcnt[v][threadIdx.x];
      cur[threadIdx.x] += add;
    }
    __syncthreads();
  }
}

int pack_blocks(i64 n) { return int(std::max<i64>(1, std::min<i64>(2048, (n + 8191) / 8192))); }

}  // namespace

void top_route_hist(const float* rows, i64 n, int dim, u32* node, int level, const u64* pivots, int prev_axis,
                    int axis, const float* params, int bins, u32* hist, hipStream_t stream) {
  if (n <= 0) return;
  const int nb_total = (1 << level) * bins;
  if (nb_total > kMaxTopBins) throw std::invalid_argument("top_route_hist: nodes * bins exceeds 8192");
  const int grid = int(std::min<i64>(2048, (n + kBlock - 1) / kBlock));
  k_top_route_hist<<<grid, kBlock, size_t(nb_total) * 4, stream>>>(rows, n, dim, node, level, pivots, prev_axis,
                                                                    axis, params, bins, hist);
  PKD_LAUNCH_CHECK();
}

void top_collect_middle(const float* rows, i64 n, int dim, const u32* node, int level, int axis, const float* params,
                        int bins, const u32* bstar, float* out_rows, i64 cap, unsigned long long* out_count,
                        hipStream_t stream) {
  PKD_HIP_CHECK(hipMemsetAsync(out_count, 0, 8, stream));
  if (n <= 0) return;
  const int grid = int(std::min<i64>(2048, (n + kBlock - 1) / kBlock));
  k_top_collect<<<grid, kBlock, 0, stream>>>(rows, n, dim, node, level, axis, params, bins, bstar, out_rows, cap,
                                              out_count);
  PKD_LAUNCH_CHECK();
}

size_t top_pack_scratch_bytes(i64 n, int P) { return size_t(2) * pack_blocks(n) * size_t(P) * 4; }

void top_pack(const float* rows, i64 n, int dim, u32* node, int levels, const u64* pivots, int last_axis, int P,
              float* out_rows, u32* counts, void* scratch, hipStream_t stream) {
  if (P > 64 || P != (1 << levels)) throw std::invalid_argument("top_pack: P must be 2^levels <= 64");
  const int blocks = pack_blocks(n);
  const i64 per_block = (std::max<i64>(n, 1) + blocks - 1) / blocks;
  u32* bcount = static_cast<u32*>(scratch);
  u32* offsets = bcount + size_t(blocks) * P;
  k_pack_count<<<blocks, kBlock, 0, stream>>>(rows, n, dim, node, pivots, last_axis, P, per_block, bcount);
  PKD_LAUNCH_CHECK();
  k_pack_scan<<<1, 64, 0, stream>>>(bcount, blocks, P, offsets, counts);
  PKD_LAUNCH_CHECK();
  k_pack_scatter<<<blocks, kBlock, 0, stream>>>(rows, n, dim, node, P, per_block, offsets, out_rows);
  PKD_LAUNCH_CHECK();
}

}  // namespace pkdtree
