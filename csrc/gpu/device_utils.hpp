// Wave64 / workgroup helpers for gfx950 (CDNA4). Wave width is 64 everywhere: ballots are
// 64-bit, lane ranks come from v_mbcnt, scans use 64-lane shuffles.
#pragma once
#include <hip/hip_runtime.h>

#include "pkdtree/common.hpp"

namespace pkdtree {
namespace dev {

constexpr int kWave = 64;

__device__ __forceinline__ int lane() { return int(__lane_id()); }

// Number of set bits of `mask` in lanes below this one.
__device__ __forceinline__ u32 mbcnt(u64 mask) {
  return __builtin_amdgcn_mbcnt_hi(u32(mask >> 32), __builtin_amdgcn_mbcnt_lo(u32(mask), 0u));
}

// Inclusive prefix sum over the 64 lanes with DPP moves only (no LDS round trips): shifts of
// 1, 2, 4, 8 inside each row of 16 lanes, then row_bcast:15 / row_bcast:31 carry the row
// totals across rows (GFX9 DPP controls, available on CDNA4).
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
  v += u32(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, true));  // row_shr:1
  v += u32(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, true));  // row_shr:2
  v += u32(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, true));  // row_shr:4
  v += u32(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, true));  // row_shr:8
  v += u32(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));  // row_bcast:15 -> rows 1, 3
  v += u32(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));  // row_bcast:31 -> rows 2, 3
  return v;
}

// Inclusive scan inside aligned groups of G lanes (G power of two <= 64).
template <int G>
__device__ __forceinline__ u32 group_incl_scan(u32 v) {
  const int l = lane() & (G - 1);
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const u32 t = __shfl_up(v, o, G);
    if (l >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ u32 wave_min_u32(u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (u32)__shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ u32 wave_max_u32(u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (u32)__shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ u64 shfl_u64(u64 v, int src) {
  const u32 lo = __shfl(u32(v), src, kWave);
  const u32 hi = __shfl(u32(v >> 32), src, kWave);
  return (u64(hi) << 32) | lo;
}
__device__ __forceinline__ u64 wave_min_u64(u64 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const u64 t = shfl_u64(v, lane() ^ o);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const u64 t = shfl_u64(v, lane() ^ o);
    v = t > v ? t : v;
  }
  return v;
}

// Multi-split rank of a wave's lanes by zone q (< 16; callers use 15 for "no zone"): this lane's
// rank among the lanes of its zone, lower lanes first, from 4 bit-sliced ballots instead of one
// ballot per zone; lane z < NZ stores zone z's count to cnt[z * stride] (one LDS store per wave
// instead of one single-lane store per zone). All 64 lanes must call it.
template <int NZ>
__device__ __forceinline__ u32 wave_zone_rank(u32 q, u32* cnt, int stride) {
  static_assert(NZ <= 16, "4-bit zones");
  const u64 b0 = __ballot(q & 1u), b1 = __ballot(q & 2u), b2 = __ballot(q & 4u), b3 = __ballot(q & 8u);
  auto same = [&](u32 z) {
    return ((z & 1u) ? b0 : ~b0) & ((z & 2u) ? b1 : ~b1) & ((z & 4u) ? b2 : ~b2) & ((z & 8u) ? b3 : ~b3);
  };
  const u32 ln = u32(lane());
  if (ln < u32(NZ)) cnt[ln * u32(stride)] = u32(__popcll(same(ln)));
  return mbcnt(same(q));
}

// Bucketing used by every histogram/partition pair. Monotone non-decreasing in x, so the
// bucket order never contradicts the key order; identical inputs give identical buckets
// in every kernel (-ffp-contract=off, no FMA possible in this expression).
struct BucketParams {
  float lo;
  float scale;
};

__device__ __forceinline__ u32 bucket_of(float x, BucketParams p, int nb) {
  float t = (x - p.lo) * p.scale;
  t = fminf(fmaxf(t, 0.0f), float(nb - 1));
  return u32(t);
}

// Error-word gate of a build's kernels. Once a build has set its sticky error word (a sampled
// band missed its median, a staging region overflowed, a consistency check failed) its tree is
// invalid and is redone by the caller; every kernel after the first point where that can happen
// returns here instead of running on a layout whose segments no longer hold what the geometry
// says. (A missed top leaves the tail slots of under-filled level-4 segments holding whatever the
// workspace held before: on a REUSED builder those are rows of its previous build, i.e. duplicate
// (key, id) composites, which the exact-rank kernels below turn into colliding ranks and slot
// indices past their segment -- the intermittent hipErrorIllegalAddress of round 5.)
// Workgroup-uniform: thread 0 reads the word once and the block agrees on it through LDS, so a
// word set concurrently (another workgroup of the same kernel, another stream of a split build)
// can never split a workgroup at a later barrier. Every thread must call it (it holds a barrier).
// Split form for the long kernels with an early barrier of their own (k_tail3, the subtree
// kernel): thread 0 issues the load at the very start, into an LDS word, and the block tests it
// after that barrier, so the load's latency hides behind the kernel's own first loads instead of
// stalling every workgroup's start (the one-barrier form cost the 100 M build's 65 536 subtree
// workgroups ~24 us).
__device__ __forceinline__ void build_failed_issue(const u32* err, u32* flag) {
  if (threadIdx.x == 0) *flag = *err;
}
__device__ __forceinline__ bool build_failed(const u32* err) {
  __shared__ u32 flag;
  if (threadIdx.x == 0) flag = *err;  // plain load: kernel boundaries order the earlier kernels' writes
  __syncthreads();
  return flag != 0u;
}

PKD_HD BucketParams make_params(float lo, float hi, int nb) {
  BucketParams p;
  p.lo = lo;
  const float span = hi - lo;
  p.scale = (span > 0.0f) ? float(nb) / span : 0.0f;
  return p;
}

}  // namespace dev
}  // namespace pkdtree
