// Definitions of the LDS subtree kernel (build_subtree.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "pkdtree/common.hpp"

namespace pkdtree {
namespace subtree_detail {

struct SubArgs {
  const float* cols;
  i64 ncol;
  int dim;
  const i64* seg_lo;
  const i64* seg_n;
  const float* cells;  // heap-indexed [h][dim][2] cell of every segment root
  i64 heap0;
  int depth_base;
  float* out_pts;
  u32* out_ids;
  u32* err;
  unsigned long long* stamps;  // diagnostic build only (PKD_SUBTREE_STAMPS): [blocks][kStampSlots] s_memtime
  int narrow_k;                // narrow (ldim > 0): id column; the input row index follows it
  const float* in_rows;
  i64 in_rs;
  int ldim;                    // narrow: LDS key slots (slot t = key of subtree level t), 0 otherwise
  int small_seg;               // first-use levels whose sub-segments hold <= this many points rank by comparison
};

// Orders this wave's LDS writes before its later LDS reads (different lanes): waits for the
// wave's outstanding LDS operations and fences the compiler.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kStampSlots = 32;
constexpr int kStampBlocks = 4096;
// slot 0 start, 1 rows loaded, 2 + t after level t (rank kernel), 30 before the store, 31 end
// The pointer test is a kernel argument (scalar branch): with stamps off no wave touches its
// exec mask here.
__device__ __forceinline__ void stamp(const SubArgs& a, int i) {
  // wave 0 stores (every lane the same value to the same word): a wave-uniform condition
  if (a.stamps != nullptr && blockIdx.x < kStampBlocks && __builtin_amdgcn_readfirstlane(threadIdx.x) < 64)
    a.stamps[blockIdx.x * kStampSlots + i] = __builtin_amdgcn_s_memtime();
}

__device__ __forceinline__ void report(u32* err, u32 code, u32 t, u32 v) {
  atomicOr(err, 4u);
  if (atomicCAS(err + 1, 0u, code) == 0u) {
    err[2] = t;
    err[3] = v;
  }
}

}  // namespace subtree_detail

}  // namespace pkdtree
