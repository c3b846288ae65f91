// pkdtree — MI355X-native parallel kd-tree.
// Shared host/device definitions: index types, the total order used by the exact
// builder, and the bit-exact squared-distance kernel.
//
// Reference parity notes (paths relative to the reference repo):
//  * Point::distance_squared (kdtree_sequential.cpp:14-25) sums (a_i-b_i)^2 over i in
//    increasing order in fp32 with separately rounded mul and add (built with -mavx but
//    no -mfma, so no contraction). sq_dist() below keeps that exact order; every TU of
//    this project is compiled with -ffp-contract=off.
//  * Point::compare (Node.cpp:46-48) orders by one coordinate only, which leaves ties to
//    the (unstable) std::sort. The exact builder here instead uses the total order
//    (orderable(key), id) so the tree is unique for any input and identical for any
//    number of GPUs.
#pragma once

#include <cstdint>
#include <cstddef>
#include <cstring>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PKD_HD __host__ __device__ __forceinline__
#else
#define PKD_HD inline
#endif

namespace pkdtree {

using u16 = std::uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

// Map an fp32 bit pattern to an unsigned key with the same order as the float
// (-inf < ... < -0 < +0 < ... < +inf). NaNs are unsupported input.
PKD_HD u32 orderable_bits(u32 b) { return (b & 0x80000000u) ? ~b : (b | 0x80000000u); }
PKD_HD u32 unorderable_bits(u32 k) { return (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k; }

PKD_HD u32 float_bits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __float_as_uint(f);
#else
  u32 b; std::memcpy(&b, &f, 4); return b;
#endif
}
PKD_HD float bits_float(u32 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __uint_as_float(b);
#else
  float f; std::memcpy(&f, &b, 4); return f;
#endif
}

PKD_HD u32 orderable(float f) { return orderable_bits(float_bits(f)); }
PKD_HD float from_orderable(u32 k) { return bits_float(unorderable_bits(k)); }

// Composite key that realises the exact builder's total order.
PKD_HD u64 composite_key(float key, u32 id) { return (u64(orderable(key)) << 32) | u64(id); }

// Squared Euclidean distance with the reference's summation order (see header).
template <typename T>
PKD_HD float sq_dist(const T* a, const float* b, int dim) {
  float acc = 0.0f;
  for (int i = 0; i < dim; ++i) {
    float t = float(a[i]) - b[i];
    float sq = t * t;
    acc = acc + sq;
  }
  return acc;
}

// Strided variant (coordinate i of point a at a[i*stride]), same order.
PKD_HD float sq_dist_strided(const float* a, size_t stride, const float* b, int dim) {
  float acc = 0.0f;
  for (int i = 0; i < dim; ++i) {
    float t = a[size_t(i) * stride] - b[i];
    float sq = t * t;
    acc = acc + sq;
  }
  return acc;
}

// Pack (non-negative float distance, index) so that unsigned min == lexicographic
// (dist, index) min. Used by the NN kernels and by the cross-rank MIN reductions.
PKD_HD u64 pack_dist_idx(float d2, u32 idx) { return (u64(float_bits(d2)) << 32) | u64(idx); }
PKD_HD float packed_dist(u64 p) { return bits_float(u32(p >> 32)); }
PKD_HD u32 packed_idx(u64 p) { return u32(p & 0xffffffffu); }

constexpr u64 kPackedInf = (u64(0x7f800000u) << 32) | 0xffffffffull;  // (+inf, max idx)

// Implicit in-order tree geometry: the node of segment [lo, lo+n) sits at
// lo + n/2; the left child is [lo, lo+n/2), the right child [lo+n/2+1, lo+n).
PKD_HD i64 median_pos(i64 lo, i64 n) { return lo + n / 2; }
PKD_HD i64 left_n(i64 n) { return n / 2; }
PKD_HD i64 right_n(i64 n) { return n - n / 2 - 1; }

// ceil(log2(n+1)): the left child (n/2) is never smaller than the right one.
inline int tree_height(i64 n) {
  int h = 0;
  for (; n > 0; n /= 2) ++h;
  return h;
}

}  // namespace pkdtree
