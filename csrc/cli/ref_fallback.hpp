// GPU reference mode with the CPU std::sort builder as the fallback where ties decide.
//
// The reference sorts with std::sort, which is unstable: where equal keys meet at a segment's
// deciding ranks, its tree is whatever its library's introsort produced. ReferenceBuilder
// counts those segments (read_ties); when there are any, the tree is rebuilt on the host by
// build_reference_cpu -- the reference's own recursion and std::sort call on the same input
// order (kdtree_sequential.cpp:30-66) -- and uploaded, so the printed output never silently
// diverges from the reference binary's.
#pragma once
#include <hip/hip_runtime.h>

#include <iostream>
#include <vector>

#include "pkdtree/cpu_tree.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {
namespace cli {

// Builds the reference tree of the device points d_pts [n][dim] (ids id_base + row) into
// d_tree / d_ids on the GPU; returns the tie count of the GPU build (non-zero: the CPU builder
// made the tree). `who` prefixes the stderr note. Synchronises `s`.
inline u32 build_reference_checked(const ReferenceBuilder& rb, const float* d_pts, i64 n, int dim, u32 id_base,
                                   float* d_tree, u32* d_ids, void* ws, hipStream_t s, const char* who) {
  if (n <= 0) return 0;
  rb.build(d_pts, nullptr, id_base, d_tree, d_ids, ws, s);
  const u32 ties = rb.read_ties(ws, s);
  if (ties == 0) return 0;
  std::cerr << who << ": reference mode: " << ties
            << " segment(s) decided by equal keys (the reference's std::sort is unstable there); "
               "building this tree with the CPU std::sort builder"
            << std::endl;
  std::vector<float> h(size_t(n) * size_t(dim)), tp(h.size());
  std::vector<u32> perm(static_cast<size_t>(n)), ids(perm.size()), ti(perm.size());
  PKD_HIP_CHECK(hipMemcpy(h.data(), d_pts, h.size() * 4, hipMemcpyDeviceToHost));
  for (i64 r = 0; r < n; ++r) ids[size_t(r)] = id_base + u32(r);
  build_reference_cpu(h.data(), n, dim, perm.data(), default_cpu_threads());  // threaded: same tree
  gather_rows(h.data(), ids.data(), perm.data(), n, dim, tp.data(), ti.data());
  PKD_HIP_CHECK(hipMemcpy(d_tree, tp.data(), tp.size() * 4, hipMemcpyHostToDevice));
  PKD_HIP_CHECK(hipMemcpy(d_ids, ti.data(), ti.size() * 4, hipMemcpyHostToDevice));
  return ties;
}

}  // namespace cli
}  // namespace pkdtree
